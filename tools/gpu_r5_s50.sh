#!/bin/bash
# Round 5: the s48 record mismatch of test_lowlat_timeout_exactly_once -- 40 runs of the test in one process (240
# batches at a 1-us timeout), each failure with the records that differ and the outcomes so far.
set -o pipefail
O=gpurun_out/s50
mkdir -p $O
timeout -k 10 400 python -u - > $O/timeout.log 2>&1 <<'PY'
import sys, collections
sys.path.insert(0, ".")
from tests import test_gpu_staged as T
fails = 0
for k in range(40):
    try:
        T.test_lowlat_timeout_exactly_once()
    except AssertionError as e:
        fails += 1
        print("run", k, "FAIL", str(e)[:2500], flush=True)
    if k % 10 == 9:
        print("runs", k + 1, "fails", fails, flush=True)
PY
rc=$?; grep -c "timeout outcomes" $O/timeout.log; grep "FAIL\|fails" $O/timeout.log | cut -c1-1200 | tail -12; exit $rc
