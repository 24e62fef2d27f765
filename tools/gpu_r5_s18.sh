#!/bin/bash
# Round 5: the fuzz parity suite alone after the submit / complete split (seed 5 failed once in s17).
set -o pipefail
O=gpurun_out/s18
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_fuzz.py > $O/fuzz.log 2>&1
rc=$?
grep -E "FAILED|AssertionError|passed|failed" $O/fuzz.log | head -20
exit $rc
