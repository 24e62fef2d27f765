#!/bin/bash
# Round 5: host GPU tests after the staging revert (the small-frame LOWLAT tests on the UMEM in place).
set -o pipefail
O=gpurun_out/s38
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_host.py > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|Error|passed|failed" $O/tests.log | cut -c1-600 | tail -6
exit $rc
