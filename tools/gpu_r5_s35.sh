#!/bin/bash
# Round 5: the pipe GPU tests incl. the mixed LOWLAT / ZEROCOPY pipe.
set -o pipefail
O=gpurun_out/s35
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_zpipe.py > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|Error|passed|failed" $O/tests.log | cut -c1-400 | tail -8
exit $rc
