#!/bin/bash
# Round 5: s17's test list again (rxloop + host + staged + fuzz) with the fuzz test's fuller failure report.
set -o pipefail
O=gpurun_out/s19
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_rxloop.py \
    tests/test_gpu_host.py tests/test_gpu_staged.py tests/test_gpu_fuzz.py > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|Error:|passed|failed" $O/tests.log | cut -c1-600 | head -20
exit $rc
