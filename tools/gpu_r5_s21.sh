#!/bin/bash
# Round 5: isolate what makes LOWLAT results go wrong later in the process (s19: timeout test + fuzz fail).
set -o pipefail
O=gpurun_out/s21
mkdir -p $O
T="timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread"
$T -k "not pipe" tests/test_gpu_rxloop.py tests/test_gpu_host.py tests/test_gpu_staged.py tests/test_gpu_fuzz.py > $O/a_nopipe.log 2>&1; echo "nopipe rc=$?"
$T tests/test_gpu_rxloop.py tests/test_gpu_staged.py tests/test_gpu_fuzz.py > $O/b_pipe_staged_fuzz.log 2>&1; echo "pipe+staged+fuzz rc=$?"
$T -k "pipe" tests/test_gpu_rxloop.py tests/test_gpu_fuzz.py > $O/c_pipe_fuzz.log 2>&1; echo "pipe+fuzz rc=$?"
for f in $O/*.log; do echo "== $f"; grep -E "^E .*(differ|Error:)|passed|failed" $f | cut -c1-400 | head -6; done
