#!/bin/bash
# Round 5: the pipe tests first again (the order that saw misdirected writes in s17-s25), twice, with the GPU-view
# failure reports; stops at the first GPU fault.
set -o pipefail
O=gpurun_out/s33
mkdir -p $O
S="tests/test_gpu_zpipe.py tests/test_gpu_host.py tests/test_gpu_staged.py tests/test_gpu_fuzz.py"
for k in 1 2; do
  timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread $S > $O/run$k.log 2>&1; echo "run$k rc=$? $(tail -1 $O/run$k.log)"
  grep -q "illegal memory access\|Memory access fault" $O/run$k.log && exit 3
done
exit 0
