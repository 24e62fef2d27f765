#!/bin/bash
# Round 5: A/B on one box -- the previous commit (_ab_old, no pipelined loop) and this tree, same test files, in turn.
# Stops at the first GPU fault.
set -o pipefail
O=$PWD/gpurun_out/s27
mkdir -p $O
T="timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread"
S="tests/test_gpu_rxloop.py tests/test_gpu_host.py tests/test_gpu_staged.py tests/test_gpu_fuzz.py"
for k in 1 2; do
  (cd _ab_old && $T $S > $O/old$k.log 2>&1); echo "old$k rc=$? $(tail -1 $O/old$k.log)"
  grep -q "illegal memory access\|Memory access fault" $O/old$k.log && exit 3
  $T $S > $O/new$k.log 2>&1; echo "new$k rc=$? $(tail -1 $O/new$k.log)"
  grep -q "illegal memory access\|Memory access fault" $O/new$k.log && exit 3
done
exit 0
