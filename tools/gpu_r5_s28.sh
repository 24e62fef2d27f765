#!/bin/bash
# Round 5: A/B/C on one box -- previous commit, this tree without the pipelined-loop tests, this tree -- in turn, twice.
# Stops at the first GPU fault.
set -o pipefail
O=$PWD/gpurun_out/s28
mkdir -p $O
T="timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread"
S="tests/test_gpu_rxloop.py tests/test_gpu_host.py tests/test_gpu_staged.py tests/test_gpu_fuzz.py"
for k in 1 2; do
  (cd _ab_old && $T $S > $O/old$k.log 2>&1); echo "old$k rc=$? $(tail -1 $O/old$k.log)"
  grep -q "illegal memory access\|Memory access fault" $O/old$k.log && exit 3
  $T -k "not pipe" $S > $O/nopipe$k.log 2>&1; echo "nopipe$k rc=$? $(tail -1 $O/nopipe$k.log)"
  grep -q "illegal memory access\|Memory access fault" $O/nopipe$k.log && exit 3
  $T $S > $O/new$k.log 2>&1; echo "new$k rc=$? $(tail -1 $O/new$k.log)"
  grep -q "illegal memory access\|Memory access fault" $O/new$k.log && exit 3
done
exit 0
