#!/bin/bash
# Round 5: whole GPU suite (driver order) + smoke + bench on the build with the final tree of the session.
set -o pipefail
O=gpurun_out/s53
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1; rc=$?
tail -1 $O/bench.log
exit $rc
