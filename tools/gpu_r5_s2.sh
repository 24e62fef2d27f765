# Round 5, session 2: the tuning-variant parity tests (pruned list + the c2 short-tile grids), the deterministic LOWLAT
# partial-timeout test, and the c2 A/B of the pipelined short-tile grids.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/s2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tune.py "tests/test_gpu_staged.py::test_lowlat_partial_timeout_deterministic" -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "FAILED|ERROR|hog claims" $O/tests.log | head
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/abbench.py --config c2 --variants=-1,30,36,37,38,39 --rounds 8 > $O/ab_c2_sgp.log 2>&1; rc=$?
tail -2 $O/ab_c2_sgp.log | cut -c1-1500
exit $rc
