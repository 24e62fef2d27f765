# Round 5, session 9: STAGED with pinned descriptor staging -- host/staged tests, the staged sweep, the PCIe ceilings.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/s9; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_host.py tests/test_gpu_rxloop.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/staged_sweep.py --reps 15 > $O/staged_sweep.jsonl 2>&1 || exit 1
cat $O/staged_sweep.jsonl
timeout -k 10 300 python -u tools/pcie_ceiling.py > $O/pcie_ceiling.json 2>&1 || exit 1
cat $O/pcie_ceiling.json
