# Round 5, session 12: the new LOWLAT serving-group rule -- host / staged / RX-loop / wire GPU tests, the auto-rule
# latency sweep, RX ring rates at 1500 B and the empty-ring 64-frame latency.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/s12; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_staged.py tests/test_gpu_rxloop.py tests/test_gpu_wire.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/hostlat.py --lens 64,512,1500 --modes lowlat --batches 64,96,128,192,256,384,512,1024 --reps 400 > $O/auto.jsonl 2>&1 || exit 1
for st in 64 256 1024; do timeout -k 10 60 tools/rxring $st lowlat 2 len=1500 >> $O/rxring.jsonl 2>&1 || exit 1; done
timeout -k 10 60 tools/rxring 64 lowlat 2 empty=1 >> $O/rxring.jsonl 2>&1 || exit 1
