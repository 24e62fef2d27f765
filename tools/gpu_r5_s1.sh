# Round 5, session 1: STAGED containment / host-pack tests, the c2 short-grid A/B, the RX-ring throughput sweep.
# A test assertion failure (pytest rc 1) does not stop the later steps; any other status (a fault, an abort, a time
# limit) ends the script.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/s1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_host.py tests/test_gpu_wire.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/staged.log 2>&1; rc=$?
tail -3 $O/staged.log; grep -E "FAILED|ERROR" $O/staged.log | head
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/abbench.py --config c2 --variants=-1,30,31,32,33,34 --rounds 6 > $O/ab_c2_sg.log 2>&1; rc=$?
tail -8 $O/ab_c2_sg.log
[ $rc -eq 0 ] || exit $rc
for m in lowlat zerocopy; do for len in 64 1500; do for st in 64 256 1024; do
  timeout -k 10 60 tools/rxring $st $m 2 len=$len >> $O/rxring.jsonl 2>&1 || exit 1
done; done; done
timeout -k 10 60 tools/rxring 64 lowlat 2 empty=1 >> $O/rxring.jsonl 2>&1 || exit 1
cut -c1-300 $O/rxring.jsonl
