# Round 5, session 6: the whole GPU suite and smoke on the HB build, then RX-loop latency (empty ring) and one c2 / c3
# bench line each.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/s6; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1; rc=$?
tail -2 $O/gputests.log; grep -E "FAILED|ERROR" $O/gputests.log | head
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
for st in 64 1024; do timeout -k 10 60 tools/rxring $st lowlat 2 empty=1 >> $O/rxring_empty.jsonl 2>&1 || exit 1; done
timeout -k 10 60 tools/rxring 1024 lowlat 2 >> $O/rxring_empty.jsonl 2>&1 || exit 1
cut -c1-330 $O/rxring_empty.jsonl
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu > $O/bench_c2.json 2>$O/bench_c2.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_c3.json 2>$O/bench_c3.err || exit 1
python3 -c "
import json
for c in ('c2','c3'):
    d=json.loads(open('$O/bench_'+c+'.json').read().strip().splitlines()[-1]); r=d['roofline']
    print(c, d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('traffic_source'))
"
