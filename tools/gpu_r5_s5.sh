# Round 5, session 5: HB confirmation (reference mode, 12 rounds) and HB in wire mode (43), with their parity tests.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/s5; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tune.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head
[ $rc -le 1 ] || exit $rc
summ() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', {k: d[k]['median_us'] for k in d if k.lstrip('-').isdigit()}, d['outputs_equal_shipped'])"; }
for c in c2 c3 c4 p98; do
  timeout -k 10 400 python -u tools/abbench.py --config $c --variants=-1,42 --rounds 12 > $O/ab_${c}_hb.log 2>&1 || exit 1
  summ $O/ab_${c}_hb.log $c
done
for c in c2 c3 c4; do
  timeout -k 10 400 python -u tools/abbench.py --config $c --opts 7 --variants=-1,43 --rounds 8 > $O/ab_${c}_wire_hb.log 2>&1 || exit 1
  summ $O/ab_${c}_wire_hb.log ${c}_wire
done
