cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1j
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x --timeout 300 -p no:cacheprovider > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 300 python tools/wexp.py 4096 0,4 4096 > $O/w.log 2>&1 || { cat $O/w.log; exit 1; }
cat $O/w.log
timeout -k 10 600 python tools/kbench.py --reps 3 --pool 10 --layouts c2_s64,c3_s4096,c4_s2048 --variants 0,52,53,54 --grids -1 > $O/kb.log 2>&1 || exit 1
grep variant $O/kb.log | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['layout'],'v',d['variant'],d['us_med'],d['gbs_med'],d['mframes_s'])"
