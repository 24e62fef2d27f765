cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1h
mkdir -p $O
summ() { grep variant $1 | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['layout'],'pool',d['pool'],'v',d['variant'],'g',d['grid'],d['us_med'],d['gbs_med'],d['mframes_s'])"; }
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -k "variants" --timeout 300 -p no:cacheprovider > $O/vparity.log 2>&1 || { tail -30 $O/vparity.log; exit 1; }
tail -1 $O/vparity.log
timeout -k 10 900 python tools/kbench.py --reps 3 --pool 10 --layouts c3_s4096,c4_s2048,c2_s64 --variants 0,50,51,52 --grids -1 > $O/kb.log 2>&1 || exit 1
summ $O/kb.log
