# Round-1 GPU session E: v4 with 64-B window write-back (40) vs partial stores (45), parity first.
cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1e
mkdir -p $O
summ() { grep variant $1 | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['layout'],'pool',d['pool'],'v',d['variant'],'g',d['grid'],d['us_med'],d['gbs_med'],d['mframes_s'])"; }
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -k "variants or golden or mixed" --timeout 300 -p no:cacheprovider > $O/vparity.log 2>&1 || { tail -30 $O/vparity.log; exit 1; }
tail -1 $O/vparity.log
timeout -k 10 900 python tools/kbench.py --reps 3 --pool 10 --layouts c3_s4096,c4_s2048,c2_s64 --variants 0,21,40,45,43,10 --grids 0,-1 > $O/kb.log 2>&1 || exit 1
summ $O/kb.log
