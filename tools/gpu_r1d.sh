# Round-1 GPU session D: ablations of the v2 kernel (write-back / records / header DMA) on cold batches.
cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1d
mkdir -p $O
summ() { grep variant $1 | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['layout'],'pool',d['pool'],'v',d['variant'],'g',d['grid'],d['us_med'],d['gbs_med'],d['mframes_s'])"; }
timeout -k 10 900 python tools/kbench.py --reps 3 --pool 10 --layouts c3_s4096,c4_s2048 --variants 0,21,22,24,27,10,-1 --grids 0,-1 > $O/kb_abl.log 2>&1 || exit 1
summ $O/kb_abl.log
