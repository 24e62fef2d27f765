cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
timeout -k 10 600 python tools/kbench.py --reps 6 --layouts c3_s4096,c2_s64 --variants 0,21,22,24,27,10 --grids 0,-1 > gpurun_out/kbench4.log 2>&1 || exit 1
grep variant gpurun_out/kbench4.log | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['layout'],d['variant'],d['grid'],d['us_med'],d['gbs_med'])"
