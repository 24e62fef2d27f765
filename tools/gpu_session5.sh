cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -k "variants" --timeout 300 > gpurun_out/vt.log 2>&1; rc=$?
tail -3 gpurun_out/vt.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python tools/kbench.py --reps 6 --layouts c3_s4096,c3_s1536,c4_s2048,c2_s64 --variants 0,30,31,32,33,10 --grids 0,-1 > gpurun_out/kbench5.log 2>&1 || exit 1
grep variant gpurun_out/kbench5.log | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['layout'],d['variant'],d['grid'],d['us_med'],d['gbs_med'])"
