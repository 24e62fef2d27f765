cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
run gputests 900 python -m pytest tests -m gpu -q --timeout 600; ok $? || exit 1
run kbench 900 python tools/kbench.py --reps 6 --layouts c3_s4096,c3_s1536,c4_s2048,c2_s64 --variants 0,1,2,4,5,6,10 --grids 0,-1,2048,1024; ok $? || exit 1
grep variant gpurun_out/kbench.log | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['layout'],d['variant'],d['grid'],d['us_med'],d['gbs_med'])"
