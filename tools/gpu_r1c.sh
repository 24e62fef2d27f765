# Round-1 GPU session C: parity of the v4 row-streaming kernels, then cold-batch sweep.
cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1c
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -2 "$O/$name.log"; return $rc; }
summ() { grep variant $1 | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['layout'],'pool',d['pool'],'v',d['variant'],'g',d['grid'],d['us_med'],d['gbs_med'],d['mframes_s'])"; }
run vparity 600 python -m pytest tests/test_gpu_parity.py -q -x -k "variants" --timeout 300 -p no:cacheprovider || exit 1
run kb_cold 900 python tools/kbench.py --reps 3 --pool 10 --layouts c3_s4096,c4_s2048,c2_s64 --variants 0,40,41,42,43,44,10 --grids 0,-1 || exit 1
summ $O/kb_cold.log
