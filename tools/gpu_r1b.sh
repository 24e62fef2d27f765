# Round-1 GPU session B: cold-batch (pool) vs warm sweep, rocprof kernel-trace stats + PMC passes of bench.py.
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r1b
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -2 "$O/$name.log"; return $rc; }
summ() { grep variant $1 | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['layout'],'pool',d['pool'],'v',d['variant'],d['us_med'],d['gbs_med'])"; }
run kb_warm 600 python tools/kbench.py --reps 5 --pool 1 --layouts c3_s4096,c3_s1504 --variants 0,10,30,-1 || exit 1
summ $O/kb_warm.log
run kb_cold 600 python tools/kbench.py --reps 3 --pool 12 --layouts c3_s4096,c3_s1504 --variants 0,10,30,-1 || exit 1
summ $O/kb_cold.log
cd /tmp
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu || exit 1
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu || exit 1
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu || exit 1
find $O -name "*.csv"
