# Round-1 GPU session A: smoke, parity suite, variant sweep, bench, rocprof kernel-trace + PMC passes.
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
mkdir -p gpurun_out/r1a
O=gpurun_out/r1a
run() { # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -3 "$O/$name.log"; return $rc
}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }  # 1 = test failures (keep going); anything else = stop
(lscpu; nproc; rocm-smi --showproductname) > $O/host.log 2>&1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; ok $? || exit 1
run gputests 900 python -m pytest tests -m gpu -q -x --timeout 600 -p no:cacheprovider; ok $? || exit 1
run kbench 600 python tools/kbench.py --reps 6 --layouts c3_s4096,c2_s64,c4_s2048 --variants 0,1,30,31,10 --grids 0; ok $? || exit 1
grep variant $O/kbench.log | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['layout'],d['variant'],d['grid'],d['us_med'],d['gbs_med'])"
run bench 600 python bench.py --steps 20 --warmup 3; ok $? || exit 1
tail -1 $O/bench.log
cd /tmp
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu || exit 1
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu || exit 1
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu || exit 1
find $GRAFT_REPO_ROOT/$O -name "*.csv" | head -20
