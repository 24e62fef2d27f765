# Full GPU pass (run through gpurun): gpu tests, smoke, bench lines for c3/c4/c2 (+wire c3), the rocprofv3
# kernel-trace summary and the FETCH_SIZE / WRITE_SIZE passes of the c3 bench (run first, so that the
# bench lines report the traffic of this build: copy $O/traffic_c3.json to profiles/ afterwards).  Usage: bash tools/gpu_full.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/${1:-full}
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log"; return $rc; }
# PMC passes first: the c3 bench line then carries the traffic of exactly this build
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu || exit 1
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu || exit 1
run traffic 60 python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write 1572864000 $O/traffic_c3.json || exit 1
export XSK_TRAFFIC_JSON=$GRAFT_REPO_ROOT/$O/traffic_c3.json
run gputests 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench_c3 400 python bench.py --steps 20 --warmup 3 || exit 1
run bench_c4 300 python bench.py --config c4 --steps 20 --warmup 3 --no-cpu || exit 1
run bench_c2 300 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu || exit 1
run bench_p98 300 python bench.py --config p98 --steps 20 --warmup 3 --no-cpu || exit 1
run bench_c3_wire 300 python bench.py --opts 7 --steps 20 --warmup 3 --no-cpu || exit 1
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu || exit 1
echo done
