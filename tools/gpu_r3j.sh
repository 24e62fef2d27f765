# Round 3: c4 in bench.py (back-to-back launches) vs the position probe, same box, twice each.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3j; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300; return $rc; }
run prof_c4_a 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c4_a -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 20 --warmup 5 --no-cpu || exit 1
run pos_c4_a 200 python tools/pool_position.py --config c4 --pool 24 || exit 1
run prof_c4_b 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c4_b -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 40 --warmup 5 --no-cpu || exit 1
run bench_c4 200 python bench.py --config c4 --steps 20 --warmup 5 --no-cpu || exit 1
run prof_c3 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --steps 40 --warmup 5 --no-cpu || exit 1
echo done
