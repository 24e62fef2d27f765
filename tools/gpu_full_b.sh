# Full pass, part 2: the GPU suite, smoke, the bench lines (with part 1's traffic summaries in profiles/), the
# N = 2 shared-GPU rehearsal and the rocprofv3 kernel-trace summary of every config.   Usage: bash tools/gpu_full_b.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/${1:-fullb}
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300; return $rc; }
run gputests 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench_c3 300 python bench.py --steps 20 --warmup 5 --host-inclusive || exit 1
run bench_c4 200 python bench.py --config c4 --steps 20 --warmup 5 --no-cpu || exit 1
run bench_c2 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu || exit 1
run bench_p98 200 python bench.py --config p98 --steps 20 --warmup 5 --no-cpu || exit 1
run bench_c3_wire 200 python bench.py --opts 7 --steps 20 --warmup 5 --no-cpu || exit 1
run bench_c4_wire 200 python bench.py --config c4 --opts 7 --steps 20 --warmup 5 --no-cpu || exit 1
run bench_c2_wire 200 python bench.py --config c2 --opts 7 --steps 20 --warmup 5 --no-cpu || exit 1
run bench_c5 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu || exit 1
XSK_BENCH_SHARE_GPU=1 run bench_c3_n2_shared 200 python bench.py --gpus 2 --steps 10 --warmup 2 --pool-cap 8 --no-cpu || exit 1
for c in c3 c4 c2; do
  run prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 20 --warmup 5 --no-cpu || exit 1
done
echo done
