cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1u
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -4 "$O/$name.log"; return $rc; }
run wiretests 600 python -u -m pytest tests/test_gpu_wire.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
run gputests 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
run bench_c3_wire 300 python bench.py --steps 20 --warmup 3 --no-cpu --opts 7 || exit 1
run bench_c4_wire 300 python bench.py --steps 20 --warmup 3 --no-cpu --opts 7 --config c4 || exit 1
run bench_c2_wire 300 python bench.py --steps 20 --warmup 3 --no-cpu --opts 7 --config c2 || exit 1
echo done
