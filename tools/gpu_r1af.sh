cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1af
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-150; return $rc; }
run wiretests 600 python -u -m pytest tests/test_gpu_wire.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for c in c3 c4 c2; do run bench_${c}_wire 300 python bench.py --steps 20 --warmup 3 --no-cpu --opts 7 --config $c || exit 1; done
for c in c3 c4; do XSK_WIRE_IMPL=1 run bench_${c}_wire_old 300 python bench.py --steps 20 --warmup 3 --no-cpu --opts 7 --config $c || exit 1; done
echo done
