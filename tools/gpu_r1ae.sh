cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1ae
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; return $rc; }
run bench_c3 400 python bench.py --steps 20 --warmup 3 || exit 1
for c in c4 c2; do run bench_$c 300 python bench.py --steps 20 --warmup 3 --no-cpu --config $c || exit 1; done
echo done
