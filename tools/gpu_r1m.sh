cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1m
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -3 "$O/$name.log"; return $rc; }
run gputests 900 python -m pytest tests -m gpu -q -x --timeout 600 -p no:cacheprovider || exit 1
for c in c3 c2 c4; do run bench_$c 300 python bench.py --steps 20 --warmup 3 --no-cpu --config $c || exit 1; done
echo done
