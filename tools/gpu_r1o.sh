cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1o
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -3 "$O/$name.log"; return $rc; }
run gputests 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
run bench_c3 300 python bench.py --steps 20 --warmup 3 --no-cpu || exit 1
run wexp 300 python tools/wexp.py 4096 0,4,11,12,13,14,5,8 4096 || exit 1
run kb_c2 300 python tools/kbench.py --layouts c2_s64 --variants 0,53 --pool 8 || exit 1
echo done
