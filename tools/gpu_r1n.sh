cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1n
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -3 "$O/$name.log"; return $rc; }
run gputests 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "classify or more_tiles or spanning" --timeout 600 -p no:cacheprovider || exit 1
run cbench 300 python tools/classify_bench.py || exit 1
cd /tmp
run cprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cprof -o run -- python3 $GRAFT_REPO_ROOT/tools/classify_bench.py || exit 1
echo done
