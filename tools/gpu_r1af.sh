cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1af
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-150; return $rc; }
run gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1


echo done
