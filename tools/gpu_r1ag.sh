cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1ag
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; return $rc; }
run gputests 900 python -u -m pytest tests -m gpu -q -x -k "spanning or more_tiles" --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1

echo done
