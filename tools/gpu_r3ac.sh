# Round 3: the GPU suite and smoke on the final tree.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3ac; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300; return $rc; }
run gputests 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench 300 python bench.py || exit 1
echo done
