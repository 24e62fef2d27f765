cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
run() { # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" ; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -5 "gpurun_out/$name.log"
  return $rc
}
rocm-smi --showproductname > gpurun_out/smi.log 2>&1
run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run gputests 900 python -m pytest tests -m gpu -q --timeout 600; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run bench 500 python bench.py --steps 10 --warmup 2 --no-cpu
