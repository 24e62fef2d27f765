cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
run gputests 900 python -m pytest tests -m gpu -q --timeout 600; ok $? || exit 1
run kbench 900 python tools/kbench.py --reps 8; ok $? || exit 1
cat gpurun_out/kbench.log
