# Round 3: LOWLAT with the templated leader poll: GPU suite, latency table.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3e; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -2 "$O/$name.log"; return $rc; }
run gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
run hostlat 400 python tools/hostlat.py --modes lowlat,zerocopy,staged --batches 64,256,1024,4096 --lens 64,1500 --reps 300 || exit 1
run smallbatch 300 python tools/smallbatch.py --reps 200 || exit 1
echo done
