# Round 3: GPU suite on the multi-workgroup LOWLAT build, then the host-UMEM latency table.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3c; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -3 "$O/$name.log"; return $rc; }
run gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run hostlat 400 python tools/hostlat.py --modes lowlat,zerocopy --batches 64,256,1024 --lens 64,1500 --reps 200 || exit 1
run hostlat_g1 200 python tools/hostlat.py --modes lowlat --batches 256,1024 --lens 64,1500 --reps 200 --groups 1 || exit 1
echo done
