# Round 3: masks-once ragged streams (product, RAGGED 2) vs the sorted streams (1001) in-process; LOWLAT with
# per-workgroup doorbell lines.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3d; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -2 "$O/$name.log"; return $rc; }
run gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for c in c4 c3 c2 p98; do run ab_$c 300 python tools/abbench.py --config $c --variants=-1,1001 --rounds 6 || exit 1; done
run hostlat 400 python tools/hostlat.py --modes lowlat --batches 64,256,1024 --lens 64,1500 --reps 300 || exit 1
run linefetch 300 python tools/linefetch.py 0,1,2,3,4 3 || exit 1
for m in 0 1 3 4; do run lf_fetch_$m 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/lf_fetch_$m -o run -- python3 $GRAFT_REPO_ROOT/tools/linefetch.py $m 1 || exit 1; done
echo done
