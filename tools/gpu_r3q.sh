# Round 3: consecutive batches on one stream vs. alternating over 2 / 3 streams (tools/overlap.py).
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3q; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-900; return $rc; }
for c in c3 c4 c2; do run overlap_$c 300 python tools/overlap.py --config $c --steps 20 --streams 1,2,3 --reps 3 || exit 1; done
echo done
