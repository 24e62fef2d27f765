# Round 3: counter delivery -- the shipped entry point (device-scope atomics into stats, -1) against the same kernel
# writing per-workgroup partial rows (product switch 0 through the tuning library).
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3x; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-900; return $rc; }
for c in c2 c3 p98; do run ab_$c 300 python tools/abbench.py --config $c --variants=-1,1000 --rounds 10 || exit 1; done
echo done
