cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1x
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -3 "$O/$name.log" | cut -c1-300; return $rc; }
run drift 300 python tools/drift.py 22 big || exit 1
echo done
