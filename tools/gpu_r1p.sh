cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1p
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -3 "$O/$name.log"; return $rc; }
run wexpA 300 python tools/wexp.py 4096 5,25,26,5,25,26 4096 || exit 1

echo done
