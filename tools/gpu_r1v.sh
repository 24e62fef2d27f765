cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1v
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -2 "$O/$name.log"; return $rc; }

run kb 600 python tools/kbench.py --layouts c3_s4096 --variants 76,85,-1 --pool 8 || exit 1
echo done
