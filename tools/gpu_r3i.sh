# Round 3: c4's per-launch time against the batch's position in the pool slab (forward / reverse order).
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3i; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300; return $rc; }
run pos_c4 200 python tools/pool_position.py --config c4 --pool 24 || exit 1
run pos_c4_sep 200 python tools/pool_position.py --config c4 --pool 24 --alloc separate || exit 1
run pos_c3 200 python tools/pool_position.py --config c3 --pool 20 || exit 1
run pos_p98 200 python tools/pool_position.py --config p98 --pool 24 || exit 1
echo done
