cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1v
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -2 "$O/$name.log"; return $rc; }
run vtests 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k variants --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
run kb 600 python tools/kbench.py --layouts c3_s4096,c4_s2048,c2_s64,p98_s2048,m512_s2048 --variants 72,73,76,77 --pool 8 || exit 1
echo done
