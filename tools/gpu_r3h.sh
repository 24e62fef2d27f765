# Round 3: ROLL (rolled tile loop: 46 KB of kernel code instead of 78 KB) A/B against the shipped kernel; tests.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3h; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -2 "$O/$name.log"; return $rc; }
run gputests 900 python -u -m pytest tests/test_gpu_tune.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for c in c4 p98 c3 c2; do run ab_$c 300 python tools/abbench.py --config $c --variants=-1,1001 --rounds 8 || exit 1; done
echo done
