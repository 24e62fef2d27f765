# Round 3: sustained-regime A/B (abbench --burst: blocks of back-to-back launches per variant, the bench's loop) of
# c4 -- shipped (-1), without PRIO (1007), RH2 (1009) -- and c3; parity of RH2 first.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3ad; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-900; return $rc; }
run tests 300 python -u -m pytest tests/test_gpu_tune.py -k "product_switch" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
run burst_c4 300 python tools/abbench.py --config c4 --variants=-1,1007,1009 --burst 8 --rounds 6 || exit 1
run burst_c3 300 python tools/abbench.py --config c3 --variants=-1,1007 --burst 12 --rounds 4 || exit 1
echo done
