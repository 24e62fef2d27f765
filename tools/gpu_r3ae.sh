# Round 3: SYNC 2 with SLACK (a heavy wave writes once all but 2 / 4 / 8 waves have read; product switch 16-18).
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3ae; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-900; return $rc; }
run tests 300 python -u -m pytest tests/test_gpu_tune.py -k "product_switch" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
for c in c3 c4; do run ab_$c 300 python tools/abbench.py --config $c --variants=-1,1016,1017,1018 --rounds 6 || exit 1; done
echo done
