# Round 3: SLACK confirmation (tune/xsk_tune_slack.hip) -- shipped (-1), SLACK 0 through the tuning library (2000), SLACK 2 (2002), SLACK 2
# for ragged-tile waves only (2001); c4, c3, c2, p98.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3af; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-900; return $rc; }
XSK_TUNE_TESTS=1 run tests 300 python -u -m pytest tests/test_gpu_tune.py -k "slack_candidate" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
for c in c4 c3 c2 p98; do run ab_$c 300 python tools/abbench.py --config $c --variants=-1,2000,2002,2001 --rounds 8 || exit 1; done
echo done
