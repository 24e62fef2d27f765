# In-process A/B of product-switch variants (tools/abbench.py), after their parity tests.
#   bash tools/gpu_ab.sh <tag> <variants> <rounds> <configs...>      e.g. bash tools/gpu_ab.sh r04b -1,14 6 c4 c3
#   OPTS=7 bash tools/gpu_ab.sh ...: the shipped entry point (-1) in wire mode (xsk_gpu_echo_dev_opts)
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/$1; V=$2; R=$3; shift 3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tune.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tune_tests.log 2>&1 || { tail -5 $O/tune_tests.log; exit 1; }
tail -1 $O/tune_tests.log
for c in "$@"; do
  timeout -k 10 400 python -u tools/abbench.py --config $c --variants=$V --rounds $R --opts ${OPTS:-0} > $O/ab_$c.log 2>&1 || { tail -3 $O/ab_$c.log; exit 1; }
  tail -1 $O/ab_$c.log | cut -c1-400
done
echo done
