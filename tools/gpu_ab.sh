# Cold A/B of tuning-library kernel variants inside one GPU call (run through gpurun): every variant of
# every config timed by bench.py --variant in its own process, the variants interleaved per repetition so
# that box drift hits them alike; prints one "config variant kernel_avg_us" line per run.
#   bash tools/gpu_ab.sh <out-dir> <configs,comma> <variants,comma> <reps>
cd "$GRAFT_REPO_ROOT" || exit 3
O=$1; CFGS=$2; VARS=$3; REPS=${4:-2}
mkdir -p $O
for r in $(seq 1 $REPS); do
  for c in ${CFGS//,/ }; do
    for v in ${VARS//,/ }; do
      f=$O/b_${v}_${c}_$r.json
      timeout -k 10 240 python bench.py --config $c --variant $v --steps 20 --warmup 3 --no-cpu > $f 2> $O/b_${v}_${c}_$r.err || { echo "FAIL $c $v rc=$?"; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$c', $v, d['roofline']['kernel_avg_us'], d['ms_per_step'])"
    done
  done
done
