# Full GPU pass (run through gpurun): the FETCH_SIZE / WRITE_SIZE passes of the c3, c4 and c2 benches (first,
# so that the bench lines report the traffic of exactly this build: the summaries are copied into the box's
# profiles/ and must be copied to the repo's profiles/ afterwards), an SQ pass per config, gpu tests, smoke,
# bench lines for c3/c4/c2/p98 (+wire c3), and the rocprofv3 kernel-trace summary of every config.
#   Usage: bash tools/gpu_full.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/${1:-full}
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log"; return $rc; }
SQ="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_WAVE_CYCLES"
declare -A ALG=([c3]=1572864000 [c4]=819879113 [c2]=67108864)
for c in c3 c4 c2; do
  B="python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 4 --warmup 1 --no-cpu"
  run pmc_fetch_$c 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_fetch_$c -o run -- $B || exit 1
  run pmc_write_$c 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_write_$c -o run -- $B || exit 1
  run pmc_sq_$c 300 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_sq_$c -o run -- $B || exit 1
  run traffic_$c 60 python3 tools/pmc_summary.py $O/pmc_fetch_$c $O/pmc_write_$c ${ALG[$c]} $O/traffic_$c.json || exit 1
  run sqsum_$c 60 python3 tools/sq_summary.py $O/pmc_sq_$c $O/sq_$c.json || exit 1
  cp $O/traffic_$c.json profiles/traffic_$c.json || exit 1
done
run gputests 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench_c3 400 python bench.py --steps 20 --warmup 3 || exit 1
run bench_c4 300 python bench.py --config c4 --steps 20 --warmup 3 --no-cpu || exit 1
run bench_c2 300 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu || exit 1
run bench_p98 300 python bench.py --config p98 --steps 20 --warmup 3 --no-cpu || exit 1
run bench_c3_wire 300 python bench.py --opts 7 --steps 20 --warmup 3 --no-cpu || exit 1
for c in c3 c4 c2; do
  run prof_$c 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 20 --warmup 3 --no-cpu || exit 1
done
echo done
