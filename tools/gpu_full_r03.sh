# Round-3 full GPU pass (run through gpurun): PMC FETCH_SIZE / WRITE_SIZE / SQ passes of the c3, c4 and c2 benches
# (first, so the bench lines below attach the traffic of exactly this build: the summaries carry its build id and
# are copied into the box's profiles/; copy them to the repo's profiles/ afterwards), the GPU suite, smoke, bench
# lines, the N=2 shared-GPU rehearsal, and the rocprofv3 kernel-trace summary of every config.
#   Usage: bash tools/gpu_full_r03.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/${1:-full}
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300; return $rc; }
SQ="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_WAVE_CYCLES"
declare -A ALG=([c3]=1572864000 [c4]=819879113 [c2]=67108864)
for c in c3 c4 c2; do
  B="python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 4 --warmup 1 --no-cpu"
  run pmc_fetch_$c 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_fetch_$c -o run -- $B || exit 1
  run pmc_write_$c 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_write_$c -o run -- $B || exit 1
  run pmc_sq_$c 240 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_sq_$c -o run -- $B || exit 1
  run traffic_$c 60 python3 tools/pmc_summary.py $O/pmc_fetch_$c $O/pmc_write_$c ${ALG[$c]} $O/traffic_$c.json || exit 1
  run sqsum_$c 60 python3 tools/sq_summary.py $O/pmc_sq_$c $O/sq_$c.json || exit 1
  cp $O/traffic_$c.json profiles/traffic_$c.json || exit 1
done
run gputests 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench_c3 300 python bench.py --steps 20 --warmup 5 --host-inclusive || exit 1
run bench_c4 200 python bench.py --config c4 --steps 20 --warmup 5 --no-cpu || exit 1
run bench_c2 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu || exit 1
run bench_p98 200 python bench.py --config p98 --steps 20 --warmup 5 --no-cpu || exit 1
run bench_c3_wire 200 python bench.py --opts 7 --steps 20 --warmup 5 --no-cpu || exit 1
run bench_c5 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu || exit 1
XSK_BENCH_SHARE_GPU=1 run bench_c3_n2_shared 200 python bench.py --gpus 2 --steps 10 --warmup 2 --pool-cap 8 --no-cpu || exit 1
for c in c3 c4 c2; do
  run prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 20 --warmup 5 --no-cpu || exit 1
done
echo done
