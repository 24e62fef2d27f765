# Full pass, part 1 (run through gpurun): PMC FETCH_SIZE / WRITE_SIZE / SQ passes of the c3, c4 and c2 benches
# and their summaries (they carry the build id; copy gpurun_out/<tag>/traffic_*.json to profiles/ afterwards, so
# part 2's bench lines attach them).   Usage: bash tools/gpu_full_a.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/${1:-fulla}
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300; return $rc; }
SQ="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_WAVE_CYCLES"
declare -A ALG=([c3]=1572864000 [c4]=819879113 [c2]=67108864 [c3_opts7]=1572864000 [c5]=1572864000)
# c3_opts7: c3 in wire mode (bench.py --opts 7 reads profiles/traffic_c3_opts7.json); c5: per launch of 1 M frames (a
# call is 64 such launches over consecutive slices of its descriptors)
for c in c3 c4 c2 c3_opts7 c5; do
  cfg=${c%_opts7}; X=""; [ "$c" != "$cfg" ] && X="--opts 7"
  S="--steps 4 --warmup 1"; [ "$c" = c5 ] && S="--steps 1 --warmup 1"
  B="python3 $GRAFT_REPO_ROOT/bench.py --config $cfg $X $S --no-cpu"
  run pmc_fetch_$c 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_fetch_$c -o run -- $B || exit 1
  run pmc_write_$c 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_write_$c -o run -- $B || exit 1
  run pmc_sq_$c 240 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_sq_$c -o run -- $B || exit 1
  run traffic_$c 60 python3 tools/pmc_summary.py $O/pmc_fetch_$c $O/pmc_write_$c ${ALG[$c]} $O/traffic_$c.json || exit 1
  run sqsum_$c 60 python3 tools/sq_summary.py $O/pmc_sq_$c $O/sq_$c.json || exit 1
done
echo done
