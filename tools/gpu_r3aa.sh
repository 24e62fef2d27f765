# Round 3: LDS pressure of the shipped kernel -- SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra / all LDS-array
# cycles), SQ_WAIT_INST_LDS, SQ_LDS_UNALIGNED_STALL, per launch, c3 / c4 / c2.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3aa; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300; return $rc; }
L="SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAIT_INST_LDS,SQ_LDS_UNALIGNED_STALL,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES"
for c in c3 c4 c2; do
  run lds_$c 240 timeout -s KILL 200 rocprofv3 --pmc $L --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/lds_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 4 --warmup 1 --no-cpu || exit 1
  run ldssum_$c 60 python3 tools/sq_summary.py $O/lds_$c $O/lds_$c.json || exit 1
done
echo done
