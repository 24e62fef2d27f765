# Round 5, session 7: LDS bank-conflict and issue counters of the shipped (HB) kernel on c3 / c4 / p98 / c2.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/s7; mkdir -p $O
export TMPDIR=/tmp
for c in c3 c4 p98 c2; do
  timeout -k 10 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_WAVE_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/$O/lds_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 4 --warmup 1 --no-cpu > $O/lds_$c.log 2>&1 || exit 1
  timeout -k 10 60 python3 tools/sq_summary.py $O/lds_$c $O/lds_$c.json | cut -c1-600 || exit 1
done
