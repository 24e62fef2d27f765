# Round 5, session 4: tuning-variant parity (HB = 42), the in-process A/B of HB on c2 / c3 / c4 / p98, LDS bank-conflict
# counters of the shipped kernel vs HB on c2, and SQ counters of the SG diagnostics.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/s4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tune.py tests/test_gpu_staged.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head
[ $rc -le 1 ] || exit $rc
for c in c2 c3 c4 p98; do
  timeout -k 10 300 python -u tools/abbench.py --config $c --variants=-1,42 --rounds 8 > $O/ab_${c}_hb.log 2>&1 || exit 1
  tail -1 $O/ab_${c}_hb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', {k: d[k]['median_us'] for k in ('-1','42')}, d['outputs_equal_shipped'])"
done
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/$O/lds_c2 -o run -- python3 $GRAFT_REPO_ROOT/tools/abbench.py --config c2 --variants=-1,42 --rounds 2 > $O/lds_c2.log 2>&1 || exit 1
timeout -k 10 60 python3 tools/sq_summary.py $O/lds_c2 $O/lds_c2_shipped.json "echo_round_kernel<false, false, 6, true, true, 2, false>" | cut -c1-500 || exit 1
timeout -k 10 60 python3 tools/sq_summary.py $O/lds_c2 $O/lds_c2_hb.json "echo_round_kernel<false, false, 6, true, true, 2, true>" | cut -c1-500 || exit 1
SQ="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_WAVE_CYCLES"
timeout -k 10 120 rocprofv3 --pmc $SQ --output-format csv -d $GRAFT_REPO_ROOT/$O/sq_sg -o run -- python3 $GRAFT_REPO_ROOT/tools/abbench.py --config c2 --variants=30,40,41 --rounds 2 > $O/sq_sg.log 2>&1 || exit 1
for v in "0>" "1>" "2>"; do
  timeout -k 10 60 python3 tools/sq_summary.py $O/sq_sg $O/sq_sg_${v%>}.json "short_grid_kernel<false, 4, true, $v" | cut -c1-500 || exit 1
done
