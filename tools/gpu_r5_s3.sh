# Round 5, session 3: the partial-timeout test, c2 diagnostics (SG without header phase / without LDS) beside the
# shipped kernel and c2floor's streaming modes, and SQ counters of the shipped c2 kernel vs SG.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/s3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest "tests/test_gpu_staged.py::test_lowlat_partial_timeout_deterministic" "tests/test_gpu_tune.py::test_short_tile_grid_variants" -v --timeout 100 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/abbench.py --config c2 --variants=-1,30,40,41 --rounds 8 > $O/ab_c2_diag.log 2>&1; rc=$?
tail -1 $O/ab_c2_diag.log | cut -c1-1500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/c2floor.py 3,2 5 > $O/c2floor.log 2>&1; rc=$?
tail -4 $O/c2floor.log
[ $rc -eq 0 ] || exit $rc
SQ="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_WAVE_CYCLES"
timeout -k 10 120 rocprofv3 --pmc $SQ --output-format csv -d $GRAFT_REPO_ROOT/$O/sq_ab -o run -- python3 $GRAFT_REPO_ROOT/tools/abbench.py --config c2 --variants=-1,30,40 --rounds 2 > $O/sq_ab.log 2>&1 || exit 1
for k in echo_round_kernel short_grid_kernelILb0ELi4ELb1ELi0 short_grid_kernelILb0ELi4ELb1ELi1; do
  timeout -k 10 60 python3 tools/sq_summary.py $O/sq_ab $O/sq_$k.json $k | cut -c1-600 || exit 1
done
timeout -k 10 120 python -u tools/slab_ceiling.py 128 > $O/slab_ceiling.jsonl 2>&1 || exit 1
cat $O/slab_ceiling.jsonl
