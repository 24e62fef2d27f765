cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1at
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
KB="python3 $GRAFT_REPO_ROOT/tools/kbench.py --layouts c4_s2048,c3_s4096 --variants 10,85,76 --pool 2 --reps 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU --kernel-trace --output-format csv -d $O/sq -o run -- $KB > $O/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace --output-format csv -d $O/tcc -o run -- $KB > $O/tcc.log 2>&1 || exit 1
echo done
