cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1bj
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
KB="python3 $GRAFT_REPO_ROOT/tools/kbench.py --layouts c4_s2048,c3_s4096 --variants 92,88 --pool 2 --reps 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/sq -o run -- $KB > $O/sq.log 2>&1 || exit 1
echo done
