cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1bm
mkdir -p $O
GLDS_KINDS=0,7,9 GLDS_CASES=c4like_rows_s2048,c3_rows_s4096 timeout -k 10 300 python tools/glds.py > $O/glds.log 2>&1 || exit 1
timeout -k 10 300 python tools/kbench.py --layouts c4_s2048 --variants 92,89,10 --pool 8 --reps 8 > $O/kb.log 2>&1 || exit 1
echo done
