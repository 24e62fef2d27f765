cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1aw
mkdir -p $O
timeout -k 10 400 python tools/kbench.py --layouts c2_s64,p98_s2048 --variants 86,85,89,70,78,10 --pool 8 --reps 8 > $O/kb.log 2>&1 || exit 1
echo done
