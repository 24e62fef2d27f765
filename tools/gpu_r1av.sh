cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1av
mkdir -p $O
timeout -k 10 200 python tools/kbench.py --layouts c3_s4096 --variants 88,90,91 --pool 8 --reps 3 > $O/kb0.log 2>&1 || exit 1
timeout -k 10 500 python tools/kbench.py --layouts c3_s4096,c4_s2048,c2_s64,p98_s2048 --variants 88,90,91 --pool 8 --reps 8 > $O/kb.log 2>&1 || exit 1
echo done
