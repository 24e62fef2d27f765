cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1ak
mkdir -p $O
timeout -k 10 400 python tools/kbench.py --layouts c4_s2048,c4ramp_s2048 --variants 10,76,85,79 --pool 8 --reps 8 > $O/kb.log 2>&1 || exit 1
echo done
