cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1bl
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "variants_parity or uniform_tiles or valid_parity or golden" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 500 python tools/kbench.py --layouts c2_s64,p98_s2048 --variants 88,92 --pool 8 --reps 12 > $O/kb.log 2>&1 || exit 1
echo done
