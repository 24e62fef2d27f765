cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1bg
mkdir -p $O
GLDS_KINDS=0,7,9 GLDS_CASES=c3_rows_s4096,c3_framemajor_s4096,c3_rows128_s4096,contig_1.5GB timeout -k 10 300 python tools/glds.py > $O/glds.log 2>&1 || exit 1
echo done
