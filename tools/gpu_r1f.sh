cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1f
mkdir -p $O
timeout -k 10 300 python tools/wexp.py 4096 > $O/w4096.log 2>&1 || { cat $O/w4096.log; exit 1; }
cat $O/w4096.log
timeout -k 10 300 python tools/wexp.py 1536 0,1,4 4096 > $O/w1536.log 2>&1 || exit 1
cat $O/w1536.log
