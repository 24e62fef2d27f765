cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1ai
mkdir -p $O
timeout -k 10 300 python tools/xcd_balance.py > $O/xcd.log 2>&1 || exit 1
echo done
