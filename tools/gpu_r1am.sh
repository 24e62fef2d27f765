cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1am
mkdir -p $O
timeout -k 10 400 python tools/statsmode.py > $O/stats.log 2>&1 || exit 1
echo done
