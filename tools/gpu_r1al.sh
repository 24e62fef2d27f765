cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1al
mkdir -p $O
timeout -k 10 300 python tools/glds.py > $O/glds.log 2>&1 || exit 1
echo done
