cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1bc
mkdir -p $O
timeout -k 10 500 python tools/wireab.py > $O/wire.log 2>&1 || { tail -5 $O/wire.log; exit 1; }
echo done
