cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1l
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout 600 -p no:cacheprovider > $O/gputests.log 2>&1; rc=$?
tail -30 $O/gputests.log
exit $rc
