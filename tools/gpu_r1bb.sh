cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1bb
mkdir -p $O
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > $O/bench_c3.log 2>&1 || exit 1
tail -1 $O/bench_c3.log
echo done
