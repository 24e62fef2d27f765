cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1as
mkdir -p $O
timeout -k 10 600 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu > $O/bench_c5.log 2>&1 || exit 1
tail -1 $O/bench_c5.log
echo done
