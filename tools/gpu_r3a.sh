cd "$GRAFT_REPO_ROOT" || exit 3
mkdir -p gpurun_out/r3a
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3a/bench_c3.json 2> gpurun_out/r3a/bench_c3.err && \
XSK_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --pool-cap 6 > gpurun_out/r3a/bench_n2.json 2> gpurun_out/r3a/bench_n2.err
echo rc=$?
