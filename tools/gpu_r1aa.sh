cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1aa
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300; return $rc; }


run c5test 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "synth or full_size" --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
run bench_c5_n1 600 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu || exit 1
XSK_BENCH_SHARE_GPU=1 run bench_c3_n2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --pool-cap 3 --no-cpu || exit 1
XSK_BENCH_SHARE_GPU=1 run bench_c5_n2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config c5 --steps 3 --warmup 1 --pool-cap 1 --no-cpu || exit 1
echo done
