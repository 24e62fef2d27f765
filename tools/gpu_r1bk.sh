cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r1bk
mkdir -p $O
XSK_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 10 --warmup 2 --pool-cap 4 > $O/n2.log 2>&1 || { tail -20 $O/n2.log; exit 1; }
grep "^{" $O/n2.log | tail -1 | cut -c1-400
echo done
