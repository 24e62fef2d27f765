# GPU session K: full suite (incl. multi-chunk staged pipeline), host-inclusive bench, N=2 rehearsal on one GPU.
cd "$GRAFT_REPO_ROOT" || exit 3
O=$GRAFT_REPO_ROOT/gpurun_out/r1k
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -3 "$O/$name.log"; return $rc; }
run gputests 900 python -m pytest tests -m gpu -q -x --timeout 600 -p no:cacheprovider || exit 1
run bench_hi 600 python bench.py --steps 10 --warmup 2 --no-cpu --host-inclusive || exit 1
XSK_BENCH_SHARE_GPU=1 run bench_n2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --pool-cap 3 --no-cpu || exit 1
echo done
