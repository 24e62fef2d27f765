# Round 3: rank 0's multi-GPU host-inclusive leg, rehearsed on one GPU (N = 2 and 4 ranks on cuda:0, gloo), and the
# default bench line.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3o; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-1500; return $rc; }
XSK_BENCH_SHARE_GPU=1 run n2_shared 300 python bench.py --gpus 2 --steps 10 --warmup 2 --pool-cap 6 --no-cpu || exit 1
XSK_BENCH_SHARE_GPU=1 run n4_shared 300 python bench.py --gpus 4 --steps 10 --warmup 2 --pool-cap 4 --no-cpu || exit 1
run bench_c3 300 python bench.py --steps 20 --warmup 5 || exit 1
echo done
