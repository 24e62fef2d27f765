# Round 3: the read-ceiling kernel rewritten (per-workgroup contiguous shares) -- its test and the bench lines that
# carry it; lab variants 173-175 (the shipped kernel with U = 2 / 3 / 6) -- parity and in-process A/B.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3r; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-900; return $rc; }
run tests 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tune.py -k "stream_read or kernel_variants_parity" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
run bench_c3 200 python bench.py --steps 20 --warmup 5 --no-cpu || exit 1
run bench_c2 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu || exit 1
for c in c3 c4 c2; do run ab_$c 300 python tools/abbench.py --config $c --variants=-1,158,173,174,175 --rounds 4 || exit 1; done
echo done
