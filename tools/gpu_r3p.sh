# Round 3: two 8-wave workgroups per CU (lab variants 170 / 172) -- parity, then in-process A/B against the shipped
# entry point and the lab's copy of it (158).
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3p; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-900; return $rc; }
run tests 300 python -u -m pytest tests/test_gpu_tune.py -k "kernel_variants_parity" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
for c in c3 c4 c2; do run ab_$c 300 python tools/abbench.py --config $c --variants=-1,158,170,172 --rounds 4 || exit 1; done
echo done
