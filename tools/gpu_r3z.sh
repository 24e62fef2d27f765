# Round 3: LOWLAT contexts per device capped at XSK_GPU_LOWLAT_PER_DEVICE (further ones run as ZEROCOPY) -- the host
# tests, then host-UMEM throughput of Q independent RX queues (tools/rxqueues) at 64-frame batches.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3z; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-600; return $rc; }
run tests 600 python -u -m pytest tests/test_gpu_host.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for q in 1 2 4 6 8; do run lowlat_q${q}_64 60 ./tools/rxqueues $q 64 lowlat 2 len=64 || exit 1; done
for q in 1 4 8; do run lowlat_q${q}_1500 60 ./tools/rxqueues $q 64 lowlat 2 len=1500 || exit 1; done
for q in 1 4 8; do run zerocopy_q${q}_64 60 ./tools/rxqueues $q 64 zerocopy 2 len=64 || exit 1; done
echo done
