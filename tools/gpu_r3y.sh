# Round 3: host-UMEM throughput of Q independent RX queues (one context, UMEM and thread each) at RX-loop batch sizes.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3y; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-600; return $rc; }
for m in lowlat zerocopy; do
  for q in 1 2 4 8; do run ${m}_q${q}_64 60 ./tools/rxqueues $q 64 $m 2 len=64 || exit 1; done
  for q in 1 4; do run ${m}_q${q}_1500 60 ./tools/rxqueues $q 64 $m 2 len=1500 || exit 1; done
done
echo done
