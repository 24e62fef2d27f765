# Round 3: per-workgroup end-time spread of the shipped kernel (timing probes 10-12: shares as shipped, share g ^ 1,
# round-interleaved shares), c3 / c4 / c2.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3l; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-600; return $rc; }
for c in c3 c4 c2; do run spread_$c 240 python tools/wg_spread.py --config $c --variants 10,11,12 --rounds 2 || exit 1; done
echo done
