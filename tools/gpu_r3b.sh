# Round 3 check of the refactored product kernel: GPU suite, in-process A/B product (-1) vs the lab copy of
# the round-2 kernel (158), one bench line.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3b; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -2 "$O/$name.log"; return $rc; }
run gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for c in c3 c4 c2; do run ab_$c 300 python tools/abbench.py --config $c --variants=-1,158 --rounds 4 || exit 1; done
run bench_c3 300 python bench.py --steps 20 --warmup 5 --no-cpu || exit 1
echo done
