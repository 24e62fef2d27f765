# Round-1 GPU session I: shipped v5 kernel — full GPU suite, smoke, bench (+CPU baseline, host-inclusive),
# rocprofv3 kernel-trace stats and separate FETCH_SIZE / WRITE_SIZE passes of the bench command.
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r1i
mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -3 "$O/$name.log"; return $rc; }
run gputests 900 python -m pytest tests -m gpu -q -x --timeout 600 -p no:cacheprovider || exit 1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run kb 600 python tools/kbench.py --reps 3 --pool 10 --layouts c2_s64,c3_s4096,c4_s2048 --variants 0,53 --grids -1 || exit 1
grep variant $O/kb.log | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['layout'],'v',d['variant'],d['us_med'],d['gbs_med'],d['mframes_s'])"
run bench 600 python bench.py --steps 20 --warmup 3 --host-inclusive || exit 1
for c in c2 c4; do run bench_$c 300 python bench.py --steps 20 --warmup 3 --no-cpu --config $c || exit 1; done
cd /tmp
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu || exit 1
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu || exit 1
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu || exit 1
echo done
