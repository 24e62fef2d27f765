# Parameterised GPU session (run through gpurun): named steps in order, each its own process under its own time limit,
# output under gpurun_out/<tag>/<step>.log; the session stops at the first step that fails (a fault, an abort or a time
# limit ends the GPU work of the call).  The two full passes are tools/gpu_full_a.sh (PMC) and tools/gpu_full_b.sh
# (suite, smoke, bench lines, kernel traces); this runner is for everything between them.
#   bash tools/gpu_run.sh <tag> <step>...
# steps:
#   tests               the whole -m gpu suite, in collection order, once
#   tests:<path>        one test file or node id
#   smoke               __graft_entry__.smoke()
#   bench:<config>      bench.py --config <config> --steps 20 --warmup 5 --no-cpu
#   hostlat             tools/hostlat.py, LOWLAT / ZEROCOPY, 64 and 1024 frames of 64 and 1500 B (C1 shape)
#   rxring              tools/rxring, plain and depth-4 pipelined RX loop at 64- and 1024-frame steps, every reply
#                       checked and every failure attributed (tools/rxring.c)
#   rxdiag              tools/rxring_runs.py --diag: where the pipelined 1024 x 1500-B failures sit, and which variants have them
#   probe               tools/migrate_probe.py (page sharing, churn, NUMA migration, THP collapse under a live UMEM)
#   devptr              the device alias hipHostRegister gives a page-aligned UMEM against its host address
#   spread              tools/wg_spread.py: the shipped c3 kernel's per-workgroup start / end spread (timing probe 10)
#   overlap             tools/overlap.py: consecutive c3 batches on one stream vs alternating over 2 and 3 streams
#   overlapprof         rocprofv3 --kernel-trace of tools/overlap.py (1 and 2 streams): each launch's own duration
#   readbw              tools/readbw.py: read kernels over slab sizes, each fitted as rate + per-launch intercept
#   prof:<config>       rocprofv3 --kernel-trace --stats of bench.py --config <config>
cd "$GRAFT_REPO_ROOT" || exit 3
T=${1:?tag}; shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400; return $rc; }
PYT="python -u -m pytest -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider"
for s in "$@"; do
  case $s in
    tests) run tests 900 $PYT tests -m gpu || exit 1 ;;
    tests:*) run "tests_$(echo ${s#tests:} | sed 's/.*:://; s/.*\///; s/\.py$//' | tr -c 'a-zA-Z0-9_\n' _)" 600 $PYT "${s#tests:}" -m gpu || exit 1 ;;
    smoke) run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench:*) run "bench_${s#bench:}" 300 python bench.py --config ${s#bench:} --steps 20 --warmup 5 --no-cpu || exit 1 ;;
    hostlat) run hostlat 400 python tools/hostlat.py --lens 64,1500 --modes lowlat,zerocopy --batches 64,1024 --reps 300 || exit 1 ;;
    rxring) run rxring 400 python tools/rxring_runs.py || exit 1 ;;
    rxdiag) run rxdiag 400 python tools/rxring_runs.py --diag || exit 1 ;;
    probe) run probe 400 python tools/migrate_probe.py --seconds 10 || exit 1 ;;
    devptr) run devptr 120 python tools/migrate_probe.py --probes devptr || exit 1 ;;
    spread) run spread 300 python tools/wg_spread.py --config c3 --variants 10 --rounds 3 || exit 1 ;;
    overlap) run overlap 300 python tools/overlap.py --config c3 --steps 20 --streams 1,2,3 || exit 1 ;;
    readbw) run readbw 400 python tools/readbw.py || exit 1 ;;
    overlapprof) run overlapprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/overlapprof -o run -- python3 $GRAFT_REPO_ROOT/tools/overlap.py --config c3 --steps 20 --streams 1,2 --reps 2 || exit 1 ;;
    prof:*) c=${s#prof:}; run prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 20 --warmup 5 --no-cpu || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
