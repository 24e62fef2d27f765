# Round 3: does the c4 bench slow down because the shader clock drops under sustained load?  GRBM_GUI_ACTIVE
# (GPU-busy clock cycles) per launch against the launch's duration, c4 and c3, 40 back-to-back steps each.
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r3k; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/$name.log" | cut -c1-300; return $rc; }
for c in c4 c3; do
  run clk_$c 200 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/clk_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 40 --warmup 5 --no-cpu || exit 1
done
echo done
