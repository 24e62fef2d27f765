cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r1g
mkdir -p $O
timeout -k 10 300 python tools/wexp.py 4096 0,1,4,7,8 4096 > $O/w4096.log 2>&1 || { cat $O/w4096.log; exit 1; }
cat $O/w4096.log
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
WEXP_POOL=2 timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$c -o run -- python3 $GRAFT_REPO_ROOT/tools/wexp.py 4096 0,1,4,5,8 4096 > $O/pmc_$c.log 2>&1 || exit 1
done
ls $O/pmc_*
