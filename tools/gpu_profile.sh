# Profile one bench config on the GPU box (run through gpurun): the rocprofv3 kernel-trace summary, the
# FETCH_SIZE / WRITE_SIZE passes (-> traffic_<cfg>.json, tools/pmc_summary.py) and one SQ pass
# (-> sq_<cfg>.json, tools/sq_summary.py), every pass its own process under its own time limit.
#   bash tools/gpu_profile.sh <out-dir> <config> <algorithmic-bytes-per-launch> [extra bench args]
cd "$GRAFT_REPO_ROOT" || exit 3
export TMPDIR=/tmp
O=$1; C=$2; A=$3; shift 3
mkdir -p $O
B="python3 $GRAFT_REPO_ROOT/bench.py --config $C --steps 10 --warmup 2 --no-cpu $*"
SQ="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_WAVE_CYCLES"
run() { local name=$1 to=$2; shift 2
  echo "== $C $name $(date +%T)"; timeout -k 10 "$to" "$@" > "$O/${C}_$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -1 "$O/${C}_$name.log"; return $rc; }
run stats 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/${C}_stats -o run -- $B || exit 1
run fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/${C}_fetch -o run -- $B || exit 1
run write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/${C}_write -o run -- $B || exit 1
run sq 240 rocprofv3 --pmc $SQ --output-format csv -d $GRAFT_REPO_ROOT/$O/${C}_sq -o run -- $B || exit 1
run traffic 60 python3 tools/pmc_summary.py $O/${C}_fetch $O/${C}_write $A $O/traffic_$C.json || exit 1
run sqsum 60 python3 tools/sq_summary.py $O/${C}_sq $O/sq_$C.json || exit 1
