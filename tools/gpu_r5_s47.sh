#!/bin/bash
# Round 5 experiment: more LOWLAT channels per process.  tools/_lib_c is the library and rxring built with
# XSK_GPU_LOWLAT_PER_DEVICE 8 and XSK_GPU_RX_PIPE_MAX 8; the slot cap is min(that, GPU_MAX_HW_QUEUES), so under the
# box's GPU_MAX_HW_QUEUES=4 a depth-8 pipe runs 4 LOWLAT + 4 ZEROCOPY contexts, under GPU_MAX_HW_QUEUES=8 eight LOWLAT.
set -o pipefail
O=gpurun_out/s47
mkdir -p $O
R="len=64 huge=1 ring=16384 frames=16384 nic=burst"
X=tools/_lib_c/rxring
run() { local q=$1; shift
  env GPU_MAX_HW_QUEUES=$q timeout -k 10 60 $X "$@" $R | sed "s/^{/{\"hw_queues\": $q, /" >> $O/q.jsonl; local rc=$?
  tail -1 $O/q.jsonl | cut -c1-330; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
run 4 64 lowlat 3 pipe=4 && run 8 64 lowlat 3 pipe=4 && run 8 64 lowlat 3 pipe=8 && run 4 64 lowlat 3 pipe=8 &&
  run 8 64 lowlat 3 pipe=6 && run 8 1024 lowlat 3 pipe=8 && run 4 1024 lowlat 3 pipe=4 && run 8 64 lowlat 3 pipe=8
