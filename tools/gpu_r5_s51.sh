#!/bin/bash
# Round 5: eight doorbell channels as separate RX queues (tools/rxring queues=8, 64-frame steps, one LOWLAT context per
# queue and thread) and two depth-4 pipes, under GPU_MAX_HW_QUEUES=8; then test_gpu_staged.py alone in file order (the
# s48 record mismatch came late in a whole-suite process).
set -o pipefail
O=gpurun_out/s51
mkdir -p $O
R="len=64 huge=1 nic=thread"
run() { env GPU_MAX_HW_QUEUES=8 timeout -k 10 60 tools/rxring "$@" $R >> $O/q8.jsonl; local rc=$?
  tail -1 $O/q8.jsonl | cut -c1-200; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
run 64 lowlat 3 queues=4 && run 64 lowlat 3 queues=8 && run 64 lowlat 3 queues=2 pipe=4 && run 1024 lowlat 3 queues=8 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_staged.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/staged.log 2>&1; rc=$?
tail -2 $O/staged.log; exit $rc
