#!/bin/bash
# Round 5 experiment: sixteen doorbell channels.  tools/_lib_c = library + rxring built with XSK_GPU_LOWLAT_PER_DEVICE 16
# and XSK_GPU_RX_PIPE_MAX 16; run under GPU_MAX_HW_QUEUES=16 (and 8 for the same depths, as the control).
set -o pipefail
O=gpurun_out/s52
mkdir -p $O
X=tools/_lib_c/rxring
run() { local q=$1; shift
  env GPU_MAX_HW_QUEUES=$q timeout -k 10 60 $X "$@" len=64 huge=1 | sed "s/^{/{\"hw_queues\": $q, /" >> $O/q16.jsonl; local rc=$?
  tail -1 $O/q16.jsonl | cut -c1-160; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
run 16 64 lowlat 2 pipe=16 ring=16384 frames=16384 nic=burst && run 16 64 lowlat 2 pipe=12 ring=16384 frames=16384 nic=burst &&
  run 8 64 lowlat 2 pipe=8 ring=16384 frames=16384 nic=burst && run 16 64 lowlat 2 queues=16 nic=thread &&
  run 16 64 lowlat 2 queues=2 pipe=8 nic=thread && run 16 64 lowlat 2 queues=4 pipe=4 nic=thread
python3 - <<'PY'
import json
for l in open("gpurun_out/s52/q16.jsonl"):
    d = json.loads(l)
    print(d["hw_queues"], d["step"], "queues", d["queues"], "pipe", d["pipe"], "total", d["mframes_s_total"],
          "modes", sorted(set(q["mode"] for q in d["per_queue"])), "fail", d["failures"],
          "timeouts", [q["lowlat_timeouts_all_partial_failed"] for q in d["per_queue"]][:4])
PY
