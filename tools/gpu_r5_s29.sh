#!/bin/bash
# Round 5: the pipelined RX loop's throughput per queue (rxring pipe=D): LOWLAT 64 / 1500 B at 64-1024-frame steps and
# depth 1-4, ZEROCOPY at depth 2-4, the empty-ring latency at depth 4 against the plain step.
set -o pipefail
O=gpurun_out/s29
mkdir -p $O
for len in 64 1500; do
  for step in 64 256 1024; do
    for d in 1 2 3 4; do
      timeout -k 10 60 tools/rxring $step lowlat 2 len=$len pipe=$d frames=16384 >> $O/rxpipe.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
    done
  done
done
for d in 1 2 4; do
  timeout -k 10 60 tools/rxring 64 zerocopy 2 len=64 pipe=$d frames=16384 >> $O/rxpipe.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
done
timeout -k 10 60 tools/rxring 64 lowlat 2 len=64 pipe=4 empty=1 >> $O/rxpipe.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
timeout -k 10 60 tools/rxring 64 lowlat 2 len=64 empty=1 >> $O/rxpipe.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
timeout -k 10 60 tools/rxring 64 lowlat 2 len=64 frames=16384 >> $O/rxpipe.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
timeout -k 10 60 tools/rxring 1024 lowlat 2 len=64 frames=16384 nic=inline >> $O/rxpipe.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
timeout -k 10 60 tools/rxring 64 lowlat 2 len=64 frames=16384 nic=inline >> $O/rxpipe.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
timeout -k 10 60 tools/rxring 64 lowlat 2 len=64 queues=2 pipe=2 frames=16384 >> $O/rxpipe.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/s29/rxpipe.jsonl"):
    d = json.loads(l)
    q = d["per_queue"][0]
    print(d["timing"], d["queues"], d["mode"], "len", d["len"], "step", d["step"], "pipe", d["pipe"], "empty", d["empty"], "Mf/s", d["mframes_s_total"],
          "us/step", q["us_per_step"], "p50", q["p50_us"], "p99", q["p99_us"], "fps", q["frames_per_step"], "mode", q["mode"],
          "fail", d["failures"], "rc", d["rc"])
PY
