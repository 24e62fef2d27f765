#!/bin/bash
# Round 5: the pipelined RX loop against the plain step, application + GPU alone (rxring nic=burst: the RX ring holds a
# burst of 16384 frames, timed until every one is completed, NIC work untimed).
set -o pipefail
O=gpurun_out/s30
mkdir -p $O
R="ring=16384 frames=16384 nic=burst"
for len in 64 1500; do
  for step in 64 256 1024; do
    for d in 0 1 2 3 4; do
      timeout -k 10 60 tools/rxring $step lowlat 2 len=$len pipe=$d $R >> $O/rxpipe.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
    done
  done
done
for d in 0 2 4; do
  timeout -k 10 60 tools/rxring 64 zerocopy 2 len=64 pipe=$d $R >> $O/rxpipe.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
done
python3 - <<'PY'
import json
for l in open("gpurun_out/s30/rxpipe.jsonl"):
    d = json.loads(l)
    q = d["per_queue"][0]
    print(d["timing"], d["mode"], "len", d["len"], "step", d["step"], "pipe", d["pipe"], "Mf/s", d["mframes_s_total"],
          "us/step", q["us_per_step"], "p50", q["p50_us"], "p99", q["p99_us"], "fps", q["frames_per_step"], "mode", q["mode"],
          "checked", d["checked"], "fail", d["failures"], "rc", d["rc"])
PY
