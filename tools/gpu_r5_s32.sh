#!/bin/bash
# Round 5, after the submit / complete split and the pipelined loop: the default bench line (c3 + host-inclusive legs)
# and the pipe's burst sweep at 64-B frames again (the fill-ring restock moved to the end of every step).
set -o pipefail
O=gpurun_out/s32
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 1; }
tail -c 1500 $O/bench_c3.json
R="ring=16384 frames=16384 nic=burst"
for step in 64 1024; do
  for d in 0 4; do
    timeout -k 10 60 tools/rxring $step lowlat 2 len=64 pipe=$d $R >> $O/rxpipe.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/s32/rxpipe.jsonl"):
    d = json.loads(l)
    print(d["timing"], "step", d["step"], "pipe", d["pipe"], "Mf/s", d["mframes_s_total"], "fail", d["failures"])
PY
