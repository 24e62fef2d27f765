#!/bin/bash
# Round 5: the pipelined RX loop (xsk_gpu_rx_pipe_*) -- its GPU tests, the host-path suites the submit / complete split
# touches, then rxring throughput at depth 1-4.
set -o pipefail
O=gpurun_out/s17
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rxloop.py \
    tests/test_gpu_host.py tests/test_gpu_staged.py tests/test_gpu_fuzz.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for len in 64 1500; do
  for step in 64 256 1024; do
    for d in 1 2 4; do
      timeout -k 10 60 tools/rxring $step lowlat 2 len=$len pipe=$d frames=16384 >> $O/rxpipe.jsonl 2>&1 || exit 1
    done
  done
done
for d in 2 4; do
  timeout -k 10 60 tools/rxring 64 zerocopy 2 len=64 pipe=$d frames=16384 >> $O/rxpipe.jsonl 2>&1 || exit 1
done
timeout -k 10 60 tools/rxring 64 lowlat 2 len=64 pipe=4 empty=1 >> $O/rxpipe.jsonl 2>&1 || exit 1
timeout -k 10 60 tools/rxring 64 lowlat 2 len=64 empty=1 >> $O/rxpipe.jsonl 2>&1 || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/s17/rxpipe.jsonl"):
    d = json.loads(l)
    q = d["per_queue"][0]
    print(d["mode"], "len", d["len"], "step", d["step"], "pipe", d["pipe"], "empty", d["empty"], "Mf/s", d["mframes_s_total"],
          "us/step", q["us_per_step"], "p50", q["p50_us"], "mode", q["mode"], "fail", d["failures"], "rc", d["rc"])
PY
