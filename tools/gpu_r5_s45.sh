#!/bin/bash
# Round 5: the default bench line with the RX-loop leg (tools/rxring in a child process).
set -o pipefail
O=gpurun_out/s45
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.log 2> $O/bench.err; rc=$?
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], json.dumps(d.get('rx_loop')))"
exit $rc
