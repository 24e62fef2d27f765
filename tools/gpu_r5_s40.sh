#!/bin/bash
# Round 5: the UMEM allocator (xsk_gpu_umem_alloc, transparent huge pages) -- its GPU test, then the pipelined and
# plain RX loop on 4 KiB vs huge pages (rxring nic=burst).
set -o pipefail
O=gpurun_out/s40
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_host.py -k "huge_page" > $O/tests.log 2>&1; rc=$?
grep -E "huge-page bytes|FAILED|Error|passed|failed" $O/tests.log | cut -c1-300 | tail -8
[ $rc -eq 0 ] || exit $rc
R="ring=16384 frames=16384 nic=burst"
for huge in 0 1; do
  for len in 64 1500; do
    for step in 64 1024; do
      for d in 0 4; do
        timeout -k 10 60 tools/rxring $step lowlat 2 len=$len pipe=$d huge=$huge $R >> $O/rxpipe_pages.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
      done
    done
  done
done
python3 -c "
import json
for l in open('gpurun_out/s40/rxpipe_pages.jsonl'):
    d=json.loads(l); print('huge', d['huge'], 'len', d['len'], 'step', d['step'], 'pipe', d['pipe'], 'Mf/s', d['mframes_s_total'], 'fail', d['failures'])
"
