#!/bin/bash
# Round 5: which pipelined-loop test, run first, makes the later LOWLAT tests go wrong (s19: 4 of 4 runs failed).
set -o pipefail
O=gpurun_out/s22
mkdir -p $O
T="timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread"
R=tests/test_gpu_rxloop.py
i=0
for sel in "$R::test_rx_pipe_end_to_end[2-2-64]" "$R::test_rx_pipe_end_to_end[2-4-64]" "$R::test_rx_pipe_end_to_end[2-3-1024]" \
           "$R::test_rx_pipe_end_to_end[0-3-64]" "$R::test_rx_pipe_end_to_end[1-2-256]" "$R::test_rx_pipe_partial_timeouts" \
           "$R::test_rx_pipe_end_to_end[2-1-64]" "$R"; do
  i=$((i+1))
  $T "$sel" tests/test_gpu_host.py tests/test_gpu_staged.py > $O/run$i.log 2>&1
  echo "run$i [$sel] rc=$? $(tail -1 $O/run$i.log)"
done
