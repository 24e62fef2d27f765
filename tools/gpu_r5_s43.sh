#!/bin/bash
# Round 5: soak of the RX ring loop for the once-seen 256-frame slice answered non-REPLY (s40): ~60 s runs instead of
# 2 s ones (each ~4 G frames), with rxring now sorting any unanswered frame by what its header holds (still the
# request / the reply / other) and reporting the LOWLAT timeouts of the run.
set -o pipefail
O=gpurun_out/s43
mkdir -p $O
R="ring=16384 frames=16384 nic=burst len=64"
run() { timeout -k 10 100 tools/rxring "$@" >> $O/soak.jsonl 2>> $O/soak.err; local rc=$?
  tail -1 $O/soak.jsonl | cut -c1-400; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
run 1024 lowlat 60 huge=1 $R && run 1024 lowlat 60 huge=1 $R && run 1024 lowlat 60 huge=0 $R &&
  run 64 lowlat 60 pipe=4 huge=1 $R && run 1024 lowlat 60 pipe=4 huge=1 $R && run 1024 lowlat 60 huge=1 $R
