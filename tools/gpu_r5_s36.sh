#!/bin/bash
# Round 5: LOWLAT 64-frame call latency by UMEM layout (scattered 4 KiB pages, huge pages, packed) -- is reaching 64
# scattered pages part of the 8.3 us?
set -o pipefail
O=gpurun_out/s36
mkdir -p $O
for len in 64 98; do
  timeout -k 10 200 python -u tools/layout_lat.py --reps 400 --len $len >> $O/layout.jsonl 2>&1 || exit 1
done
cat $O/layout.jsonl
