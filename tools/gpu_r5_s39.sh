#!/bin/bash
# Round 5: LOWLAT per-call latency with the UMEM on 4 KiB pages vs transparent huge pages (and whether the box gave
# them: umem_huge_kb), 64 / 1500-B frames x 64 / 1024 per call.
set -o pipefail
O=gpurun_out/s39
mkdir -p $O
timeout -k 10 300 python -u tools/hostlat.py --modes lowlat --lens 64,1500 --batches 64,1024 --reps 300 > $O/pages4k.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u tools/hostlat.py --modes lowlat --lens 64,1500 --batches 64,1024 --reps 300 --huge > $O/pages2m.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u tools/hostlat.py --modes lowlat --lens 64,1500 --batches 64,1024 --reps 300 --scramble > $O/pages4k_scr.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u tools/hostlat.py --modes lowlat --lens 64,1500 --batches 64,1024 --reps 300 --scramble --huge > $O/pages2m_scr.jsonl 2>&1 || exit 1
for f in pages4k pages2m pages4k_scr pages2m_scr; do
  python3 -c "
import json,sys
for l in open('$O/$f.jsonl'):
    d=json.loads(l); print('$f', d['frame_len'], d['batch'], d['us_per_call'], d.get('umem_huge_kb'))
"
done
