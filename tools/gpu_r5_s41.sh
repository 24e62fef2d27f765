#!/bin/bash
# Round 5: s40's one failing row (LOWLAT, huge-page UMEM, 1024-frame plain steps: 256 frames = one workgroup's slice
# answered DROP) -- how often, with the descriptor slots coarse-grained (tools/_lib_a: the library before) and
# fine-grained (this build)?
set -o pipefail
O=gpurun_out/s41
mkdir -p $O
R="ring=16384 frames=16384 nic=burst"
for k in 1 2 3 4 5 6; do
  LD_LIBRARY_PATH=$PWD/tools/_lib_a timeout -k 10 60 tools/rxring 1024 lowlat 2 len=64 huge=1 $R >> $O/a.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
  timeout -k 10 60 tools/rxring 1024 lowlat 2 len=64 huge=1 $R >> $O/b.jsonl 2>&1 || [ $? -eq 1 ] || exit 1
done
for f in a b; do
  python3 -c "
import json
for l in open('$O/$f.jsonl'):
    d=json.loads(l); print('$f', 'Mf/s', d['mframes_s_total'], 'frames', d['frames'], 'checked', d['checked'], 'fail', d['failures'])
"
done
