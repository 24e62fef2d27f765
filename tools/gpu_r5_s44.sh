#!/bin/bash
# Round 5 A/B: LOWLAT short-tile frame loads nontemporal (A, shipped) vs system-coherent volatile (B, tools/_lib_b:
# xsk_lowlat.hip built with -DXSK_LL_SYSLOAD=1).  Interleaved: the empty-ring 64 x 64-B step through rxring (every reply
# checked), hostlat's 64-frame call, and the saturated 1024-frame ring.
set -o pipefail
O=gpurun_out/s44
mkdir -p $O
B="LD_LIBRARY_PATH=$PWD/tools/_lib_b"
one() { local tag=$1; shift
  if [ "$tag" = B ]; then env LD_LIBRARY_PATH=$PWD/tools/_lib_b timeout -k 10 120 "$@"; else timeout -k 10 120 "$@"; fi; }
for k in 1 2 3; do
  for t in A B; do
    one $t tools/rxring 64 lowlat 4 empty=1 len=64 huge=1 | sed "s/^{/{\"lib\": \"$t\", /" >> $O/empty.jsonl || [ $? -eq 1 ] || exit 1
    one $t python3 tools/hostlat.py --modes lowlat --lens 64,98 --batches 64 --reps 3000 --huge | sed "s/^{/{\"lib\": \"$t\", /" >> $O/hostlat.jsonl || exit 1
    one $t tools/rxring 1024 lowlat 4 len=64 huge=1 ring=16384 frames=16384 nic=burst | sed "s/^{/{\"lib\": \"$t\", /" >> $O/burst.jsonl || [ $? -eq 1 ] || exit 1
    tail -1 $O/burst.jsonl | cut -c1-120
  done
done
python3 - <<'PY'
import json
for f in ("empty", "hostlat", "burst"):
    for l in open(f"gpurun_out/s44/{f}.jsonl"):
        d = json.loads(l)
        if f == "hostlat":
            print(f, d["lib"], d["frame_len"], d["us_per_call"], d["last_batch_gpu_us"]["wave0_in_transform"])
        else:
            q = d["per_queue"][0]
            print(f, d["lib"], q["mframes_s"], q["us_per_step"], q["p50_us"], "fail", d["failures"])
PY
