#!/usr/bin/env python3
"""Plain-read ceiling over slab sizes: xsk_gpu_stream_read_dev -- one 16-wave workgroup per CU
over a contiguous share, 16-B nontemporal loads, the bench's `roofline.read_ceiling_gbs` kernel -- over prefixes of one
device allocation from 64 MiB to the c5 slab (64 M frames at a 2 KiB stride = 128 GiB), 5 timed launches each after a
warm one (HIP events), the slab written first so every page is backed.  One JSON line per size.

    python tools/slab_ceiling.py [max_gib=128]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import xsknet_amd as X  # noqa: E402


def main():
    max_gib = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    dev = torch.device("cuda:0")
    free, _ = torch.cuda.mem_get_info(dev)
    top = min(max_gib << 30, (free - (4 << 30)) & ~((1 << 30) - 1))
    slab = torch.empty(top, dtype=torch.uint8, device=dev)
    slab.view(torch.int64).fill_(0x0101010101010101)  # every page backed and written
    out = torch.zeros(1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    sizes = [64 << 20, 256 << 20, 1 << 30, 1536 << 20, 4 << 30, 16 << 30, 32 << 30, 64 << 30, 96 << 30, 128 << 30]
    for b in [x for x in sizes if x <= top]:
        X.stream_read_dev(slab, b, out, s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        e0.record(s)
        for _ in range(reps):
            X.stream_read_dev(slab, b, out, s)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(json.dumps({"slab_bytes": b, "slab_gib": round(b / 2**30, 3), "us_per_read": round(ms * 1e3, 1),
                          "read_ceiling_gbs": round(b / (ms / 1e3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
