#!/usr/bin/env python3
"""Counter delivery A/B (GPU box): the fold launch (mode 0) vs per-workgroup device atomics (mode 1),
timed over the whole xsk_gpu_echo_dev call (kernel + fold) on cold pooled batches, interleaved."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import xsknet_amd as X  # noqa: E402

LAYOUTS = {"c3_s4096": (1 << 20, 1500, 1500, 4096), "c2_s64": (1 << 20, 64, 64, 64),
           "c4_s2048": (1 << 20, 64, 1500, 2048)}


def main():
    L = X.lib()
    dev = torch.device("cuda:0")
    for lname, (n, lo, hi, stride) in LAYOUTS.items():
        pool = 8
        umems = [torch.empty(n * stride, dtype=torch.uint8, device=dev) for _ in range(pool)]
        descs = [torch.empty(n * 16, dtype=torch.uint8, device=dev) for _ in range(pool)]
        for b in range(pool):
            X.synth_dev(umems[b], descs[b], n, 0, stride, 0x5EED0003, b * n, 1, 0, lo, hi)
        verds = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(pool)]
        recs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        ws = torch.zeros(X.workspace_size(0, n), dtype=torch.uint8, device=dev)
        stats = {m: torch.zeros(4, dtype=torch.int64, device=dev) for m in (0, 1)}
        times = {0: [], 1: []}
        for rep in range(9):
            for m in (0, 1):
                assert L.xsk_gpu__set_stats_atomic(m) == 0
                for b in range(pool):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    X.echo_dev(umems[b], descs[b], n, verds[b], recs, stats[m], ws)
                    e1.record()
                    if rep:
                        times[m].append((e0, e1))
                for b in range(pool):
                    X.rearm_dev(umems[b], descs[b], verds[b], n)
            torch.cuda.synchronize()
        L.xsk_gpu__set_stats_atomic(0)
        same = bool(torch.equal(stats[0], stats[1]))
        for m in (0, 1):
            ts = sorted(a.elapsed_time(b) for a, b in times[m])
            print(json.dumps({"layout": lname, "stats_mode": ["fold launch", "device atomics"][m],
                              "us_med": round(ts[len(ts) // 2] * 1e3, 2), "us_min": round(ts[0] * 1e3, 2),
                              "counters_equal": same, "counters": stats[m].tolist()}), flush=True)
        del umems, descs, verds
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
