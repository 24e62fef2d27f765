#!/usr/bin/env python3
"""Per-launch kernel time over a pool of cold c3 batches in forward / reverse / forward order: tells a
batch-address effect from a time (clock/thermal) effect (tuning tool)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import xsknet_amd as X  # noqa: E402


def main():
    n, stride, pool = 1 << 20, 4096, int(sys.argv[1]) if len(sys.argv) > 1 else 20
    how = sys.argv[2] if len(sys.argv) > 2 else "separate"  # separate | big (one allocation, views)
    dev = torch.device("cuda:0")
    umems, descs = [], []
    big = torch.empty(pool * n * stride, dtype=torch.uint8, device=dev) if how == "big" else None
    for b in range(pool):
        u = big[b * n * stride:(b + 1) * n * stride] if big is not None else torch.empty(n * stride, dtype=torch.uint8, device=dev)
        d = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        X.synth_dev(u, d, n, 0, stride, 0x5EED0003, b * n, 1, 0, 1500, 1500)
        umems.append(u)
        descs.append(d)
    verds = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(pool)]
    recs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ws = torch.zeros(X.workspace_size(0, n), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    out = []
    for phase, order in (("fwd", range(pool)), ("rev", range(pool - 1, -1, -1)), ("fwd2", range(pool))):
        evs = []
        for b in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            X.echo_dev(umems[b], descs[b], n, verds[b], recs, stats, ws)
            e1.record()
            evs.append((b, e0, e1))
        torch.cuda.synchronize()
        out.append({"phase": phase, "us": [[b, round(e0.elapsed_time(e1) * 1e3, 1)] for b, e0, e1 in evs]})
        for b in range(pool):
            X.rearm_dev(umems[b], descs[b], verds[b], n)
        torch.cuda.synchronize()
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
