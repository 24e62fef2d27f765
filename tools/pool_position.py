#!/usr/bin/env python3
"""Is a config's kernel time a function of where its batch sits in the pool slab, or of when it runs?
One slab of P never-touched batches (bench.py's layout); pass 1 launches batches 0 .. P-1 in order, pass 2
(after regenerating every batch) P-1 .. 0; each launch timed with its own events.  Prints both series indexed by
batch position.

    python tools/pool_position.py [--config c4] [--pool 24] [--alloc slab|separate]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xsknet_amd as X  # noqa: E402
from bench import CONFIGS  # noqa: E402
from xsknet_amd import shard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--pool", type=int, default=24)
    ap.add_argument("--alloc", default="slab", choices=("slab", "separate"))
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, lo, hi, stride, seed, _ = CONFIGS[args.config]
    bb = n * stride
    P = args.pool
    slab = torch.empty(P * bb, dtype=torch.uint8, device=dev) if args.alloc == "slab" else None
    umems = [slab[b * bb:(b + 1) * bb] if slab is not None else torch.empty(bb, dtype=torch.uint8, device=dev)
             for b in range(P)]
    descs = [torch.empty(n * 16, dtype=torch.uint8, device=dev) for _ in range(P)]
    verd = torch.empty(n, dtype=torch.uint8, device=dev)
    recs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ws = torch.zeros(X.workspace_size(0, n), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def regen():
        for b in range(P):
            first, step = shard.shard_range(b, n, 0, 1)
            X.synth_dev(umems[b], descs[b], n, 0, stride, seed, first, step, 0, lo, hi)
        torch.cuda.synchronize()

    out = {"config": args.config, "pool": P, "alloc": args.alloc}
    for name, order in (("forward", list(range(P))), ("reverse", list(range(P - 1, -1, -1))),
                        ("forward_again", list(range(P)))):
        regen()
        evs = {}
        for b in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            X.echo_dev(umems[b], descs[b], n, verd, recs, stats, ws, stream)
            e1.record(stream)
            evs[b] = (e0, e1)
        torch.cuda.synchronize()
        out[name] = [round(evs[b][0].elapsed_time(evs[b][1]) * 1e3, 1) for b in range(P)]
        print(json.dumps({"pass": name, "us_by_batch_position": out[name]}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
