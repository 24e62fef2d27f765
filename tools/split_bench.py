"""One large device-resident batch as ONE launch of the round kernel against the same batch cut into S launches of
n / S frames (GPU box).  A share of many rounds writes every round's windows while other workgroups read; a launch of
1 M frames is two rounds, and its second round's windows go out as the launch ends.  Prints the median ms per batch
of each split over cold (re-armed) batches.

    python tools/split_bench.py [--config c5] [--frames 0] [--splits 1,8,16,32,64] [--reps 3]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS  # noqa: E402
import xsknet_amd as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=0, help="frames in the batch (0: the config's)")
    ap.add_argument("--splits", default="1,8,16,32,64")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    n0, lo, hi, stride, seed, _ = CONFIGS[a.config]
    n = a.frames or n0
    splits = [int(x) for x in a.splits.split(",")]
    dev = torch.device("cuda", 0)
    umem = torch.empty(n * stride, dtype=torch.uint8, device=dev)
    descs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    verd = torch.empty(n, dtype=torch.uint8, device=dev)
    recs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    stats = torch.zeros(32, dtype=torch.uint8, device=dev)
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    X.synth_dev(umem, descs, n, 0, stride, seed, 0, 1, 0, lo, hi)
    verd.zero_()
    torch.cuda.synchronize()
    times = {s: [] for s in splits}
    nbytes = None
    for r in range(a.reps + 1):
        for s in splits:
            X.rearm_dev(umem, descs, verd, n, stream)  # untimed: the frames are requests again (cold for the kernel)
            per = -(-n // s)
            per = (per + 63) // 64 * 64
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i0 in range(0, n, per):
                m = min(per, n - i0)
                X.echo_dev(umem, descs[i0 * 16:(i0 + m) * 16], m, verd[i0:i0 + m], recs[i0 * 16:(i0 + m) * 16], stats,
                           ws, stream)
            e1.record(stream)
            torch.cuda.synchronize()
            assert bool((verd == 0).all().item()), s
            if r:
                times[s].append(e0.elapsed_time(e1))
    if nbytes is None:
        nbytes = n * (lo + hi) // 2 if lo == hi else None
    for s in splits:
        t = float(np.median(times[s]))
        line = {"config": a.config, "frames": n, "splits": s, "frames_per_launch": -(-n // s), "ms": round(t, 3),
                "us_per_mframe": round(t * 1e3 / (n / 1e6), 2)}
        if nbytes:
            line["tbs"] = round(nbytes / (t / 1e3) / 1e12, 3)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
