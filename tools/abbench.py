"""In-process cold A/B of kernel variants (tuning aid, not the bench).

Box-to-box and process-to-process drift (±3 % on c3) hides differences of a few microseconds between
separate `bench.py --variant` runs.  This tool times several variants inside ONE process on ONE pool of
never-touched batches: in round r, batch b runs variant V[(b + r) % len(V)], so every variant sees every
pool position; each launch is bracketed by its own pair of HIP events on the launch stream.  Between rounds
the pool is regenerated (untimed), so diagnostic variants with wrong results cannot poison the next round.
Variant -1 is the shipped entry point (xsk_gpu_echo_dev); v >= 0 is the product kernel's source at the alternative
switch v of tune/xsk_tune_product.hip (xsk_gpu__product_variant; 1000 + v is accepted too, the round-3 numbering).

    python tools/abbench.py --config c4 --variants=-1,9 --rounds 8
    python tools/abbench.py --config c3 --opts 7 --variants=-1,2,21   # wire mode: -1 is xsk_gpu_echo_dev_opts(7)
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
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--variants", default="-1,0")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--pool", type=int, default=0, help="batches in the pool (0: as many as fit, <= 24)")
    ap.add_argument("--burst", type=int, default=0,
                    help="sustained regime: each variant runs BURST consecutive launches per round (the bench's back-"
                         "to-back loop) and only the second half of each burst is counted; 0 = interleave per launch")
    ap.add_argument("--opts", type=int, default=0,
                    help="wire-format options of the shipped entry point (-1; xsk_gpu_echo_dev_opts) -- the tuning "
                         "variants carry their own (tune/xsk_tune_product.hip), so pair them accordingly")
    args = ap.parse_args()
    V = [int(v) for v in args.variants.split(",")]
    dev = torch.device("cuda", 0)
    n, lo, hi, stride, seed, desc = CONFIGS[args.config]
    bb = n * stride
    free, _ = torch.cuda.mem_get_info(dev)
    pool = args.pool or max(len(V), min(24, int(free * 0.8) // (bb + n * 16) - 1))
    pool -= pool % (len(V) * args.burst if args.burst else len(V))
    slab = torch.empty(pool * bb, dtype=torch.uint8, device=dev)
    descs = [torch.empty(n * 16, dtype=torch.uint8, device=dev) for _ in range(pool)]
    verd = torch.empty(n, dtype=torch.uint8, device=dev)
    recs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ws = torch.zeros(max(1 << 20, X.workspace_size(0, n)), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    tune = X.tune_lib() if any(v >= 0 for v in V) else None

    def regen():
        for b in range(pool):
            X.synth_dev(slab[b * bb:(b + 1) * bb], descs[b], n, 0, stride, seed + b, 0, 1, 0, lo, hi)
        torch.cuda.synchronize()

    def launch(v, b):
        u = slab[b * bb:(b + 1) * bb]
        if v < 0:
            X.echo_dev(u, descs[b], n, verd, recs, stats, ws, stream, opts=args.opts)
        else:
            rc = tune.xsk_gpu__product_variant(v % 1000, 0, u.data_ptr(), u.numel(), descs[b].data_ptr(), n,
                                               verd.data_ptr(), recs.data_ptr(), ws.data_ptr(), stream.cuda_stream)
            assert rc == 0, rc

    # warm-up: every variant once on a batch that is then regenerated
    regen()
    for i, v in enumerate(V):
        launch(v, i % pool)
    times = {v: [] for v in V}
    for r in range(args.rounds):
        regen()
        evs = []
        if args.burst:  # blocks of `burst` back-to-back launches per variant (the bench's loop), block order rotating
            half = args.burst // 2
            for blk in range(pool // args.burst):
                v = V[(blk + r) % len(V)]
                b0 = blk * args.burst
                for b in range(b0, b0 + args.burst - half):  # warms the clock state: not counted
                    launch(v, b)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for b in range(b0 + args.burst - half, b0 + args.burst):
                    launch(v, b)
                e1.record(stream)
                evs.append((v, e0, e1, half))
        else:
            for b in range(pool):
                v = V[(b + r) % len(V)]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                launch(v, b)
                e1.record(stream)
                evs.append((v, e0, e1, 1))
        torch.cuda.synchronize()
        for v, e0, e1, m in evs:  # microseconds per launch (a burst's counted half: its average)
            times[v].append(e0.elapsed_time(e1) * 1000.0 / m)
        print(json.dumps({"round": r, **{str(v): round(float(np.median(times[v][-max(1, len(evs) // len(V)):])), 2)
                                         for v in V}}), flush=True)
    # every variant's outputs against the shipped entry point's on one fresh batch: slab, verdicts, records (a variant
    # that skips a store would otherwise time faster and pass unnoticed)
    regen()
    # a batch too large for a third copy (c5's 128 GiB) is verified on its first n / 16 frames (descriptors in
    # address order, so they lie in the slab's first nv * stride bytes)
    nv = n if torch.cuda.mem_get_info(dev)[0] > bb + (1 << 30) else n // 16
    vb = nv * stride if nv < n else bb
    ref_u = slab[:vb].clone()
    ref_v = torch.full((nv,), 0xEE, dtype=torch.uint8, device=dev)
    ref_r = torch.zeros(nv * 16, dtype=torch.uint8, device=dev)
    X.echo_dev(ref_u, descs[0], nv, ref_v, ref_r, stats, ws, stream, opts=args.opts)
    verified = {}
    for v in V:
        u = slab[bb:bb + vb] if pool > 1 else slab[:vb]
        u.copy_(slab[:vb] if pool > 1 else ref_u)  # (pool of one: compare the shipped kernel with itself)
        verd.fill_(0xEE)
        recs.zero_()
        if v < 0:
            X.echo_dev(u, descs[0], nv, verd, recs, stats, ws, stream, opts=args.opts)
        else:
            rc = tune.xsk_gpu__product_variant(v % 1000, 0, u.data_ptr(), u.numel(), descs[0].data_ptr(), nv,
                                               verd.data_ptr(), recs.data_ptr(), ws.data_ptr(), stream.cuda_stream)
            assert rc == 0, rc
        torch.cuda.synchronize()
        verified[str(v)] = bool(torch.equal(u, ref_u) and torch.equal(verd[:nv], ref_v) and
                                torch.equal(recs[:nv * 16], ref_r))
    out = {"config": args.config, "opts": args.opts, "pool": pool, "verified_frames": nv, "rounds": args.rounds, "desc": desc, "outputs_equal_shipped": verified}
    for v in V:
        t = np.sort(np.array(times[v]))
        k = len(t) // 8
        out[str(v)] = {"median_us": round(float(np.median(t)), 2), "mean_us": round(float(t.mean()), 2),
                       "trim_mean_us": round(float(t[k:len(t) - k].mean()), 2), "min_us": round(float(t[0]), 2),
                       "n": int(len(t))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
