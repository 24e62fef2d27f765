"""Per-workgroup end-time spread of the shipped round kernel (tuning aid, not the bench).

Runs the timing-probe variants of tune/xsk_tune_product.hip (10: shares as shipped, 11: share g ^ 1, 12:
round-interleaved shares) over a pool of never-touched batches, interleaved like tools/abbench.py, and prints per
launch: the event time, the workgroups' end-time min / mean / max and the mean end per XCC (read from the
hardware register, not assumed from the workgroup index).

    python tools/wg_spread.py --config c3 --variants 10,11,12 --rounds 2
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
    ap.add_argument("--variants", default="10,11,12")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--pool", type=int, default=12)
    args = ap.parse_args()
    V = [int(v) for v in args.variants.split(",")]
    dev = torch.device("cuda", 0)
    n, lo, hi, stride, seed, _ = CONFIGS[args.config]
    bb = n * stride
    free, _ = torch.cuda.mem_get_info(dev)
    pool = max(len(V), min(args.pool, int(free * 0.8) // (bb + n * 16) - 1))
    pool -= pool % len(V)
    slab = torch.empty(pool * bb, dtype=torch.uint8, device=dev)
    descs = [torch.empty(n * 16, dtype=torch.uint8, device=dev) for _ in range(pool)]
    verd = torch.empty(n, dtype=torch.uint8, device=dev)
    recs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    wss = [torch.zeros(1 << 20, dtype=torch.uint8, device=dev) for _ in range(pool)]
    stream = torch.cuda.current_stream(dev)
    tune = X.tune_lib()
    summary = {v: {"us": [], "end_max": [], "end_mean": [], "xcc": []} for v in V}
    for r in range(args.rounds + 1):  # round 0: warm-up
        for b in range(pool):
            X.synth_dev(slab[b * bb:(b + 1) * bb], descs[b], n, 0, stride, seed + b, 0, 1, 0, lo, hi)
        torch.cuda.synchronize()
        evs = []
        for b in range(pool):
            v = V[(b + r) % len(V)]
            u = slab[b * bb:(b + 1) * bb]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            rc = tune.xsk_gpu__product_variant(v, 0, u.data_ptr(), u.numel(), descs[b].data_ptr(), n, verd.data_ptr(),
                                               recs.data_ptr(), wss[b].data_ptr(), stream.cuda_stream)
            assert rc == 0, rc
            e1.record(stream)
            evs.append((v, b, e0, e1))
        torch.cuda.synchronize()
        if r == 0:
            continue
        for v, b, e0, e1 in evs:
            w = wss[b].view(torch.int64)[8192:8192 + 4 * 1024].cpu().numpy().reshape(-1, 4)
            w = w[w[:, 0] != 0]
            t0 = w[:, 0].min()
            end = (w[:, 1] - t0) / 100.0  # 100-MHz wall clock -> us
            xcc = w[:, 2] & 0xFFFFFFFF
            bal = v >= 20  # BAL kernels: column 3 = the static part's end, high half of column 2 = pool units run
            extra = {}
            if bal:
                st = (w[:, 3] - t0) / 100.0
                units = w[:, 2] >> 32
                extra = {"static_end_min": round(float(st.min()), 1), "static_end_mean": round(float(st.mean()), 1),
                         "static_end_max": round(float(st.max()), 1), "units_min": int(units.min()),
                         "units_mean": round(float(units.mean()), 2), "units_max": int(units.max())}
            per_xcc = [round(float(end[xcc == x].mean()), 1) for x in range(8) if (xcc == x).any()]
            us = e0.elapsed_time(e1) * 1000.0
            rec = {"variant": v, "batch": b, "us": round(us, 1), "wg": int(len(w)),
                   "start_max": round(float((w[:, 0] - t0).max() / 100.0), 2),
                   "end_min": round(float(end.min()), 1), "end_mean": round(float(end.mean()), 1),
                   "end_max": round(float(end.max()), 1), "end_per_xcc": per_xcc,
                   "wg_per_xcc": [int((xcc == x).sum()) for x in range(8)],
                   "slowest_wg": int(np.argmax(end)), "slowest_xcc": int(xcc[np.argmax(end)]), **extra}
            print(json.dumps(rec), flush=True)
            S = summary[v]
            S["us"].append(us)
            S["end_max"].append(float(end.max()))
            S["end_mean"].append(float(end.mean()))
            S["xcc"].append(per_xcc)
    out = {"config": args.config, "pool": pool}
    for v in V:
        S = summary[v]
        out[str(v)] = {"us_median": round(float(np.median(S["us"])), 1),
                       "end_max_median": round(float(np.median(S["end_max"])), 1),
                       "end_mean_median": round(float(np.median(S["end_mean"])), 1),
                       "end_per_xcc_mean": [round(float(x), 1) for x in np.mean(np.array(S["xcc"]), axis=0)]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
