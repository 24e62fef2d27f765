"""Consecutive batches on one stream vs. alternating over S streams (tuning aid, not the bench).

A round-kernel launch ends ~15 us (c3) after its average workgroup and ~3 us after its last one
(tools/wg_spread.py); a second stream lets the next batch's workgroups start on the CUs the current batch has
left.  Each batch has its own outputs.  Per mode: wall time per step over K steps between synchronizes, and the
per-launch kernel duration (events around each launch on its own stream).

    python tools/overlap.py --config c3 --steps 20 --streams 1,2
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import CONFIGS  # noqa: E402
import xsknet_amd as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--streams", default="1,2")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, lo, hi, stride, seed, _ = CONFIGS[args.config]
    K = args.steps
    bb = n * stride
    free, _ = torch.cuda.mem_get_info(dev)
    pool = min(K, int(free * 0.8) // (bb + n * 16) - 1)
    slab = torch.empty(pool * bb, dtype=torch.uint8, device=dev)
    descs = [torch.empty(n * 16, dtype=torch.uint8, device=dev) for _ in range(pool)]
    verds = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(pool)]
    recs = [torch.empty(n * 16, dtype=torch.uint8, device=dev) for _ in range(pool)]
    stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    wss = [torch.zeros(max(16, X.workspace_size(0, n)), dtype=torch.uint8, device=dev) for _ in range(pool)]
    S_list = [int(x) for x in args.streams.split(",")]
    streams = [torch.cuda.Stream(dev) for _ in range(max(S_list))]
    main_s = torch.cuda.current_stream(dev)
    out = {"config": args.config, "steps": K, "pool": pool}
    for rep in range(args.reps):
        for S in S_list:
            for b in range(pool):
                X.synth_dev(slab[b * bb:(b + 1) * bb], descs[b], n, 0, stride, seed + b, 0, 1, 0, lo, hi)
            torch.cuda.synchronize()
            evs = []
            e_start = torch.cuda.Event(enable_timing=True)
            e_start.record(main_s)
            for st in streams[:S]:
                st.wait_event(e_start)
            t0 = time.perf_counter()
            for k in range(K):
                b = k % pool
                st = streams[k % S]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                X.echo_dev(slab[b * bb:(b + 1) * bb], descs[b], n, verds[b], recs[b], stats, wss[b], st)
                e1.record(st)
                evs.append((e0, e1))
            ends = []
            for st in streams[:S]:
                e = torch.cuda.Event(enable_timing=True)
                e.record(st)
                ends.append(e)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            span = max(e_start.elapsed_time(e) for e in ends) * 1e3
            per = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in evs)
            ok = all(bool((v == 0).all().item()) for v in verds[:min(K, pool)])
            rec = {"rep": rep, "streams": S, "span_us_per_step": round(span / K, 2),
                   "wall_us_per_step": round(wall * 1e6 / K, 2),
                   "launch_us_median": round(per[len(per) // 2], 2), "launch_us_mean": round(sum(per) / len(per), 2),
                   "mframes_s": round(n * K / span, 1), "verdicts_ok": ok}
            print(json.dumps(rec), flush=True)
            out.setdefault(str(S), []).append(rec["span_us_per_step"])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
