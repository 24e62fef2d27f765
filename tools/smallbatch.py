#!/usr/bin/env python3
"""Device-resident small batches (n <= XSK_GPU_LOWLAT_MAX, UMEM in HBM): the shipped geometry -- sub-tiles on ONE
workgroup, chosen for the PCIe (zerocopy) path -- against the same sub-tiles spread over W workgroups
(xsk_gpu__echo_dev_grid), ADVICE r02.  A pool of fresh batches (2 KiB stride), each geometry launched back to
back on its own batches; per-launch HIP events; median per launch and the wall time of the whole loop.

    python tools/smallbatch.py [--ns 64,256,1024] [--lens 64,1500] [--ws 1,2,4,8,16] [--reps 200]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xsknet_amd as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="64,256,1024")
    ap.add_argument("--lens", default="64,1500")
    ap.add_argument("--ws", default="1,2,4,8,16")
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    stride = 2048
    for ln in (int(x) for x in args.lens.split(",")):
        for n in (int(x) for x in args.ns.split(",")):
            ws_list = [int(x) for x in args.ws.split(",")]
            pool = args.reps * len(ws_list)
            umem = torch.empty(pool * n * stride, dtype=torch.uint8, device=dev)
            descs = torch.empty(pool * n * 16, dtype=torch.uint8, device=dev)
            for b in range(pool):  # batch b: frames at its own UMEM offset, descriptors relative to the slab
                X.synth_dev(umem, descs[b * n * 16:(b + 1) * n * 16], n, b * n * stride, stride, 0x5EED3131 + b, 0, 1,
                            0, ln, ln)
            verd = torch.empty(n, dtype=torch.uint8, device=dev)
            stats = torch.zeros(40, dtype=torch.uint8, device=dev)
            wsp = torch.zeros(max(16, X.workspace_size(0, n)), dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            res = {}
            b = 0
            for rnd in range(2):  # round 0 warms up (on batches that are then not reused)
                for w in ws_list:
                    evs = []
                    for r in range(args.reps // 2):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(stream)
                        X.echo_dev(umem, descs[b * n * 16:(b + 1) * n * 16], n, verd, None, stats, wsp, stream, grid=w)
                        e1.record(stream)
                        evs.append((e0, e1))
                        b += 1
                    torch.cuda.synchronize()
                    if rnd:
                        ts = sorted(a.elapsed_time(c) * 1e3 for a, c in evs)
                        res[w] = {"median_us": round(ts[len(ts) // 2], 2), "min_us": round(ts[0], 2)}
            v = verd.cpu()
            assert bool((v == 0).all()), "every frame a reply"
            print(json.dumps({"frame_len": ln, "n": n, "per_workgroups": res}), flush=True)
            del umem, descs


if __name__ == "__main__":
    main()
