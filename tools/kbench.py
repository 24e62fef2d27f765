#!/usr/bin/env python3
"""Kernel tuning sweep for the echo transform (GPU box).  One process, interleaved variants.

Times each kernel launch with HIP events on its own stream; the batch is re-armed (untimed) after
every launch so every timed launch sees fresh echo requests.  Variants (xsk_gpu__echo_variant):
0/1/2/3 = ring depth P 4/8/2/6, 10+x = stream-only ceiling of the same P (LITE).
Prints one JSON line per (config, variant, grid) to stdout.
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import xsknet_amd as X  # noqa: E402

LAYOUTS = {
    "c3_s4096": (1 << 20, 1500, 1500, 4096),
    "c3_s2048": (1 << 20, 1500, 1500, 2048),
    "c3_s1536": (1 << 20, 1500, 1500, 1536),
    "c2_s64": (1 << 20, 64, 64, 64),
    "c4_s2048": (1 << 20, 64, 1500, 2048),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layouts", default=",".join(LAYOUTS))
    ap.add_argument("--variants", default="0,1,2,3,10,11")
    ap.add_argument("--grids", default="0")  # 0 = library default; comma list of caps, -1 = full grid
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    L = X.lib()
    L.xsk_gpu__echo_variant.argtypes = [C.c_int, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.xsk_gpu__echo_variant.restype = C.c_int
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    for lname in args.layouts.split(","):
        n, lo, hi, stride = LAYOUTS[lname]
        umem = torch.empty(n * stride, dtype=torch.uint8, device=dev)
        descs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        X.synth_dev(umem, descs, n, 0, stride, 0x5EED0003, 0, 1, 0, lo, hi)
        nbytes = int(descs.view(torch.int32).view(-1, 4)[:, 2].to(torch.int64).sum().item())
        verd = torch.zeros(n, dtype=torch.uint8, device=dev)
        recs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
        # read ceiling over exactly this slab
        out = torch.zeros(1, dtype=torch.int64, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        X.stream_read_dev(umem, n * stride, out)
        e0.record()
        for _ in range(5):
            X.stream_read_dev(umem, n * stride, out)
        e1.record()
        torch.cuda.synchronize()
        slab_gbs = n * stride * 5 / (e0.elapsed_time(e1) / 1e3) / 1e9
        print(json.dumps({"layout": lname, "slab_read_gbs": round(slab_gbs, 1), "frame_bytes": nbytes}), flush=True)
        variants = [int(v) for v in args.variants.split(",")]
        grids = [int(g) for g in args.grids.split(",")]
        times = {(v, g): [] for v in variants for g in grids}
        for rep in range(args.reps):
            for v in variants:
                for g in grids:
                    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    maxg = 0 if g == 0 else (0xFFFFFFFF if g < 0 else g)
                    ev0.record()
                    rc = L.xsk_gpu__echo_variant(v, maxg, umem.data_ptr(), n * stride, descs.data_ptr(), n,
                                                 verd.data_ptr(), recs.data_ptr(), ws.data_ptr(), sp)
                    ev1.record()
                    assert rc == 0, rc
                    if v < 10:
                        X.rearm_dev(umem, descs, verd, n)
                    times[(v, g)].append((ev0, ev1))
            torch.cuda.synchronize()
        for (v, g), evs in times.items():
            ms = sorted(a.elapsed_time(b) for a, b in evs[1:])  # drop the first (cold) rep
            med = ms[len(ms) // 2]
            print(json.dumps({"layout": lname, "variant": v, "grid": g, "us_med": round(med * 1e3, 2),
                              "us_min": round(ms[0] * 1e3, 2), "gbs_med": round(nbytes / (med / 1e3) / 1e9, 1),
                              "mframes_s": round(n / (med / 1e3) / 1e6, 1)}), flush=True)
        del umem, descs, verd, recs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
