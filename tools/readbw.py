"""HBM read-rate sweep: the bench's read ceiling against other read kernels, over slab sizes, and
a least-squares fit of time = intercept + bytes / rate per kernel -- so the ceiling is stated as a rate plus a per-launch
fixed cost instead of one per-launch figure.

Kernels: `shipped` = xsk_gpu_stream_read_dev (the bench's roofline.read_ceiling_gbs); the rest are tools/readbw.hip
variants (shape 0 contiguous shares / 1 grid-stride, U loads in flight per lane, plain or nontemporal loads, workgroups
per CU x threads).  Each (kernel, size) is timed as 10 back-to-back launches between two events, best of 3.

    python tools/readbw.py [--sizes-gib 0.5,1,1.5,2,4,8] [--reps 10] > profiles/r06/readbw.jsonl
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import xsknet_amd as X  # noqa: E402

SO = os.path.join(ROOT, "tools", "libreadbw.so")

# name: (shape, U, nontemporal, workgroups per CU, threads)
VARIANTS = {
    "c1024_u4_nt": (0, 4, 1, 1, 1024),  # the shipped kernel's shape, rebuilt here
    "c1024_u8_nt": (0, 8, 1, 1, 1024),
    "c1024_u8": (0, 8, 0, 1, 1024),
    "c512x2_u8_nt": (0, 8, 1, 2, 512),
    "c256x4_u16_nt": (0, 16, 1, 4, 256),
    "c256x8_u8": (0, 8, 0, 8, 256),
    "g256x8_u8_nt": (1, 8, 1, 8, 256),
    "g256x8_u16": (1, 16, 0, 8, 256),
    "g1024x2_u4_nt": (1, 4, 1, 2, 1024),
}


def build():
    src = os.path.join(ROOT, "tools", "readbw.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", SO, src],
                       check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-gib", default="0.5,1,1.5,2,4,8")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    build()
    if args.build_only:
        return
    lib = ctypes.CDLL(SO)
    lib.readbw_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    sizes = [int(float(s) * 2**30) for s in args.sizes_gib.split(",")]
    slab = torch.randint(0, 255, (max(sizes),), dtype=torch.uint8, device=dev)
    out = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    kernels = {"shipped": None, **VARIANTS}
    fits = {}
    for name, v in kernels.items():
        pts = []
        for size in sizes:
            def launch():
                if v is None:
                    X.stream_read_dev(slab, size, out, stream)
                else:
                    shape, u, nt, wpc, thr = v
                    rc = lib.readbw_launch(slab.data_ptr(), size, out.data_ptr(), shape, u, nt, cus * wpc, thr,
                                           stream.cuda_stream)
                    assert rc == 0, rc
            launch()
            torch.cuda.synchronize()
            best = None
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.reps):
                    launch()
                e1.record(stream)
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.reps
                best = us if best is None else min(best, us)
            pts.append((size, best))
            print(json.dumps({"kernel": name, "variant": v, "gib": round(size / 2**30, 3), "us": round(best, 2),
                              "tb_s": round(size / best / 1e6, 3)}), flush=True)
        x = np.array([p[0] for p in pts], float)
        y = np.array([p[1] for p in pts], float)
        big = x >= 2**30  # the fit over >= 1 GiB (smaller reads are launch-bound)
        slope, icpt = np.polyfit(x[big], y[big], 1)
        fits[name] = {"rate_tb_s": round(1 / slope / 1e6, 3), "intercept_us": round(icpt, 1),
                      "at_1p5gib_tb_s": round(float(np.interp(1.5 * 2**30, x, x / y)) / 1e6, 3)}
    best = max(fits, key=lambda k: fits[k]["at_1p5gib_tb_s"])
    print(json.dumps({"tool": "readbw", "cus": cus, "fits": fits, "fastest_at_1p5gib": best}), flush=True)


if __name__ == "__main__":
    main()
