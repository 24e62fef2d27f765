"""STAGED host-inclusive call time against the batch size (GPU box): where the host-inclusive rate of DESIGN.md §3.4
loses to the PCIe copy ceiling of tools/pcie_ceiling.py.  1500-B echo requests at a 4 KiB stride (the bench's
host-inclusive shape); for each n the median of `--reps` calls of xsk_gpu_process, each on re-armed requests.  A line
per n: ms per call, Mframes/s, and the time per chunk of 32 768 frames beyond the first.

    python tools/staged_sweep.py [--ns 32768,65536,131072,262144] [--reps 15]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402  (frame generator and re-arm only: untimed)
import xsknet_amd as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="32768,65536,131072,262144")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--len", type=int, default=1500)
    ap.add_argument("--stride", type=int, default=4096)
    a = ap.parse_args()
    ns = [int(x) for x in a.ns.split(",")]
    nmax = max(ns)
    umem = np.zeros(nmax * a.stride, np.uint8)
    descs = oracle.synth_batch(umem, nmax, 0, a.stride, 0x5EED0003, mode=0, len_lo=a.len, len_hi=a.len,
                               threads=min(16, oracle.cpu_threads()))
    prev = None
    for n in ns:
        d = np.ascontiguousarray(descs[:n])
        work = X.umem_copy(umem)  # page-aligned, as xsk_gpu_init requires
        ts = []
        with X.EchoContext(work, 0, max_batch=n, mode=X.MODE_STAGED) as ctx:
            v, _, _ = ctx.process(d, want_recs=False)  # warm
            for _ in range(a.reps):
                oracle.rearm(work, d, v)
                t0 = time.perf_counter()
                v, _, _ = ctx.process(d, want_recs=False)
                ts.append(time.perf_counter() - t0)
                assert (v == X.TX_REPLY).all()
        t = float(np.median(ts))
        line = {"n": n, "ms": round(t * 1e3, 3), "mframes_per_s": round(n / t / 1e6, 2),
                "gbs_frames": round(n * a.len / t / 1e9, 2)}
        if prev:
            line["ms_per_extra_chunk"] = round((t - prev[1]) / ((n - prev[0]) / 32768) * 1e3, 3)
        prev = (n, t)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
