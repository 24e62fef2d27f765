#!/usr/bin/env python3
"""How much of a LOWLAT RX-loop call is spent reaching frames scattered over the UMEM's pages?  (round-5 diagnosis)

Replays 4096 64-B echo requests through tools/echo_replay in 64-frame LOWLAT calls (reps=R, C timing) for three
layouts of the same frames: the C1 shape (one frame per 4 KiB chunk at the 256-B headroom: 64 pages per call), the
same on transparent huge pages (huge=1), and packed (64-B pitch: one 4 KiB page per call).  Prints one JSON line per
layout with us_per_call and the kernel's own phase trace of the last batch.

    python tools/layout_lat.py [--reps 300] [--len 64]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--len", type=int, default=64)
    args = ap.parse_args()
    exe = os.path.join(ROOT, "tools", "echo_replay")
    n = 4096
    with tempfile.TemporaryDirectory() as td:
        for name, stride, base, extra in (("c1_4k_pages", 4096, 256, []), ("c1_huge_pages", 4096, 256, ["huge=1"]),
                                          ("packed_64b", max(64, (args.len + 15) & ~15), 0, [])):
            umem = np.zeros(max(n * stride + base, 1 << 16), np.uint8)
            d = oracle.synth_batch(umem, n, base, stride, seed=0x5EEDC000, mode=0, len_lo=args.len, len_hi=args.len)
            paths = {k: os.path.join(td, f"{name}.{k}") for k in "udov"}
            umem.tofile(paths["u"])
            np.ascontiguousarray(d).tofile(paths["d"])
            r = subprocess.run([exe, paths["u"], paths["d"], paths["o"], paths["v"], "64", "lowlat", f"reps={args.reps}"]
                               + extra, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(json.dumps({"layout": name, "error": r.stderr[-300:]}))
                return 1
            kv = dict(x.split("=") for x in r.stdout.split())
            rec = {"layout": name, "frame_len": args.len, "stride": stride, "batch": 64,
                   "us_per_call": round(float(kv["us_per_call"]), 2)}
            if "trace_ns" in kv:
                t = [int(x) for x in kv["trace_ns"].split(",")]
                rec["gpu_us"] = {"poll_period": t[0] / 1e3, "acquire": t[1] / 1e3, "transform": t[2] / 1e3,
                                 "release": t[3] / 1e3, "streamed": t[5] / 1e3, "header_phase": t[6] / 1e3,
                                 "writes_issued": t[7] / 1e3, "host_doorbell_to_done": t[11] / 1e3}
            print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
