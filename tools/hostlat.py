#!/usr/bin/env python3
"""Per-call latency of the host-UMEM drop-in at RX-loop batch sizes, timed in C (tools/echo_replay reps=R).

The C1 shape: 4096 frames in a 16 MiB UMEM of 4 KiB chunks at a 256-B headroom (xsk_utils.h:6-7), processed
in batches of 64 (RX_BATCH_SIZE, xsk_utils.h:8) up to 4096 frames, for the zerocopy, staged and low-latency
(resident polling kernel) modes, and the multi-context path (``--gpus 0,0``).  Each timed pass restores the
UMEM (untimed) so every call transforms echo requests.  Prints one JSON line per (frame length, mode, batch).

  python tools/hostlat.py [--lens 64,1500] [--modes zerocopy,staged,lowlat] [--batches 64,256,1024,4096] [--opts 7]
                          [--gpus 0,0] [--reps 200] [--scramble]

--scramble puts the descriptors in a random order over the UMEM's chunks: the RX ring of a client after its free stack
(xsk_receive.c:55-71) has recycled frames in arbitrary order, so a batch's frames scatter over the 16 MiB.
"""
import argparse
import itertools
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import oracle  # noqa: E402  (frame generator only)


def run_one(exe, p, flen, mode, batch, tile, args):
    cmd = [exe, p("u"), p("d"), p("o"), p("v"), str(batch), mode, f"reps={args.reps}"] + (["flush=1"] if args.flush else []) + \
        (["huge=1"] if args.huge else [])
    if args.gpus:
        cmd.insert(7, f"gpus={args.gpus}")
    if tile:
        cmd.append(f"tile={tile}")
    if args.groups:
        cmd.append(f"groups={args.groups}")
    if args.opts:
        cmd.append(f"opts={args.opts}")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print(json.dumps({"frame_len": flen, "mode": mode, "batch": batch, "error": r.stderr[-300:]}))
        sys.exit(1)
    kv = dict(x.split("=") for x in r.stdout.split())
    us = float(kv["us_per_call"])
    rec = {"frame_len": flen, "mode": mode, "batch": batch, "gpus": args.gpus or "0", "tile": tile or "auto", "groups": args.groups or "auto",
           "opts": args.opts, "umem_flushed": bool(args.flush), "umem_huge_pages": bool(args.huge), "scrambled": bool(args.scramble),
           "us_per_call": round(us, 2), "mframes_s": round(batch / us, 3), "calls": int(kv["calls"])}
    if "huge_kb" in kv:  # the UMEM's AnonHugePages: whether the kernel backed it with 2 MiB pages
        rec["umem_huge_kb"] = int(kv["huge_kb"])
    if "trace_ns" in kv:  # LOWLAT: the last batch's phases on the GPU
        t = [int(x) for x in kv["trace_ns"].split(",")]
        rec["last_batch_gpu_us"] = {
            "poll_period": t[0] / 1e3, "acquire": t[1] / 1e3, "transform": t[2] / 1e3, "release": t[3] / 1e3,
            "wave0_in_transform": {"descriptors": t[4] / 1e3, "streamed": t[5] / 1e3, "header_phase": t[6] / 1e3,
                                   "writes_issued": t[7] / 1e3, "counters": t[8] / 1e3},
            "shader_clock_mhz": t[9], "host_before_doorbell": t[10] / 1e3, "host_doorbell_to_done": t[11] / 1e3}
        if len(t) >= 15 and t[12]:  # this kernel instance: doorbell reads per batch, stale descriptor reads
            rec["polls_per_batch"] = round(t[13] / t[12], 2)
            rec["stale_reads_per_batch"] = round(t[14] / t[12], 3)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="64,1500")
    ap.add_argument("--modes", default="zerocopy,staged,lowlat")
    ap.add_argument("--batches", default="64,256,1024,4096")
    ap.add_argument("--gpus", default="")
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--flush", action="store_true", help="evict the UMEM from the CPU caches before each pass")
    ap.add_argument("--huge", action="store_true", help="the UMEM on transparent huge pages (2 MiB)")
    ap.add_argument("--tiles", default="", help="LOWLAT frames per wave to sweep (echo_replay tile=), e.g. 4,16,64")
    ap.add_argument("--groups", type=int, default=0, help="LOWLAT serving workgroups (echo_replay groups=; 0: by size)")
    ap.add_argument("--opts", type=int, default=0, help="wire-format options (echo_replay opts=; 7 = every option)")
    ap.add_argument("--scramble", action="store_true", help="descriptors in a random order over the UMEM's chunks")
    args = ap.parse_args()
    exe = os.path.join(ROOT, "tools", "echo_replay")
    n, chunk = 4096, 4096
    with tempfile.TemporaryDirectory() as td:
        p = lambda s: os.path.join(td, s)  # noqa: E731
        for flen in (int(x) for x in args.lens.split(",")):
            umem = np.zeros(n * chunk, np.uint8)
            descs = oracle.synth_batch(umem, n, 256, chunk, seed=0x5EED0001, mode=0, len_lo=flen, len_hi=flen)
            if args.scramble:
                descs = np.ascontiguousarray(descs[np.random.default_rng(0x5C).permutation(n)])
            umem.tofile(p("u"))
            descs.tofile(p("d"))
            for mode, batch in itertools.product(args.modes.split(","), (int(x) for x in args.batches.split(","))):
                for tile in (args.tiles.split(",") if args.tiles and mode == "lowlat" else [""]):
                    rec = run_one(exe, p, flen, mode, batch, tile, args)
                    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
