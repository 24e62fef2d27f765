#!/usr/bin/env python3
"""Kernel tuning sweep for the echo transform (GPU box).  One process, interleaved variants.

Times each kernel launch with HIP events on the launch stream.  Two regimes:
  --pool 1  : one batch, re-armed (untimed) after every launch -> warm TLB, headers L3-warm
  --pool K  : K distinct batches, launched back to back (each timed), re-armed after the sweep;
              with K batches >> Infinity Cache this is the bench's cold-data regime.
Variants (xsk_gpu__echo_variant): 0/1/2/3 = ring depth P 4/8/2/6, 10+x = stream-only ceiling of the
same P (LITE), 50+ = the shipped row-streaming kernel at other settings, see xsk_tune.hip.
-1 = stream_read over the slab.
Prints one JSON line per (layout, variant, grid) to stdout.
"""
import argparse
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
    "c3_s1504": (1 << 20, 1500, 1500, 1504),
    "c2_s64": (1 << 20, 64, 64, 64),
    "c4_s2048": (1 << 20, 64, 1500, 2048),
    "c4ramp_s2048": (1 << 20, 1500, 1500, 2048),  # lengths overwritten: 64..1500 ramp, the same in every tile
    "p98_s2048": (1 << 20, 98, 98, 2048),      # a default ping (56-B payload) per frame
    "m512_s2048": (1 << 20, 64, 512, 2048),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layouts", default=",".join(LAYOUTS))
    ap.add_argument("--variants", default="0,1,2,3,10,11")
    ap.add_argument("--grids", default="0")  # 0 = library default; comma list of caps, -1 = full grid
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--pool", type=int, default=1)
    ap.add_argument("--slab", action="store_true", help="the pool's batches in one allocation")
    ap.add_argument("--no-recs", action="store_true", help="pass no record buffer (records are optional)")
    args = ap.parse_args()
    L = X.tune_lib()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    for lname in args.layouts.split(","):
        n, lo, hi, stride = LAYOUTS[lname]
        free, _ = torch.cuda.mem_get_info(dev)
        pool = max(1, min(args.pool, int(free * 0.8) // (n * stride + n * 16)))
        umems, descss = [], []
        slab = torch.empty(pool * n * stride, dtype=torch.uint8, device=dev) if args.slab else None
        for b in range(pool):
            u = slab[b * n * stride:(b + 1) * n * stride] if slab is not None else \
                torch.empty(n * stride, dtype=torch.uint8, device=dev)
            d = torch.empty(n * 16, dtype=torch.uint8, device=dev)
            X.synth_dev(u, d, n, 0, stride, 0x5EED0003, b * n, 1, 0, lo, hi)
            if lname.startswith("c4ramp"):  # equal bytes per tile, ragged inside (mean 782 B)
                ramp = 64 + (torch.arange(n, device=dev) % 64) * 1436 // 63
                d.view(torch.int32).view(-1, 4)[:, 2] = ramp.to(torch.int32)
            umems.append(u)
            descss.append(d)
        nbytes = int(descss[0].view(torch.int32).view(-1, 4)[:, 2].to(torch.int64).sum().item())
        verds = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(pool)]
        recs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
        out = torch.zeros(1, dtype=torch.int64, device=dev)
        variants = [int(v) for v in args.variants.split(",")]
        grids = [int(g) for g in args.grids.split(",")]
        times = {(v, g): [] for v in variants for g in grids}
        for rep in range(args.reps):
            for v in variants:
                for g in grids:
                    maxg = 0 if g == 0 else (0xFFFFFFFF if g < 0 else g)
                    evs = []
                    for b in range(pool):
                        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        ev0.record()
                        if v == -1:
                            X.stream_read_dev(umems[b], n * stride, out)
                        else:
                            rc = L.xsk_gpu__echo_variant(v, maxg, umems[b].data_ptr(), n * stride,
                                                         descss[b].data_ptr(), n, verds[b].data_ptr(),
                                                         None if args.no_recs else recs.data_ptr(), ws.data_ptr(), sp)
                            assert rc == 0, rc
                        ev1.record()
                        evs.append((ev0, ev1))
                    if (0 <= v < 10 or v >= 20) and v not in (85, 105, 106, 109, 114, 115):  # NOWR variants write nothing: nothing to re-arm
                        for b in range(pool):
                            X.rearm_dev(umems[b], descss[b], verds[b], n)
                    if rep > 0:
                        times[(v, g)].extend(evs)
            torch.cuda.synchronize()
        for wv in [v for v in variants if v in (79, 94, 102)]:  # per-workgroup start/end wall clock (workspace tail)
            torch.cuda.synchronize()  # batch wv's launch reads is a request batch (every sweep re-arms)
            assert L.xsk_gpu__echo_variant(wv, 0, umems[0].data_ptr(), n * stride, descss[0].data_ptr(), n,
                                           verds[0].data_ptr(), recs.data_ptr(), ws.data_ptr(), sp) == 0
            torch.cuda.synchronize()
            t = ws.view(torch.int64)[8192:8192 + 2 * 256].cpu().view(256, 2).double() / 100.0  # us
            t0 = t[:, 0].min()
            st, en = t[:, 0] - t0, t[:, 1] - t0
            print(json.dumps({"layout": lname, "wg_timing": True, "variant": wv, "start_max": round(float(st.max()), 1),
                              "end_min": round(float(en.min()), 1), "end_med": round(float(en.median()), 1),
                              "end_max": round(float(en.max()), 1),
                              "end_mean_per_xcd": [round(float(en[x::8].mean()), 1) for x in range(8)],
                              "end_sorted_deciles": [round(float(en.sort().values[min(255, int(i * 25.6))]), 1)
                                                     for i in range(11)]}), flush=True)
        for (v, g), evs in times.items():
            ms = sorted(a.elapsed_time(b) for a, b in evs)
            med = ms[len(ms) // 2]
            nb = n * stride if v == -1 else nbytes
            print(json.dumps({"layout": lname, "pool": pool, "variant": v, "grid": g, "us_med": round(med * 1e3, 2),
                              "us_min": round(ms[0] * 1e3, 2), "gbs_med": round(nb / (med / 1e3) / 1e9, 1),
                              "mframes_s": round(n / (med / 1e3) / 1e6, 1)}), flush=True)
        del umems, descss, verds, recs, slab
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
