#!/usr/bin/env python3
"""Is the round kernel's per-XCD speed stable from launch to launch?  Runs the timing-probe variant
(79: echo_kernel6 + per-workgroup start/end wall clock) over a pool of cold c3 batches and prints the
per-XCD mean end time of every launch (workgroup g runs on XCD g % 8)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import xsknet_amd as X  # noqa: E402


def main():
    L = X.tune_lib()
    n, stride, pool = 1 << 20, 4096, 8
    dev = torch.device("cuda:0")
    umems, descs = [], []
    for b in range(pool):
        u = torch.empty(n * stride, dtype=torch.uint8, device=dev)
        d = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        X.synth_dev(u, d, n, 0, stride, 0x5EED0003, b * n, 1, 0, 1500, 1500)
        umems.append(u)
        descs.append(d)
    verd = torch.zeros(n, dtype=torch.uint8, device=dev)
    recs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    prev = None
    for rep in range(3):
        for b in range(pool):
            assert L.xsk_gpu__echo_variant(79, 0, umems[b].data_ptr(), n * stride, descs[b].data_ptr(), n,
                                           verd.data_ptr(), recs.data_ptr(), ws.data_ptr(), sp) == 0
            torch.cuda.synchronize()
            t = ws.view(torch.int64)[8192:8192 + 512].cpu().view(256, 2).double() / 100.0
            en = t[:, 1] - t[:, 0].min()
            xcd = [round(float(en[x::8].mean()), 1) for x in range(8)]
            dur = t[:, 1] - t[:, 0]
            # per-workgroup stability: correlation with the previous launch, raw and with XCD means removed
            corr = corr_res = None
            if prev is not None:
                corr = float(torch.corrcoef(torch.stack([dur, prev]))[0, 1])
                xm = torch.stack([dur[x::8].mean() for x in range(8)]).repeat(32)
                pm = torch.stack([prev[x::8].mean() for x in range(8)]).repeat(32)
                corr_res = float(torch.corrcoef(torch.stack([dur - xm, prev - pm]))[0, 1])
            prev = dur
            print(json.dumps({"rep": rep, "batch": b, "end_max": round(float(en.max()), 1),
                              "end_mean": round(float(en.mean()), 1), "xcd_mean": xcd,
                              "corr_prev": None if corr is None else round(corr, 3),
                              "corr_prev_within_xcd": None if corr_res is None else round(corr_res, 3)}), flush=True)
            X.rearm_dev(umems[b], descs[b], verd, n)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
