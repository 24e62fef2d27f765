#!/usr/bin/env python3
"""Wire-mode kernel A/B (GPU box): xsk_gpu__set_wire_impl 0 / 2 interleaved on cold pooled batches, every
option on; checks that both give identical outputs."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import xsknet_amd as X  # noqa: E402


def main():
    L = X.lib()
    L.xsk_gpu__set_wire_impl.argtypes = [C.c_int]
    dev = torch.device("cuda:0")
    for lname, (n, lo, hi, stride, mode) in {"c3_s4096": (1 << 20, 1500, 1500, 4096, 0),
                                            "c4_s2048": (1 << 20, 64, 1500, 2048, 0),
                                            "mixed_s2048": (1 << 20, 20, 1500, 2048, 1)}.items():
        pool = 6
        umems = [torch.empty(n * stride, dtype=torch.uint8, device=dev) for _ in range(pool)]
        descs = [torch.empty(n * 16, dtype=torch.uint8, device=dev) for _ in range(pool)]
        for b in range(pool):
            X.synth_dev(umems[b], descs[b], n, 0, stride, 0x5EED0003, b * n, 1, mode, lo, hi)
        ref = [u.clone() for u in umems[:1]]
        verds = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(pool)]
        recs = {i: torch.zeros(n * 16, dtype=torch.uint8, device=dev) for i in (0, 2)}
        ws = torch.zeros(X.workspace_size(0, n), dtype=torch.uint8, device=dev)
        stats = {i: torch.zeros(40, dtype=torch.uint8, device=dev) for i in (0, 2)}
        times = {0: [], 2: []}
        outs = {}
        for rep in range(8):
            for impl in (0, 2):
                assert L.xsk_gpu__set_wire_impl(impl) == 0
                for b in range(pool):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    X.echo_dev(umems[b], descs[b], n, verds[b], recs[impl], stats[impl], ws, opts=X.OPT_ALL)
                    e1.record()
                    if rep:
                        times[impl].append((e0, e1))
                if rep == 0:
                    torch.cuda.synchronize()
                    outs[impl] = (umems[0].clone(), verds[0].clone(), recs[impl].clone())
                for b in range(pool):  # restore the input batches (re-arm is reference-mode only)
                    if b == 0:
                        umems[0].copy_(ref[0])
                    else:
                        X.synth_dev(umems[b], descs[b], n, 0, stride, 0x5EED0003, b * n, 1, mode, lo, hi)
            torch.cuda.synchronize()
        L.xsk_gpu__set_wire_impl(0)
        same = all(torch.equal(a, b) for a, b in zip(outs[0], outs[2])) and torch.equal(stats[0], stats[2])
        for impl in (0, 2):
            ts = sorted(a.elapsed_time(b) for a, b in times[impl])
            print(json.dumps({"layout": lname, "wire_impl": impl, "us_med": round(ts[len(ts) // 2] * 1e3, 2),
                              "us_min": round(ts[0] * 1e3, 2), "outputs_identical": same}), flush=True)
        del umems, descs, verds
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
