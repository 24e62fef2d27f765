"""PCIe ceilings behind the host-inclusive rate: what the copy engines move between a pinned host
UMEM and the device at the bench's host-inclusive shape (262 144 frames of 1500 B at a 4 KiB stride), next to
`bench.py --host-inclusive`'s staged rate.

    python tools/pcie_ceiling.py [--frames 262144] [--len 1500] [--stride 4096] [--reps 5]

Prints one JSON line: GB/s of a dense H2D copy of the frame bytes, of the 2-D strided H2D copy STAGED issues for a
uniform-stride chunk (hipMemcpy2DAsync, 32 768-row chunks on two streams as the pipeline does), of the same 2-D copy
as one call, and of the D2H copy of one 64-B sector per frame (STAGED's copy-back)."""
import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

H2D, D2H = 1, 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=262144)
    ap.add_argument("--len", type=int, default=1500)
    ap.add_argument("--stride", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=32768)
    a = ap.parse_args()
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy2DAsync.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int,
                                     C.c_void_p]
    dev = torch.device("cuda", 0)
    n, L, S = a.frames, a.len, a.stride
    host = torch.empty(n * S, dtype=torch.uint8).pin_memory()
    host.fill_(0x5A)
    d_span = torch.empty(n * S, dtype=torch.uint8, device=dev)
    d_dense = torch.empty(n * L, dtype=torch.uint8, device=dev)
    h_dense = host[:n * L]
    s0 = torch.cuda.current_stream(dev)
    s1 = torch.cuda.Stream(dev)
    frame_bytes = n * L

    def timed(fn):
        best = None
        for _ in range(a.reps + 1):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s0)
            s1.wait_stream(s0)  # the second stream's chunks start after e0
            fn()
            s0.wait_stream(s1)
            e1.record(s0)
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 1e3
            best = t if best is None or t < best else best
        return best

    def dense():
        d_dense.copy_(h_dense, non_blocking=True)

    def two_d(chunked):
        rows = a.chunk if chunked else n
        for ci, r0 in enumerate(range(0, n, rows)):
            m = min(rows, n - r0)
            st = (s0 if ci % 2 == 0 else s1).cuda_stream
            rc = hip.hipMemcpy2DAsync(C.c_void_p(d_span.data_ptr() + r0 * S), S, C.c_void_p(host.data_ptr() + r0 * S),
                                      S, L, m, H2D, C.c_void_p(st))
            assert rc == 0, rc

    def back():
        rc = hip.hipMemcpy2DAsync(C.c_void_p(host.data_ptr()), S, C.c_void_p(d_span.data_ptr()), S, 64, n, D2H,
                                  C.c_void_p(s0.cuda_stream))
        assert rc == 0, rc

    s1.wait_stream(s0)
    out = {"frames": n, "len": L, "stride": S, "frame_bytes": frame_bytes}
    t = timed(dense)
    out["h2d_dense_gbs"] = round(frame_bytes / t / 1e9, 2)
    t = timed(lambda: two_d(True))
    out["h2d_2d_chunked_gbs"] = round(frame_bytes / t / 1e9, 2)
    out["h2d_2d_chunked_mframes"] = round(n / t / 1e6, 2)
    t = timed(lambda: two_d(False))
    out["h2d_2d_one_call_gbs"] = round(frame_bytes / t / 1e9, 2)
    t = timed(back)
    out["d2h_sectors_gbs"] = round(n * 64 / t / 1e9, 2)
    out["d2h_sectors_us"] = round(t * 1e6, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
