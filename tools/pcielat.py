#!/usr/bin/env python3
"""Drive tools/pcielat.hip: latency of one wave's reads of pinned host memory (LOWLAT diagnostics).

  hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/libpcielat.so tools/pcielat.hip
  python tools/pcielat.py
Prints one JSON line per pattern: median and min microseconds over the reps (fresh lines every rep).
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = {0: "one 8-B read", 1: "64 x 64 B at 4 KiB stride, nt loads", 2: "64 x 64 B at 4 KiB stride, plain loads",
         3: "64 x 64 B at 4 KiB stride, sc0|sc1 buffer loads", 4: "64 x 64 B contiguous (4 KiB), nt loads",
         5: "64 x 16 B contiguous (1 KiB), nt loads", 6: "16 dependent 8-B reads of one word",
         7: "16 dependent 8-B reads of 16 lines", 8: "64 x 64-B plain stores + system release fence",
         9: "64 x 64-B sc0|sc1 stores + wait for acks", 10: "system release fence alone",
         11: "64 x 64-B plain stores + wait for acks", 12: "64 x 64-B nt stores + wait for acks",
         13: "L2+L1 invalidation (buffer_inv sc0 sc1), then pattern 1", 14: "the invalidation alone"}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    L = C.CDLL(os.path.join(ROOT, "tools", "libpcielat.so"))
    L.pcielat_run.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
    hip = C.CDLL("libamdhip64.so")
    torch.cuda.init()
    size = 64 << 20
    for kind in ("hipHostMalloc", "hipHostRegister"):
        host = C.c_void_p()
        if kind == "hipHostMalloc":
            assert hip.hipHostMalloc(C.byref(host), C.c_size_t(size), C.c_uint(2)) == 0  # hipHostMallocMapped
        else:  # a page-aligned malloc'd buffer registered like a UMEM (xsk_gpu_init)
            libc = C.CDLL("libc.so.6")
            assert libc.posix_memalign(C.byref(host), C.c_size_t(4096), C.c_size_t(size)) == 0
            C.memset(host, 0, size)
            assert hip.hipHostRegister(host, C.c_size_t(size), C.c_uint(2)) == 0  # hipHostRegisterMapped
        run(L, hip, host, size, reps, kind)
        if kind == "hipHostMalloc":
            pingpong(L, hip)
        if kind == "hipHostMalloc":
            hip.hipHostFree(host)
        else:
            hip.hipHostUnregister(host)


def pingpong(L, hip):
    """Doorbell + completion floor: host posts, one wave polls and answers, host spins on the answer."""
    fl = C.c_void_p()
    assert hip.hipHostMalloc(C.byref(fl), C.c_size_t(4096), C.c_uint(2 | 0x40000000)) == 0  # mapped | coherent
    dfl = C.c_void_p()
    assert hip.hipHostGetDevicePointer(C.byref(dfl), fl, 0) == 0
    L.pcielat_pingpong.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_double)]
    names = {0: "one poll in flight, relaxed answer", 1: "answer after a system release fence",
             2: "polls alternate two lines, relaxed answer"}
    for mode in (0, 1, 2):
        ns = C.c_double()
        rc = L.pcielat_pingpong(dfl, fl, 20000, mode, C.byref(ns))
        print(json.dumps({"pingpong": names[mode], "rc": rc, "us_per_exchange": round(ns.value / 1e3, 3)}), flush=True)
    hip.hipHostFree(fl)


def run(L, hip, host, size, reps, kind):
    dptr = C.c_void_p()
    assert hip.hipHostGetDevicePointer(C.byref(dptr), host, 0) == 0
    buf = np.ctypeslib.as_array((C.c_uint8 * size).from_address(host.value))
    out = torch.zeros(2, dtype=torch.int64, device="cuda:0")
    for pat in range(15):
        ts = []
        for r in range(reps):
            off = (r * 262144) % (size - 262144)  # a fresh 256-KiB window every rep
            buf[off:off + 262144:64] += 1          # host writes: the lines are the CPU's again
            assert L.pcielat_run(C.c_void_p(dptr.value + off), pat, 4096, C.c_void_p(out.data_ptr())) == 0
            ts.append(int(out[0].item()) * 10 / 1e3)
        ts.sort()
        if pat in (6, 7):  # per read
            ts = [t / 16 for t in ts]
        print(json.dumps({"memory": kind, "pattern": pat, "what": NAMES[pat], "us_med": round(ts[len(ts) // 2], 3),
                          "us_min": round(ts[0], 3)}), flush=True)


if __name__ == "__main__":
    main()
