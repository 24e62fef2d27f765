"""Does tearing one context down wait for another context's resident LOWLAT grid?  (round 6)

tools/migrate_probe.py's churn probe made 888 contexts in 12 s beside a ZEROCOPY context and ONE beside a LOWLAT
context.  This tool times, each beside a LOWLAT context that a second thread keeps busy with 64-frame batches for
--busy-seconds (a fresh busy phase per case):
  - xsk_gpu_init / process / xsk_gpu_fini of a second context, each mode;
  - hipHostFree of pinned memory, and hipHostUnregister of a registration, that a kernel has read;
  - the HIP calls of a lifecycle on buffers no kernel has used;
and the same with no resident grid.  A call that waits for every stream of the device returns only when the busy phase
ends (`ended_beside_busy_grid`: false).  One JSON line per case.  Result (profiles/r06/fini_block.jsonl and
fini_block_steps.txt): hipFree, and hipHostFree / hipHostUnregister of memory a kernel has used, wait; so every
context's close waits (its UMEM unregistration), until the resident grid stops or idles 50 ms (its idle exit) --
unless the UMEM is shared with another context (its registration stays) and the buffers are kept for reuse while a
grid runs, as the library does since round 6: `lifecycle over its UMEM's second half`.

    python tools/fini_block.py [--busy-seconds 3]
"""
import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402  -- frames for the busy context
import xsknet_amd as X  # noqa: E402

hip = C.CDLL("libamdhip64.so")
P = C.c_void_p


def hip_calls():
    """Each HIP call of a context's lifecycle on a buffer of its own: seconds per call."""
    out = {}
    p = P()

    def t(name, fn):
        t0 = time.perf_counter()
        rc = fn()
        out[name] = {"s": round(time.perf_counter() - t0, 4), "rc": int(rc)}

    t("hipMalloc", lambda: hip.hipMalloc(C.byref(p), C.c_size_t(1 << 20)))
    t("hipFree", lambda: hip.hipFree(p))
    h = P()
    t("hipHostMalloc", lambda: hip.hipHostMalloc(C.byref(h), C.c_size_t(1 << 16), 0))
    t("hipHostFree", lambda: hip.hipHostFree(h))
    u = X.umem_zeros(1 << 20)
    t("hipHostRegister", lambda: hip.hipHostRegister(P(u.ctypes.data), C.c_size_t(u.nbytes), 2))
    t("hipHostUnregister", lambda: hip.hipHostUnregister(P(u.ctypes.data)))
    s = P()
    t("hipStreamCreate", lambda: hip.hipStreamCreateWithFlags(C.byref(s), 1))
    t("hipStreamDestroy", lambda: hip.hipStreamDestroy(s))
    e = P()
    t("hipEventCreate", lambda: hip.hipEventCreateWithFlags(C.byref(e), 2))
    t("hipEventDestroy", lambda: hip.hipEventDestroy(e))
    q = P()
    hip.hipMalloc(C.byref(q), C.c_size_t(4096))
    hb = (C.c_uint8 * 4096)()
    t("hipMemset (null stream)", lambda: hip.hipMemset(q, 0, C.c_size_t(4096)))
    t("hipMemcpy D2H (null stream)", lambda: hip.hipMemcpy(hb, q, C.c_size_t(4096), 2))
    out["note"] = "the 4-KiB buffer of the memset/memcpy rows is left allocated (its hipFree would wait)"
    return out


def used_then_released(kind):
    """A buffer a kernel has read (xsk_gpu_stream_read_dev over its mapped address), then released: seconds."""
    lib = X.lib()
    s, out = P(), P()
    hip.hipStreamCreateWithFlags(C.byref(s), 1)
    hip.hipMalloc(C.byref(out), C.c_size_t(4096))  # (left allocated: its hipFree would wait)
    n = 1 << 20
    if kind == "hipHostFree":
        h = P()
        assert hip.hipHostMalloc(C.byref(h), C.c_size_t(n), 2) == 0
        ptr, keep = h.value, None
    else:
        keep = X.umem_zeros(n)
        ptr = keep.ctypes.data
        assert hip.hipHostRegister(P(ptr), C.c_size_t(n), 2) == 0
    assert lib.xsk_gpu_stream_read_dev(P(ptr), C.c_uint64(n), out, s) == 0
    assert hip.hipStreamSynchronize(s) == 0
    t0 = time.perf_counter()
    rc = hip.hipHostFree(P(ptr)) if kind == "hipHostFree" else hip.hipHostUnregister(P(ptr))
    t1 = time.perf_counter()
    rc2 = hip.hipStreamDestroy(s)  # a stream that ran a kernel
    t2 = time.perf_counter()
    return {kind: {"s": round(t1 - t0, 4), "rc": int(rc)}, "hipStreamDestroy after a kernel": {"s": round(t2 - t1, 4),
                                                                                               "rc": int(rc2)}}


def lifecycle(mode, shared=None):
    """init / process / fini of a context over a UMEM of its own, or over the second half of `shared` (the busy
    context's UMEM: two RX queues on one UMEM)"""
    u = X.umem_zeros(256 * 2048) if shared is None else shared
    off = 0 if shared is None else shared.nbytes // 2
    d = oracle.synth_batch(u, 64, off, 2048, 0x5EEDF000 + mode, mode=1, len_lo=20, len_hi=1500)
    t0 = time.perf_counter()
    c = X.EchoContext(u, 0, max_batch=64, mode=mode)
    t1 = time.perf_counter()
    c.process(d)
    t2 = time.perf_counter()
    c.close()
    t3 = time.perf_counter()
    return {"init_s": round(t1 - t0, 4), "process_s": round(t2 - t1, 4), "fini_s": round(t3 - t2, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--busy-seconds", type=float, default=3.0)
    args = ap.parse_args()
    hip.hipSetDevice(0)
    print(json.dumps({"case": "idle device", "hip": hip_calls(),
                      **{f"mode{m}": lifecycle(m) for m in (X.MODE_ZEROCOPY, X.MODE_STAGED, X.MODE_LOWLAT)}}),
          flush=True)
    # each case beside a LOWLAT context kept busy on another thread (a fresh busy phase per case: a teardown that waits
    # for the device returns only when that phase ends, so the next case would no longer be measured beside a busy grid)
    u = X.umem_zeros(2 * 2048 * 2048)  # the busy context serves the first half
    d = oracle.synth_batch(u, 2048, 0, 2048, 0x5EEDF100, mode=1, len_lo=20, len_hi=1500)
    req = u[:u.nbytes // 2].copy()

    def beside_busy(fn):
        stop, calls, end = threading.Event(), [0], [None]

        def busy():
            with X.EchoContext(u, 0, max_batch=64, mode=X.MODE_LOWLAT) as c:
                assert c.mode == X.MODE_LOWLAT
                t_end = time.perf_counter() + args.busy_seconds
                while not stop.is_set() and time.perf_counter() < t_end:
                    u[:len(req)] = req
                    for i in range(0, len(d), 64):
                        c.process(d[i:i + 64], want_recs=False)
                        calls[0] += 1
                end[0] = time.perf_counter()

        th = threading.Thread(target=busy)
        th.start()
        time.sleep(0.5)
        r = fn()
        t_done = time.perf_counter()
        stop.set()
        th.join()
        r["ended_beside_busy_grid"] = bool(t_done < end[0])
        r["busy_calls"] = calls[0]
        return r

    for m in (X.MODE_ZEROCOPY, X.MODE_STAGED, X.MODE_LOWLAT):  # the library's own teardown ...
        print(json.dumps({"case": f"beside a busy LOWLAT context: mode{m} lifecycle", "busy_seconds": args.busy_seconds,
                          **beside_busy(lambda: lifecycle(m))}), flush=True)
    for m in (X.MODE_ZEROCOPY, X.MODE_STAGED, X.MODE_LOWLAT):  # ... over the busy context's UMEM (shared) ...
        print(json.dumps({"case": f"beside a busy LOWLAT context: mode{m} lifecycle over its UMEM's second half",
                          "busy_seconds": args.busy_seconds, **beside_busy(lambda: lifecycle(m, shared=u))}),
              flush=True)
    for kind in ("hipHostFree", "hipHostUnregister"):  # host memory a kernel has read, released
        print(json.dumps({"case": f"beside a busy LOWLAT context: {kind} of host memory a kernel read",
                          "busy_seconds": args.busy_seconds, **beside_busy(lambda: used_then_released(kind))}),
              flush=True)
    # ... then the raw calls (a raw hipFree waits here until the busy phase ends)
    print(json.dumps({"case": "beside a busy LOWLAT context: raw HIP calls", "busy_seconds": args.busy_seconds,
                      **beside_busy(lambda: {"hip": hip_calls()})}), flush=True)

if __name__ == "__main__":
    main()
