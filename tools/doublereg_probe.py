"""What the HIP runtime does when one host range is registered twice (round 6): hipHostRegister of the same range, of an
overlapping range and of a disjoint neighbour while the first registration is live, and xsk_gpu_init twice over one
UMEM (what several AF_XDP sockets sharing one UMEM -- XDP_SHARED_UMEM -- would do, one context per RX queue).

    python tools/doublereg_probe.py
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import xsknet_amd as X  # noqa: E402

hip = C.CDLL("libamdhip64.so")
P = C.c_void_p


def main():
    hip.hipSetDevice(0)
    out = {}
    u = X.umem_zeros(16 << 20)
    base, n = u.ctypes.data, u.nbytes
    reg = lambda b, s, f=2: int(hip.hipHostRegister(P(b), C.c_size_t(s), f))  # noqa: E731
    unreg = lambda b: int(hip.hipHostUnregister(P(b)))  # noqa: E731
    out["first"] = reg(base, n)
    out["same range again"] = reg(base, n)
    out["same range, portable|mapped"] = reg(base, n, 3)
    out["second half"] = reg(base + n // 2, n // 2)
    out["first half"] = reg(base, n // 2)
    out["unregister base"] = unreg(base)
    out["unregister base again"] = unreg(base)
    out["unregister mid"] = unreg(base + n // 2)
    out["halves: register first half"] = reg(base, n // 2)
    out["halves: register second half"] = reg(base + n // 2, n // 2)
    out["halves: whole range"] = reg(base, n)
    out["halves: unregister first"] = unreg(base)
    out["halves: unregister second"] = unreg(base + n // 2)

    class Attr(C.Structure):
        _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p), ("hostPointer", C.c_void_p),
                    ("isManaged", C.c_int), ("allocationFlags", C.c_uint)]

    def attr(b):
        a = Attr()
        rc = int(hip.hipPointerGetAttributes(C.byref(a), P(b)))
        hip.hipGetLastError()
        return {"rc": rc, "type": a.type, "dev_ptr_is_host": a.devicePointer == b}
    out["attributes: unregistered"] = attr(base)
    reg(base, n)
    out["attributes: registered"] = attr(base)
    out["attributes: registered, mid-range"] = attr(base + n // 2)
    unreg(base)
    out["attributes: after unregister"] = attr(base)
    print(json.dumps({"case": "hipHostRegister", **out}), flush=True)
    hip.hipGetLastError()  # (the deliberate 713 above would otherwise be the next launch check's "error")
    res = {}
    for m in (X.MODE_ZEROCOPY, X.MODE_STAGED, X.MODE_LOWLAT):
        a = X.EchoContext(u, 0, max_batch=64, mode=m)
        try:
            b = X.EchoContext(u, 0, max_batch=64, mode=m)
            res[f"mode{m}"] = "second init ok"
            b.close()
        except X.XskGpuError as e:
            res[f"mode{m}"] = str(e)
        a.close()
    print(json.dumps({"case": "xsk_gpu_init twice over one UMEM", **res}), flush=True)
    if "--after-close" in sys.argv:
        after_close(u)
    if "--unregistered-under" in sys.argv:
        unregistered_under(u)


def after_close(u):
    """Context A and context B over the same UMEM; B closes; A serves batches: exact?  (one GPU process, once)"""
    import numpy as np
    import oracle
    umem = np.zeros(u.nbytes, np.uint8)
    descs = oracle.synth_batch(umem, 2048, 0, 4096, 0x5EEDD0B1, mode=1, len_lo=20, len_hi=1500)
    ref = umem.copy()
    v_ref, _, _ = oracle.echo_batch(ref, descs)
    for m in (X.MODE_ZEROCOPY, X.MODE_STAGED, X.MODE_LOWLAT):
        r = {}
        u[:] = umem
        a = X.EchoContext(u, 0, max_batch=2048, mode=m)
        b = X.EchoContext(u, 0, max_batch=2048, mode=m)
        b.close()
        try:
            v, _, _ = a.process(descs, want_recs=False)
            r["verdicts_exact"] = bool((v == v_ref).all())
            r["bytes_exact"] = bool((u == ref).all())
            bad = np.nonzero((u != ref).reshape(-1, 4096).any(axis=1))[0]
            r["wrong_frames"] = int(len(bad))
            r["first_wrong"] = bad[:8].tolist()
        except X.XskGpuError as e:
            r["error"] = str(e)
        a.close()
        print(json.dumps({"case": f"mode{m}: A and B over one UMEM, B closed, A serves 2048 frames", **r}), flush=True)



def unregistered_under(u):
    """What round 5's library did after the second of two contexts over one UMEM closed: the runtime registration gone
    (one raw hipHostUnregister) under a live context, which then serves 2048 frames.  Every verdict and frame against
    the oracle; a wrong frame is matched against the other frames' replies."""
    import numpy as np
    import oracle
    umem = np.zeros(u.nbytes, np.uint8)
    descs = oracle.synth_batch(umem, 2048, 0, 4096, 0x5EEDD0B2, mode=1, len_lo=20, len_hi=1500)
    ref = umem.copy()
    v_ref, _, _ = oracle.echo_batch(ref, descs)
    for m in (X.MODE_ZEROCOPY, X.MODE_STAGED, X.MODE_LOWLAT):
        r = {}
        u[:] = umem
        a = X.EchoContext(u, 0, max_batch=2048, mode=m)
        hip.hipGetLastError()
        r["raw_unregister"] = int(hip.hipHostUnregister(P(u.ctypes.data)))
        hip.hipGetLastError()
        try:
            v, _, _ = a.process(descs, want_recs=False)
            r["verdicts_exact"] = bool((v == v_ref).all())
            rows = (u != ref).reshape(-1, 4096).any(axis=1)
            bad = np.nonzero(rows)[0]
            r["wrong_frames"] = int(len(bad))
            r["untouched_frames"] = int(sum((u[i * 4096:(i + 1) * 4096] == umem[i * 4096:(i + 1) * 4096]).all()
                                            for i in bad))
            r["first_wrong"] = bad[:8].tolist()
        except X.XskGpuError as e:
            r["error"] = str(e)
        hip.hipGetLastError()
        a.close()
        hip.hipGetLastError()
        print(json.dumps({"case": f"mode{m}: registration removed under a live context, 2048 frames", **r}), flush=True)


if __name__ == "__main__":
    main()
