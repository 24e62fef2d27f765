"""Does a GPU translation of a host UMEM page outlive the page's registration?  (round 6)

tools/doublereg_probe.py showed that the HIP runtime keeps one registration per base and counts nothing (a second
hipHostRegister of a base succeeds, the first hipHostUnregister removes it for every user), and that a context whose
registration was removed that way still serves its next batch exactly: the GPU keeps its translation.  A registered
pageable UMEM is tracked through the MMU notifier (HMM): when the kernel moves a page, the GPU's translation follows
(tools/migrate_probe.py: 5.1 M page moves, 0 wrong).  This probe asks what happens to the translation of an
UNREGISTERED range that a context still uses when its pages move:

  arm "registered"    the context's registration in place, the UMEM's pages moved to the other NUMA node
  arm "unreg_stay"    registration removed under the context (one raw hipHostUnregister), pages not moved
  arm "unreg_moved"   registration removed, pages moved

Safety: the GPU never writes through a translation that may be stale.  The UMEM first holds requests whose ICMP type
is 13 (not an echo request: verdict DROP_NOT_ECHO, the transform writes nothing) and the context serves them once, so the
GPU has translated every page.  Then the arm's action, then the CPU rewrites every frame as an echo request (type 8) in
the pages it now has, and the context serves the batch again.  A fresh translation answers TX_REPLY for every frame
(and rewrites it); a stale one reads the old pages -- type 13 -- and answers DROP_NOT_ECHO, writing nothing.

    python tools/stale_probe.py [--modes 0,1,2] [--arms registered,unreg_stay,unreg_moved]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402  -- the checker
import xsknet_amd as X  # noqa: E402
from tools.migrate_probe import PAGE, as_array, libc, mmap_aligned, move_pages, numa_nodes  # noqa: E402

hip = C.CDLL("libamdhip64.so")
MADV_NOHUGEPAGE = 15
TYPE_OFF = 14 + 20  # ICMP type byte of a frame with a 20-B IPv4 header


def node_of(p, size):
    """The NUMA node of each page (move_pages with nodes=NULL queries)."""
    n = size // PAGE
    pages = (C.c_void_p * n)(*[p + i * PAGE for i in range(n)])
    status = (C.c_int * n)()
    libc.syscall(279, 0, C.c_ulong(n), pages, None, status, 0)
    return np.array(list(status))


def run(mode, arm, nframes=1024, stride=4096):
    size = nframes * stride
    raw, p = mmap_aligned(size)
    libc.madvise(p, size, MADV_NOHUGEPAGE)
    u = as_array(p, size)
    u[:] = 0
    req = np.zeros(size, np.uint8)
    descs = oracle.synth_batch(req, nframes, 0, stride, 0x5EED57A1 + mode, mode=0, len_lo=64, len_hi=1500)
    ref = req.copy()
    v_ref, _, _ = oracle.echo_batch(ref, descs)
    old = req.copy()
    addrs = descs["addr"].astype(np.int64)
    assert (old[addrs + TYPE_OFF] == 8).all()
    old[addrs + TYPE_OFF] = 13
    out = {"mode": mode, "arm": arm, "frames": nframes}
    u[:] = old
    ctx = X.EchoContext(u, 0, max_batch=nframes, mode=mode)
    try:
        v, _, _ = ctx.process(descs, want_recs=False)
        out["first_pass_all_drop"] = bool((v != X.TX_REPLY).all()) and bool((u == old).all())
        hip.hipGetLastError()
        if arm.startswith("unreg"):
            out["raw_unregister"] = int(hip.hipHostUnregister(C.c_void_p(p)))
            hip.hipGetLastError()
        if arm in ("registered", "unreg_moved"):
            before = node_of(p, size)
            nodes = numa_nodes()
            target = [n for n in nodes if n != int(np.bincount(before[before >= 0]).argmax())][:1]
            if not target:
                out["skipped"] = f"one NUMA node ({nodes})"
                return out
            rc, moved = move_pages(p, size, target[0])
            out["moved_pages"] = int(moved)
            out["pages"] = size // PAGE
        u[:] = req  # every frame an echo request again, in the pages the CPU has now
        v, _, _ = ctx.process(descs, want_recs=False)
        fresh = v == v_ref
        out["verdicts_fresh"] = int(fresh.sum())
        out["verdicts_stale_drop"] = int(((v != X.TX_REPLY) & (v_ref == X.TX_REPLY)).sum())
        rows = (u != ref).reshape(nframes, stride).any(axis=1)
        out["frames_wrong"] = int(rows.sum())
        out["frames_left_as_requests"] = int(sum((u[i * stride:(i + 1) * stride] == req[i * stride:(i + 1) * stride]).all()
                                                 for i in np.nonzero(rows)[0]))
    except X.XskGpuError as e:
        out["error"] = str(e)
    finally:
        hip.hipGetLastError()
        ctx.close()
        hip.hipGetLastError()
        libc.munmap(raw, size + (2 << 20))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="0,1,2")
    ap.add_argument("--arms", default="registered,unreg_stay,unreg_moved")
    args = ap.parse_args()
    hip.hipSetDevice(0)
    print(json.dumps({"numa_nodes": numa_nodes()}), flush=True)
    for arm in args.arms.split(","):
        for m in (int(x) for x in args.modes.split(",")):
            print(json.dumps(run(m, arm)), flush=True)


if __name__ == "__main__":
    main()
