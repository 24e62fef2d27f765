"""Diagnose a LOWLAT mismatch: run test_lowlat_mixed_batches' workload R times and, for every frame whose
verdict / record / bytes differ from the oracle, print what came back (stale verdict of the previous
call? frame untouched? frame rewritten?).  GPU box only:  python tools/lowlat_race.py [batch] [reps]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
import xsknet_amd as X  # noqa: E402


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n = 5000
    umem = np.zeros(n * 2048 + 4096, np.uint8)
    descs = oracle.synth_batch(umem, n, 256, 2048, seed=0x5EED1C1C + batch, mode=1, len_lo=20, len_hi=1900)
    ref = umem.copy()
    v_ref, r_ref, _ = oracle.echo_batch(ref, descs)
    bad_total = 0
    for rep in range(reps):
        for want in (True, False):
            work = X.umem_copy(umem)  # page-aligned, as xsk_gpu_init requires
            vs, rs = [], []
            with X.EchoContext(work, 0, max_batch=batch, mode=X.MODE_LOWLAT) as ctx:
                for i in range(0, n, batch):
                    v, r, _ = ctx.process(descs[i:i + batch], want_recs=want)
                    vs.append(v)
                    rs.append(r)
            v = np.concatenate(vs)
            bad = np.nonzero(v != v_ref)[0]
            if want:
                r = np.concatenate(rs)
                bad = np.union1d(bad, np.nonzero(r != r_ref)[0])
            for i in bad[:16]:
                a, ln = int(descs[i]["addr"]), int(descs[i]["len"])
                hi = min(a + max(ln, 64), len(umem))
                fr_ok = bool((work[a:hi] == ref[a:hi]).all())
                fr_orig = bool((work[a:hi] == umem[a:hi]).all())
                out = {"rep": rep, "recs": want, "i": int(i), "got_v": int(v[i]), "ref_v": int(v_ref[i]),
                       "prev_ref_v": int(v_ref[i - 1]) if i else None, "frame_as_ref": fr_ok,
                       "frame_untouched": fr_orig}
                if want:
                    out["got_r"] = [int(x) for x in r[i].tolist()]
                    out["ref_r"] = [int(x) for x in r_ref[i].tolist()]
                    out["prev_ref_r"] = [int(x) for x in r_ref[i - 1].tolist()] if i else None
                print(json.dumps(out), flush=True)
            diff = np.nonzero(work != ref)[0]
            print(json.dumps({"rep": rep, "recs": want, "bad_frames": int(len(bad)), "bytes_differ": int(len(diff))}),
                  flush=True)
            bad_total += len(bad) + len(diff)
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
