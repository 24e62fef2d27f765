"""Tabulate the misdirected-write reports of round 5.

Each failing GPU test printed `describe_diff` entries: frame i at address a, the offsets that differ, and the bytes
got / want / request at the first 12 of them.  The tests' inputs are seeded, so this script regenerates each test's
request image and the oracle's reply image and, for every reported frame, finds which frame's reply (or request) the
bytes that landed there belong to: the delta from the source frame's address to the landing address, in bytes, pages
and frames, and whether the in-page offset is preserved.

usage: python tools/diff_table.py gpurun_out/s22/run1.log ... (logs are scratch; the table is in DESIGN.md)
"""
import re
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import oracle  # noqa: E402  -- test infrastructure: regenerates the inputs the failing tests used

# the failing tests' inputs (tests/test_gpu_staged.py at round 5's head)
DATASETS = {
    "test_lowlat_reserved_queue_for_an_application_stream":
        [dict(n=512, base=256, stride=4096, seed=0x5EED5050 + q, mode=1, lo=20, hi=1500, size=512 * 4096)
         for q in range(4)],
    "test_multi_lowlat_with_downgraded_contexts":
        [dict(n=2560, base=0, stride=2048, seed=0x5EED5151, mode=1, lo=20, hi=1500, size=2560 * 2048)],
    "test_lowlat_timeout_exactly_once":
        [dict(n=1024, base=0, stride=2048, seed=0x5EED4F4F, mode=0, lo=1500, hi=1500, size=1024 * 2048)],
}

ENTRY = re.compile(r"frame (\d+) @(\d+) len (\d+) verdict (\d+): offsets \[([^\]]*)\] got \[([^\]]*)\] "
                   r"want \[([^\]]*)\] request \[([^\]]*)\]")


def ints(s):
    return [int(x) for x in s.split(",") if x.strip()]


def images(ds):
    umem = np.zeros(ds["size"], np.uint8)
    descs = oracle.synth_batch(umem, ds["n"], ds["base"], ds["stride"], ds["seed"], mode=ds["mode"],
                               len_lo=ds["lo"], len_hi=ds["hi"])
    ref = umem.copy()
    oracle.echo_batch(ref, descs)
    return umem, ref, descs


def main(paths):
    cache = {}
    for p in paths:
        text = Path(p).read_text(errors="replace")
        test = next((t for t in DATASETS if f"def {t}" in text), None)
        if test is None:
            print(f"{p}: no known failing test")
            continue
        for line in text.splitlines():
            entries = ENTRY.findall(line)
            if not entries:
                continue
            # which of the test's datasets: the one whose reply image has the reported `want` bytes
            for k, ds in enumerate(DATASETS[test]):
                if (test, k) not in cache:
                    cache[(test, k)] = images(ds)
                req, ref, descs = cache[(test, k)]
                e = entries[0]
                a, offs, want = int(e[1]), ints(e[4])[:12], ints(e[6])
                if [int(x) for x in ref[a + np.array(offs)]] == want:
                    break
            else:
                print(f"{p}: no dataset matches")
                continue
            addr = descs["addr"].astype(np.int64)
            print(f"{p} ({test}, dataset {k})")
            for e in entries:
                i, a, ln, v = int(e[0]), int(e[1]), int(e[2]), int(e[3])
                offs = np.array(ints(e[4])[:12])
                got = ints(e[5])
                src = []
                for img, what in ((ref, "reply"), (req, "request")):
                    for j in range(len(descs)):
                        b = int(addr[j]) - int(addr[i]) + a  # frame j at the same in-frame offsets
                        if b + offs.max() < len(img) and [int(x) for x in img[b + offs]] == got and j != i:
                            src.append((what, j, int(addr[j])))
                if [int(x) for x in req[a + offs]] == got:
                    kind = "untouched (holds its request)"
                elif [int(x) for x in ref[a + offs]] == got:
                    kind = "exact"
                elif src:
                    kind = "; ".join(f"{w} of frame {j} @{aj}: delta {a - aj:+d} B = {(a - aj) / 4096:+g} pages = "
                                     f"{i - j:+d} frames, page offset {'kept' if (a - aj) % 4096 == 0 else 'moved'}"
                                     for w, j, aj in src[:2])
                else:
                    kind = "unmatched"
                print(f"  frame {i:5d} @{a:8d} (page {a // 4096}, +{a % 4096}) len {ln:4d} verdict {v}: {kind}")


if __name__ == "__main__":
    main(sys.argv[1:])
