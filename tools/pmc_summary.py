#!/usr/bin/env python3
"""Summarise separate rocprofv3 `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes of bench.py into the
per-launch HBM traffic of the transform kernel.

    python tools/pmc_summary.py <fetch_dir> <write_dir> <algorithmic_bytes_per_launch> <out.json> [kernel-substring]

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
reports exactly half of the bytes of a wide coalesced streaming read (128-B requests tallied at 64 B),
so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNEL = "echo_round_kernel"  # the product transform (bench.py KERNEL); echo_kernel6 for lab variants
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def short_name(full):
    """`void ns::(anonymous namespace)::k<1, true>(Args, unsigned int)` -> `k<1, true>` (bench.py's KERNEL)."""
    s = full.strip()
    if s.startswith("void "):
        s = s[5:]
    if s.endswith(")"):  # drop the argument list: the '(' that matches the final ')'
        depth = 0
        for i in range(len(s) - 1, -1, -1):
            depth += {")": 1, "(": -1}.get(s[i], 0)
            if depth == 0:
                s = s[:i]
                break
    depth, cut = 0, 0
    for i, ch in enumerate(s):  # the last '::' outside template brackets
        depth += {"<": 1, ">": -1}.get(ch, 0)
        if depth == 0 and s.startswith("::", i):
            cut = i + 2
    return s[cut:]


def per_launch(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter and KERNEL in r["Kernel_Name"]]
    names = {short_name(r["Kernel_Name"]) for r in rows}
    assert len(names) == 1, f"several transform kernels in one pass: {sorted(names)}"
    return statistics.median(float(r["Counter_Value"]) for r in rows), len(rows), names.pop()


def main():
    global KERNEL
    fetch_dir, write_dir, algo, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    if len(sys.argv) > 5:
        KERNEL = sys.argv[5]
    fk, nf, name = per_launch(fetch_dir, "FETCH_SIZE")
    wk, nw, _ = per_launch(write_dir, "WRITE_SIZE")
    read_b = fk * 1024 * 2
    write_b = wk * 1024
    import xsknet_amd  # the library the passes ran (loading it needs no GPU)
    res = {
        "kernel": name,
        "build_id": xsknet_amd.build_id(),
        "launches": {"fetch_pass": nf, "write_pass": nw},
        "fetch_size_kib_raw": fk, "write_size_kib_raw": wk,
        "read_bytes_per_launch": int(read_b), "write_bytes_per_launch": int(write_b),
        "hbm_bytes_per_launch": int(read_b + write_b),
        "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": round((read_b + write_b) / algo, 4),
        "correction": "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads), KiB x1024",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
