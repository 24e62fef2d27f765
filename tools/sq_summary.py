#!/usr/bin/env python3
"""Summarise a rocprofv3 `--pmc SQ_...` pass of bench.py: the median per launch of every counter for the
transform kernel, plus derived issue figures.

    python tools/sq_summary.py <pmc_dir> <out.json> [kernel-substring]

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_BUSY_CYCLES count quad-cycles (MI355X_MICROARCH.md, cycle constants);
SQ_INSTS_* count wave-instructions summed over the chip.
"""
import csv
import glob
import json
import os
import re
import statistics
import sys


def main():
    d, out = sys.argv[1], sys.argv[2]
    ksub = sys.argv[3] if len(sys.argv) > 3 else "echo_round_kernel"
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if ksub in r["Kernel_Name"]]
    by = {}
    for r in rows:
        by.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
        by[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    med = {c: statistics.median(v.values()) for c, v in by.items()}
    m = re.search(r"echo_\w*kernel\d*<[^>]*>", rows[0]["Kernel_Name"])
    res = {"kernel": m.group(0) if m else rows[0]["Kernel_Name"][:120],
           "launches": len(next(iter(by.values()))), "median_per_launch": med}
    if "SQ_INSTS_VALU" in med:
        # a wave64 VALU op occupies a SIMD for >= 2 cycles (SIMD-32); 1024 SIMDs at ~2.4 GHz
        res["valu_issue_us_per_simd_at_2cyc_2p4ghz"] = round(med["SQ_INSTS_VALU"] * 2 / 1024 / 2.4e3, 1)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
