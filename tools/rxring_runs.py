"""Rerun every round-5 tools/rxring configuration that reported failures, with the failure accounting split by cause
(VERDICT r05 weak #6 / next #3): TX-ring-full drops against wrong verdicts, wrong replies and counter mismatches.

Round 5's `failures` counted a reply the step dropped because the TX ring was full like a wrong result.  The
configurations below are the ones with a nonzero count in profiles/r05/rxpipe_nicthread.jsonl (the NIC in a thread of
its own, a 4096-entry ring over 16384 frames) and rxpipe_pages.jsonl (burst timing on huge pages); each runs again here
and prints its rxring JSON line with the round-5 count beside it.

    python tools/rxring_runs.py [--seconds 2] > profiles/r06/rxring_attributed.jsonl
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (mode, step, len, pipe, extra args, round-5 Mframes/s, round-5 failures)
RUNS = [
    ("lowlat", 64, 64, 2, [], 12.41, 385),
    ("lowlat", 64, 64, 4, [], 27.82, 1409),
    ("lowlat", 256, 64, 1, [], 18.868, 5377),
    ("lowlat", 256, 64, 3, [], 33.535, 2325505),
    ("lowlat", 256, 64, 4, [], 32.21, 9123329),
    ("lowlat", 1024, 64, 1, [], 33.72, 103425),
    ("lowlat", 1024, 64, 2, [], 31.538, 15369217),
    ("lowlat", 1024, 64, 3, [], 35.342, 29737985),
    ("lowlat", 1024, 64, 4, [], 53.6, 50913546),
    ("lowlat", 256, 1500, 3, [], 24.223, 1793),
    ("lowlat", 1024, 1500, 3, [], 27.354, 1025),
    ("lowlat", 1024, 1500, 4, [], 24.214, 1186602),
    ("zerocopy", 64, 64, 4, [], 9.897, 193),
    ("lowlat", 1024, 64, 0, ["ring=16384", "nic=burst", "huge=1"], 73.26, 257),
]


# round 6: the runs that still failed with the split accounting (1024 x 1500-B steps, pipe depth 3-4, NIC thread),
# and the variants that tell where the failures come from
DIAG = [
    ("lowlat", 1024, 1500, 3, [], None, None),
    ("lowlat", 1024, 1500, 3, ["ring=4096", "groups=1"], None, None),
    ("lowlat", 1024, 1500, 3, ["ring=4096", "huge=1"], None, None),
    ("lowlat", 1024, 1500, 2, [], None, None),
    ("lowlat", 1024, 1500, 0, [], None, None),
    ("lowlat", 1024, 1500, 0, ["ring=4096", "queues=3"], None, None),
    ("zerocopy", 1024, 1500, 3, [], None, None),
    ("staged", 1024, 1500, 3, [], None, None),
    ("lowlat", 1024, 1500, 3, ["ring=16384", "nic=burst"], None, None),
    ("lowlat", 512, 1500, 3, [], None, None),
    ("lowlat", 1024, 512, 3, [], None, None),
    ("lowlat", 1024, 1500, 4, [], None, None),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--diag", action="store_true", help="the round-6 diagnosis variants instead of the round-5 runs")
    args = ap.parse_args()
    exe = os.path.join(ROOT, "tools", "rxring")
    bad = 0
    for mode, step, ln, pipe, extra, r5_rate, r5_fail in (DIAG if args.diag else RUNS):
        cmd = [exe, str(step), mode, str(args.seconds), f"len={ln}", "frames=16384", f"pipe={pipe}"] + \
            (extra or ["ring=4096"])
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
        line = p.stdout.strip().splitlines()[-1] if p.stdout.strip() else "{}"
        try:
            d = json.loads(line)
        except json.JSONDecodeError:
            d = {"raw": line[-400:], "stderr": p.stderr[-400:]}
        if r5_rate is not None:
            d["r5"] = {"mframes_s_total": r5_rate, "failures": r5_fail}
        d["cmd"] = " ".join(["tools/rxring"] + cmd[1:])
        bad += int(d.get("failures", 1) != 0)
        print(json.dumps(d), flush=True)
    print(json.dumps({"tool": "rxring_runs", "runs": len(DIAG if args.diag else RUNS),
                      "runs_with_correctness_failures": bad}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
