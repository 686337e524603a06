#!/usr/bin/env python3
"""Split a rocprofv3 --kernel-trace of `bench.py` by leg: the bench leg's dispatches come first (warmup + timed steps
at res 8), then the state-read leg's (res 7).  The boundary is the first k_ingest dispatch after the bench leg's
steps (warmup + steps of the command line).  Prints, per leg, each kernel's calls and average duration.

usage: python tools/kernel_stats_by_leg.py <run_kernel_trace.csv> <bench-leg steps incl. warmup>
"""
import csv
import re
import sys
from collections import defaultdict


def main(path, steps_a):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    legs = [defaultdict(list), defaultdict(list)]
    ingests = 0
    leg = 0
    for r in rows:
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        base = re.sub(r"<.*", "", name)   # (k_ingest<true> / <false>: one kernel for the leg boundary)
        if base == "k_ingest":
            ingests += 1
            if ingests == steps_a + 1:
                leg = 1
        legs[leg][name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    for i, d in enumerate(legs):
        print(f"== leg {'A (bench, res 8)' if i == 0 else 'B (state-read, res 7)'}")
        for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:14]:
            print(f"  {k:40s} calls {len(v):3d}  avg {sum(v) / len(v):8.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
