"""Summarise round-6 A/B bench logs: ms/step and kernel ms of both legs per log (usage: python tools/ab_r6.py logs...)"""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        print(f, "no JSON line")
        continue
    k = d["roofline"]["kernel_ms"]
    s = d.get("state_read_leg")
    line = f"{f}: {d['ms_per_step']:.2f} ms ingest {k['ingest']:.2f} merge {k['merge']:.2f}"
    if s:
        line += f" | state leg {s['ms_per_step']:.2f} ms ingest {s['kernel_ms']['ingest']:.2f} merge {s['kernel_ms']['merge']:.2f}"
    print(line)
