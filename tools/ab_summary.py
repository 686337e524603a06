"""Summarises an A/B directory of bench logs (tools/gpurun/gpurun_r5ab.sh): per variant and round, ms/step, events/s
and the stage times of the JSON line."""
import glob
import json
import os
import sys

d = sys.argv[1]
rows = []
for p in sorted(glob.glob(os.path.join(d, "bench_*.log"))):
    line = [l for l in open(p) if l.startswith("{")]
    if not line:
        print(os.path.basename(p), "no JSON line")
        continue
    j = json.loads(line[-1])
    k = j["roofline"]["kernel_ms"]
    extra = ""
    if "state_read_leg" in j:
        s = j["state_read_leg"]
        extra = f"  state-leg {s['ms_per_step']:.2f} ms merge {s['kernel_ms']['merge']:.2f}"
    print(f"{os.path.basename(p):28s} {j['ms_per_step']:7.2f} ms {j['value']:.3e} ev/s  ingest {k['ingest']:.3f} "
          f"part {k['partition']:.3f} merge {k['merge']:.3f} emit {k['emit']:.3f} dedup {k['dedup']:.3f}{extra}")
