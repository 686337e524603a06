"""Diagnostic: the bench's state-read leg (1e8 events per step, res 7, 1-minute advance, the same points every step)
with per-step wall time and counts.  Steps 1-4 and 6-9 of a 5-minute window re-touch every key, so a correct merge
creates no state key there (state_new == 0) and emits the same tiles as the window's first step."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "real-time-mobility-heatmap_amd"))
import bench  # noqa: E402
import mobheat  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 11
dev = torch.device("cuda", 0)
data = bench.gen_batch(n, steps, seed=2, dev=dev, span_us=60_000_000, advance_us=60_000_000)
eng = mobheat.HeatmapEngine(h3_res=7, device=0, batch_capacity_hint=n)
bad = 0
first_tiles = None
for s in range(steps):
    t0 = time.perf_counter()
    eng.process_batch_device(s, n=n, lat=data["lat"].data_ptr(), lon=data["lon"].data_ptr(),
                             ts_us=data["ts"][s].data_ptr(), speed=data["speed"].data_ptr(),
                             speed_valid=data["sv"].data_ptr(), vkey=data["vkey"].data_ptr(),
                             row_valid=data["rv"].data_ptr())
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    c = eng.last_counts()
    tm = eng.last_timings()
    if s % 5 == 0:
        first_tiles = c["tiles"]
    ok = s % 5 == 0 or (c["state_new"] == 0 and c["tiles"] == first_tiles)
    bad += not ok
    print(f"step {s:2d} {ms:8.1f} ms  tiles {c['tiles']:10d}  state_new {c['state_new']:10d}  partials {c['partials']:10d} "
          f" merge {tm.get('merge', 0):.2f} ms  {'ok' if ok else 'MISMATCH'}", flush=True)
eng.close()
print("state_leg_check", "ok" if bad == 0 else f"{bad} bad steps")
sys.exit(1 if bad else 0)
