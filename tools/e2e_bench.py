#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) rate of the drop-in boundary on one MI355X.

foreach_batch_func hands host buffers to hm_process_batch (HM_MEM_HOST): the library copies the batch's columns
to the device, runs the hot path, and copies the tiles and latest rows back.  This tool times that call on the
bench workload (C2-shaped, uniform sphere, res 8, 15 min per batch, advancing) with numpy inputs in pageable
memory and in page-locked memory (hipHostRegister through torch's pin_memory), beside the device-resident rate
bench.py reports.  It is the PCIe-inclusive figure DESIGN.md §7 quotes; bench.py's `value` stays device-resident.

usage: python tools/e2e_bench.py [--events 100000000] [--steps 4]   (one JSON line)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-mobility-heatmap_amd")]

import numpy as np  # noqa: E402

T0 = 1759572000 * 1_000_000
SPAN = 15 * 60_000_000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    import torch
    import mobheat
    n = a.events
    rng = np.random.default_rng(7)
    cols = dict(lat=np.degrees(np.arcsin(rng.uniform(-1, 1, n))), lon=rng.uniform(-180, 180, n),
                ts_us=T0 + rng.integers(0, SPAN, n), speed=rng.uniform(0, 80, n), speed_valid=rng.random(n) >= 0.1,
                vkey=rng.integers(0, 50_000, n).astype(np.uint64), row_valid=np.ones(n, bool))
    out = {"events_per_batch": n, "bytes_in_per_event": 42}
    for mode in ("pageable", "pinned"):
        if mode == "pinned":   # page-locked copies of the same columns
            cols = {k: torch.from_numpy(np.ascontiguousarray(v)).pin_memory().numpy() for k, v in cols.items()}
        eng = mobheat.HeatmapEngine(h3_res=8, batch_capacity_hint=n)
        ts0 = cols["ts_us"].copy()
        times, tiles = [], 0
        for s in range(a.steps + 2):
            cols["ts_us"][:] = ts0 + s * SPAN
            t = time.perf_counter()
            res = eng.process_batch(s, **cols, copy=False)
            dt = time.perf_counter() - t
            if s >= 2:
                times.append(dt)
                tiles = len(res.tiles)
        eng.close()
        ms = 1e3 * float(np.median(times))
        out[mode] = {"ms_per_batch": round(ms, 1), "events_per_s": n / (ms * 1e-3), "tiles_per_batch": tiles,
                     "bytes_out": tiles * 49 + int(res.latest_rows.size) * 8}
    out["what"] = ("hm_process_batch with host inputs and host outputs (H2D of the 42-B/event columns, the hot "
                   "path, D2H of the tiles and latest rows), median of the timed batches")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
