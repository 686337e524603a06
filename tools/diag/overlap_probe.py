#!/usr/bin/env python3
"""Diagnostic (round 6): how much do two batches' kernels gain from running concurrently on one GPU?

Two engines (two contexts, each with its own streams and state), each fed its own bench-shaped batches from its own
host thread (ctypes releases the GIL for the call), against one engine running the same number of batches alone.  If
the aggregate throughput of the pair is well above the single engine's, a micro-batch split into chunks whose ingest
overlaps the previous chunk's merge has room to gain; if not, the kernels contend for the same
resource.  Prints one JSON line.
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-mobility-heatmap_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    n = int(os.environ.get("N", 100_000_000))
    steps = int(os.environ.get("STEPS", 8))
    warm = 3
    dev = torch.device("cuda", 0)
    import mobheat
    datas = [bench.gen_batch(n, warm + steps, seed=1 + k, dev=dev) for k in range(2)]
    engs = [mobheat.HeatmapEngine(h3_res=8, device=0, batch_capacity_hint=n) for _ in range(2)]

    def step(k, s):
        d = datas[k]
        engs[k].process_batch_device(s, n=n, lat=d["lat"].data_ptr(), lon=d["lon"].data_ptr(),
                                     ts_us=d["ts"][s].data_ptr(), speed=d["speed"].data_ptr(),
                                     speed_valid=d["sv"].data_ptr(), vkey=d["vkey"].data_ptr(),
                                     row_valid=d["rv"].data_ptr())

    for s in range(warm):
        step(0, s)
        step(1, s)
    torch.cuda.synchronize()
    # one engine alone: `steps` batches of engine 0, then of engine 1 (serial)
    t = time.perf_counter()
    for k in range(2):
        for s in range(warm, warm + steps // 2):
            step(k, s)
    torch.cuda.synchronize()
    serial = time.perf_counter() - t
    # both engines at once, one host thread each
    t = time.perf_counter()
    ths = [threading.Thread(target=lambda k=k: [step(k, s) for s in range(warm + steps // 2, warm + steps)])
           for k in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    torch.cuda.synchronize()
    conc = time.perf_counter() - t
    for e in engs:
        e.close()
    out = {"events_per_batch": n, "batches": steps, "serial_ms_per_batch": serial / steps * 1e3,
           "concurrent_ms_per_batch": conc / steps * 1e3, "gain": serial / conc}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
