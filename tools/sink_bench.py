#!/usr/bin/env python3
"""Throughput of the tiles sink's statement encoding on one MI355X.

One C2-shaped micro-batch (uniform sphere, res 8, 15 min of event time; ~1e8 tiles at 1e8 events) runs through
hm_process_batch with device-resident inputs, then hm_encode_tile_updates turns its tiles into the MongoDB `update`
statements the reference's UpdateOne ops become (heatmap_stream.py:164-196): timed device-resident (the two
kernels + the offsets scan) and with the copy to pinned host memory.  Beside it, the reference's own per-tile
Python loop (stream.tile_ops + pymongo's bson encoding of each statement) on a bounded sample of the same tiles.

usage: python tools/sink_bench.py [--events 100000000] [--reps 5] [--sample 50000]   (one JSON line)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-mobility-heatmap_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

T0 = 1759572000 * 1_000_000
HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sample", type=int, default=50_000)
    a = ap.parse_args()
    import mobheat
    from mobheat import stream
    from mobheat.engine import TileRows
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    n = a.events
    lat = torch.rad2deg(torch.asin(torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 2 - 1))
    lon = torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 360 - 180
    ts = T0 + torch.randint(0, 15 * 60_000_000, (n,), generator=g, device=dev, dtype=torch.int64)
    sp = torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 80
    sv = (torch.rand(n, generator=g, device=dev) >= 0.1).to(torch.uint8)
    vk = torch.randint(0, 50_000, (n,), generator=g, device=dev, dtype=torch.int64)
    rv = torch.ones(n, dtype=torch.uint8, device=dev)
    eng = mobheat.HeatmapEngine(h3_res=8, batch_capacity_hint=n)
    torch.cuda.synchronize()
    out = eng.process_batch_device(0, n, lat.data_ptr(), lon.data_ptr(), ts.data_ptr(), sp.data_ptr(), sv.data_ptr(),
                                   vk.data_ptr(), rv.data_ptr())
    nt = int(out.n_tiles)
    eng.encode_tile_updates_device("ath", 45)   # warm-up (buffers)
    dev_ms = []
    for _ in range(a.reps):
        t = time.perf_counter()
        eng.encode_tile_updates_device("ath", 45)   # returns after the stream drained
        dev_ms.append((time.perf_counter() - t) * 1e3)
    host_ms = []
    for _ in range(2):
        t = time.perf_counter()
        buf, offs = eng.encode_tile_updates("ath", 45)
        host_ms.append((time.perf_counter() - t) * 1e3)
    nbytes = int(offs[-1])
    # the reference's loop on a bounded sample of the same tiles (host copy of the outputs)
    import bson
    k = min(a.sample, nt)
    pick = np.sort(np.random.default_rng(0).choice(nt, k, replace=False))

    def col(p, dt):
        arr = np.empty(nt, dt)
        mobheat._lib.check(mobheat._lib.load().hm_memcpy(arr.ctypes.data, p, arr.nbytes, 1))
        return arr[pick]
    ws = col(out.window_start_us, np.int64)
    tiles = TileRows(cell=col(out.cell, np.uint64), window_start_us=ws, window_end_us=ws + eng.tile_us,
                     count=col(out.count, np.int64), avg_speed=col(out.avg_speed, np.float64),
                     speed_null=col(out.speed_null, np.uint8).astype(bool), avg_lon=col(out.avg_lon, np.float64),
                     avg_lat=col(out.avg_lat, np.float64))
    t = time.perf_counter()
    ref = [bson.encode({"q": op._filter, "u": op._doc, "multi": False, "upsert": True})
           for op in stream.tile_ops(tiles, city="ath", h3_res=8, ttl_min=45)]
    ref_s = time.perf_counter() - t
    ok = all(buf[offs[i]:offs[i + 1]].tobytes() == r for i, r in zip(pick.tolist(), ref))
    best = min(dev_ms)
    # algorithmic HBM bytes per tile: sizes pass reads cell/ws/count (24 B) and writes a u32; the write pass reads
    # the 49-B tile row + its offset (8 B) and writes the statement
    algo = nt * (24 + 4 + 49 + 8) + nbytes
    print(json.dumps({
        "what": "tiles sink: MongoDB update statements BSON-encoded on the GPU (hm_encode_tile_updates)",
        "events": n, "tiles": nt, "bson_bytes": nbytes, "bytes_per_statement": nbytes / max(nt, 1),
        "device_ms": round(best, 3), "statements_per_s_device": nt / (best * 1e-3),
        "device_GBps_algorithmic": algo / (best * 1e-3) / 1e9, "hbm_frac": algo / (best * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "host_ms_incl_d2h": round(min(host_ms), 1), "statements_per_s_host": nt / (min(host_ms) * 1e-3),
        "reference_loop": {"sample_tiles": k, "s": round(ref_s, 3), "statements_per_s": k / ref_s,
                           "what": "stream.tile_ops (heatmap_stream.py:164-188) + bson.encode per statement, 1 core"},
        "sample_bit_exact": ok}))
    eng.close()


if __name__ == "__main__":
    main()
