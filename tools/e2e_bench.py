#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) rate of the drop-in boundary on one MI355X.

foreach_batch_func hands host buffers to hm_process_batch (HM_MEM_HOST): the library copies the batch's columns
to the device, runs the hot path, and copies the tiles and latest rows back.  This tool times that call on the
bench workload (C2-shaped, uniform sphere, res 8, 15 min per batch, advancing) with numpy inputs in pageable
memory and in page-locked memory (hipHostRegister through torch's pin_memory), beside the device-resident rate
bench.py reports.  It is the PCIe-inclusive figure DESIGN.md §7 quotes; bench.py's `value` stays device-resident.

usage: python tools/e2e_bench.py [--events 100000000] [--steps 4]   (one JSON line)
       python tools/e2e_bench.py --kafka [--events 10000000]
         foreach_batch_func on the raw Kafka `value` column (the producer's JSON records, mbta_to_kafka.py:66-74,
         decoded on the GPU by hm_decode_json) end to end through the same loopback wire sink
       python tools/e2e_bench.py --foreach [--events 10000000]
         foreach_batch_func end to end in its DEFAULT configuration (state checkpoints on, the state arena sized from
         the first batch): C1 (10k events, the reference's Boston batch) and a uniform batch of --events events (~that
         many tiles at res 8), as pandas frames, written (a) through the wire sink to a loopback server that
         acknowledges every OP_MSG (no MongoDB on the box: the server only reads the bytes and replies ok) and (b) into a
         null sink that takes the statements and sends nothing, so that the product's own host cost is separated from
         the loopback server's; per phase (stream.LAST_TIMINGS: columns, process, checkpoint export / wait, encode, sink)
         and the engine's allocations + frees after the first batch that evicted a window.
"""
import socket
import struct
import threading
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


class LoopbackMongo:
    """A TCP server on 127.0.0.1 that answers every OP_MSG with {ok: 1} (counts messages and bytes)."""

    def __init__(self):
        import bson
        self._ok = bson.encode({"ok": 1.0})
        self.srv = socket.socket()
        self.srv.bind(("127.0.0.1", 0))
        self.srv.listen(8)
        self.port = self.srv.getsockname()[1]
        self.messages = 0
        self.bytes = 0
        threading.Thread(target=self._serve, daemon=True).start()

    def _serve(self):
        while True:
            try:
                c, _ = self.srv.accept()
            except OSError:
                return
            threading.Thread(target=self._conn, args=(c,), daemon=True).start()

    def _conn(self, c):
        def exact(n):
            buf = bytearray(n)
            v = memoryview(buf)
            got = 0
            while got < n:
                k = c.recv_into(v[got:], n - got)
                if not k:
                    raise EOFError
                got += k
            return buf
        try:
            while True:
                length, rid, _, _ = struct.unpack("<iiii", exact(16))
                exact(length - 16)
                self.messages += 1
                self.bytes += length
                body = struct.pack("<I", 0) + b"\x00" + self._ok
                c.sendall(struct.pack("<iiii", 16 + len(body), 0, rid, 2013) + body)
        except (EOFError, OSError):
            c.close()


class NullSink:
    """Takes every update command's statements and sends nothing (the product's host cost alone)."""

    def update_statements(self, collection, buf, offs):
        pass

    def close(self):
        pass


def foreach_mode(a):
    import tempfile

    import pandas as pd
    from mobheat import stream, synth
    srv = LoopbackMongo()
    stream.MONGO_URI = f"mongodb://127.0.0.1:{srv.port}"
    stream.CHECKPOINT_DIR = tempfile.mkdtemp(prefix="mobheat-e2e-")   # (checkpoints ON: the default)
    out = {"what": "foreach_batch_func(df, epoch) end to end, default configuration (state checkpoints on, state arena "
                   "auto): pandas frame -> columns -> GPU path (rows stay on the device) -> checkpoint exported, its "
                   "file written while the tile and position statements (encoded on the GPU) go out as OP_MSG frames "
                   "over TCP to a loopback server that acknowledges each / into a null sink; median of the timed "
                   "batches (each batch advances 1 minute: windows re-touched, one evicted every 5 batches)",
           "checkpoint": stream.STATE_CHECKPOINT, "state_arena": stream.STATE_ARENA}
    import os
    import pyarrow as pa
    # (form: the frame handed over -- pandas, or the Arrow table pyspark's collection gives (Spark's types); columns:
    # MOBHEAT_COLUMNS, the device column path (hm_arrow_columns) or the host one (batch_columns))
    cases = [("c1", synth.c1_boston(seed=0), "wire", "pandas", "device"), ("uniform", None, "wire", "pandas", "device"),
             ("uniform", None, "null", "pandas", "device"), ("uniform", None, "null", "arrow", "device"),
             ("uniform", None, "wire", "arrow", "device"), ("uniform", None, "null", "pandas", "host"),
             ("uniform", None, "null", "arrow", "host")]
    if a.cases:
        cases = [c for c in cases if f"{c[0]}_{c[2]}_{c[3]}_{c[4]}" in a.cases.split(",")]
    for name, b, sink_kind, form, columns in cases:
        name = f"{name}_{sink_kind}_sink_{form}_{columns}"
        os.environ["MOBHEAT_COLUMNS"] = columns
        stream.SINK_FACTORY = NullSink if sink_kind == "null" else stream.MongoSink
        n = 10_000 if b is not None and name.startswith("c1") else a.events
        if b is None:
            rng = np.random.default_rng(3)
            b = dict(lat=np.degrees(np.arcsin(rng.uniform(-1, 1, n))), lon=rng.uniform(-180, 180, n),
                     ts_us=T0 + rng.integers(0, 60_000_000, n), speed=rng.uniform(0, 80, n),
                     speed_valid=rng.random(n) >= 0.15, vkey=rng.integers(0, 50_000, n).astype(np.uint64),
                     row_valid=np.ones(n, bool))
        sp = b["speed"].astype(float).copy()
        sp[~b["speed_valid"]] = np.nan
        vids = pd.Series(b["vkey"]).map("v{:05d}".format)
        frames = []
        for s in range(a.steps + 1):
            if form == "arrow":   # Spark's Arrow types: strings, nullable doubles, timestamp[us, tz=UTC]
                df = pa.table({"provider": pa.array(np.full(n, "mbta", object), pa.string()),
                               "vehicleId": pa.array(vids.to_numpy(), pa.string()),
                               "lat": pa.array(b["lat"]), "lon": pa.array(b["lon"]),
                               "speedKmh": pa.array(b["speed"].astype(float), mask=~np.asarray(b["speed_valid"], bool)),
                               "eventTs": pa.array(b["ts_us"] + s * 60_000_000, pa.timestamp("us", tz="UTC"))})
            else:
                df = pd.DataFrame({"provider": "mbta", "vehicleId": vids,
                                   "lat": b["lat"], "lon": b["lon"], "speedKmh": pd.Series(sp).astype(object).where(b["speed_valid"], None),
                                   "eventTs": pd.to_datetime(b["ts_us"] + s * 60_000_000, unit="us")})
            frames.append(df)
        stream.reset_engine()
        import shutil
        shutil.rmtree(stream.CHECKPOINT_DIR, ignore_errors=True)
        times, phases, allocs = [], [], []
        m0, b0 = srv.messages, srv.bytes
        for s, df in enumerate(frames):
            t = time.perf_counter()
            stream.foreach_batch_func(df, s)
            if s >= 1:
                times.append(time.perf_counter() - t)
                phases.append(dict(stream.LAST_TIMINGS))
            c = stream.get_engine().last_counts()
            allocs.append(c["allocs"] + c["frees"])
        ms = 1e3 * float(np.median(times))
        keys = sorted({k for p in phases for k in p})
        out[name] = {"events": n, "ms_per_batch": round(ms, 2), "events_per_s": n / (ms * 1e-3),
                     "batch_ms": [round(1e3 * x, 1) for x in times],
                     "phase_ms_median": {k: round(float(np.median([p.get(k, 0.0) for p in phases])), 2) for k in keys},
                     "checkpoint_frac": round(float(np.median([(p.get("checkpoint_export", 0) + p.get("checkpoint_wait", 0))
                                                               / (1e3 * t) for p, t in zip(phases, times)])), 3),
                     "allocs_frees_cumulative": allocs,
                     "messages_per_batch": (srv.messages - m0) / len(frames),
                     "wire_bytes_per_batch": (srv.bytes - b0) / len(frames)}
    stream.reset_engine()
    print(json.dumps(out))


def producer_values(n, seed=5, n_vehicles=50_000, unique=1_000_000):
    """n producer records (json.dumps of mbta_to_kafka.py:66-74's message) as Arrow binary (bytes, offsets): `unique`
    records made by json.dumps, repeated to n with copy c's minute digit set to c % 10 (so the copies fall into
    later minutes and windows)."""
    rng = np.random.default_rng(seed)
    m = min(n, unique)
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, m)))
    lon = rng.uniform(-180, 180, m)
    sp = rng.uniform(0, 80, m)
    nul = rng.random(m) < 0.1
    veh = rng.integers(0, n_vehicles, m)
    sec = rng.integers(0, 60, m)
    vals = [json.dumps({"provider": "opensky", "vehicleId": f"v{veh[k]:06d}", "lat": float(lat[k]), "lon": float(lon[k]),
                        "speedKmh": None if nul[k] else float(sp[k]), "bearing": 90, "accuracyM": None,
                        "ts": f"2025-10-04T10:0{0}:{s:02d}Z"}).encode()
            for k, s in enumerate(sec.tolist())]
    lens = np.array([len(v) for v in vals], np.int64)
    one = np.frombuffer(b"".join(vals), np.uint8)
    reps = (n + m - 1) // m
    buf = np.tile(one, reps)
    lens_all = np.tile(lens, reps)[:n]
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens_all, out=offs[1:])
    buf = buf[:offs[-1]].copy()
    ends = offs[1:]
    copy = np.arange(n) // m
    buf[ends - 7] = ord("0") + (copy % 10)   # the minute's last digit: ...T10:0M:SSZ"}
    return buf, offs


def kafka_mode(a):
    import pyarrow as pa
    from mobheat import stream
    srv = LoopbackMongo()
    stream.MONGO_URI = f"mongodb://127.0.0.1:{srv.port}"
    n = a.events
    t = time.perf_counter()
    buf, offs = producer_values(n)
    gen_s = time.perf_counter() - t
    table = pa.table({"value": pa.Array.from_buffers(pa.binary(), n, [None, pa.py_buffer(offs.astype(np.int32)),
                                                                       pa.py_buffer(buf)])})
    stream.reset_engine()
    times = []
    m0, b0 = srv.messages, srv.bytes
    for s in range(a.steps + 1):
        t = time.perf_counter()
        stream.foreach_batch_func(table, s)
        if s >= 1:
            times.append(time.perf_counter() - t)
    ms = 1e3 * float(np.median(times))
    stream.reset_engine()
    print(json.dumps({"what": "foreach_batch_func(df, epoch) on the raw Kafka value column (producer JSON records, "
                              "hm_decode_json on the GPU) -> GPU path -> statements encoded on the GPU -> OP_MSG frames "
                              "to a loopback server that acknowledges each; the same batch every epoch (its windows are "
                              "re-touched, as in the reference's ~2-s trigger); median of the timed batches",
                      "events": n, "value_bytes": int(offs[-1]), "ms_per_batch": round(ms, 1),
                      "events_per_s": n / (ms * 1e-3), "batch_ms": [round(1e3 * x, 1) for x in times],
                      "messages_per_batch": (srv.messages - m0) / (a.steps + 1),
                      "wire_bytes_per_batch": (srv.bytes - b0) / (a.steps + 1), "generate_s": round(gen_s, 1)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--foreach", action="store_true")
    ap.add_argument("--kafka", action="store_true")
    ap.add_argument("--cases", default="", help="--foreach: comma-separated case names (default: all)")
    a = ap.parse_args()
    if a.foreach:
        return foreach_mode(a)
    if a.kafka:
        return kafka_mode(a)
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
        for rows_on_device in (False, True):
            times, tiles = [], 0
            for s in range(a.steps + 2):
                cols["ts_us"][:] = ts0 + (s + (a.steps + 2) * rows_on_device) * SPAN
                t = time.perf_counter()
                res = eng.process_batch(s + (a.steps + 2) * rows_on_device, **cols, copy=False,
                                        rows_on_device=rows_on_device)
                dt = time.perf_counter() - t
                if s >= 2:
                    times.append(dt)
                    tiles = res.n_tiles
            ms = 1e3 * float(np.median(times))
            key = mode + ("_rows_on_device" if rows_on_device else "")
            out[key] = {"ms_per_batch": round(ms, 1), "events_per_s": n / (ms * 1e-3), "tiles_per_batch": tiles,
                        "bytes_out": 0 if rows_on_device else tiles * 49 + int(res.n_latest) * 8}
        eng.close()
    out["what"] = ("hm_process_batch with host inputs and host outputs (H2D of the 42-B/event columns, the hot "
                   "path, D2H of the tiles and latest rows), median of the timed batches; *_rows_on_device: the same "
                   "with the rows left on the device, as foreach_batch_func now runs it (the statements are encoded "
                   "from the device rows)")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
