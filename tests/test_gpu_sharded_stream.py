"""GPU: the multi-GPU path behind the reference's boundary -- foreach_batch_func(df, epoch_id) with MOBHEAT_GPUS = N
(mobheat.sharded; reference heatmap_stream.py:150,159-235,244-245).  N ranks run as this process + N-1 spawned workers,
all on the one GPU of the box with the gloo backend (RCCL refuses two ranks on one device; the 8-GPU run uses it).

The statements every rank encodes for what it owns (its tiles, the latest rows it holds) and the driver writes must be
the statements the single-GPU foreach_batch_func writes, batch after batch: byte for byte when the inputs are dyadic
(every fp64 sum is exact, so no summation order shows), and as equal documents (averages within 1e-9 relative) on
general inputs (the positions, which hold no sums, byte for byte).  A stream cut between batches (the process restarting) resumes from every rank's checkpoint chain --
also into another GPU count -- and writes what the uninterrupted stream writes.
"""
import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu

T0 = 1759572000


class Capture:
    """Sink capturing every update command's statements (RawBSONDocument bytes) per collection."""
    log = []

    def __init__(self):
        self.cur = {"tiles": [], "positions_latest": []}
        Capture.log.append(self.cur)

    def update_raw(self, collection, statements):
        self.cur[collection].extend(bytes(s.raw) for s in statements)

    def close(self):
        pass


def _frames(seed, n_batches=5, n=60_000, dyadic=True):
    """Micro-batches of a city-scale stream: 2,000 vehicles, ts advancing 4 minutes per batch over 6-minute spans
    (windows reopen across batches; some rows late by the second batch), 10% null speeds, 1% invalid rows, ties at
    vehicles' max ts.  dyadic: lat/lon/speed on binary grids (exact fp64 sums)."""
    rng = np.random.default_rng(seed)
    out = []
    for b in range(n_batches):
        if dyadic:
            lat = 42.0 + rng.integers(0, 1 << 14, n) / 65536.0
            lon = -71.25 + rng.integers(0, 1 << 14, n) / 65536.0
            speed = rng.integers(0, 160, n) * 0.5
        else:
            lat = rng.uniform(42.20, 42.45, n)
            lon = rng.uniform(-71.20, -70.95, n)
            speed = rng.uniform(0, 80, n)
        ts = T0 + b * 240 + rng.integers(0, 360, n)
        ts[: n // 50] = ts[n // 50: 2 * (n // 50)]   # (ties within vehicles at their max)
        if b == 3:
            ts[: n // 20] -= 1800   # late rows: windows already behind the watermark
        veh = rng.integers(0, 2000, n)
        sp = pd.array(speed, dtype="Float64")
        sp[rng.random(n) < 0.1] = pd.NA
        lat[rng.random(n) < 0.005] = 91.0
        vid = pd.array([f"v{v:04d}" for v in veh], dtype=object)
        vid[rng.random(n) < 0.005] = None
        out.append(pd.DataFrame({"provider": np.where(veh % 7 == 0, "mbta", "opensky"), "vehicleId": vid,
                                 "lat": lat, "lon": lon, "speedKmh": sp,
                                 "eventTs": pd.to_datetime(ts, unit="s", utc=True)}))
    return out


def _run(stream, frames, epochs):
    Capture.log.clear()
    for e in epochs:
        stream.foreach_batch_func(frames[e], e)
        print(f"[test] epoch {e}: {len(Capture.log[-1]['tiles'])} tile statements, "
              f"{len(Capture.log[-1]['positions_latest'])} positions", flush=True)
    return [dict(c) for c in Capture.log]


def _set(monkeypatch, stream, tmp_path, world, tag):
    monkeypatch.setattr(stream, "SINK_FACTORY", Capture)
    monkeypatch.setattr(stream, "N_GPUS", world)
    monkeypatch.setattr(stream, "DIST_BACKEND", "gloo")
    monkeypatch.setattr(stream, "CHECKPOINT_DIR", str(tmp_path / tag))
    monkeypatch.setattr(stream, "STATE_CHECKPOINT", True)
    stream.close_sharded()
    stream.reset_engine()


def _assert_same_statements(got, ref, what):
    """Equal multisets of statements; on a difference, the first few differing documents (decoded) in the message
    (pytest's own diff of two long byte lists takes minutes)."""
    import bson
    g, r = sorted(got), sorted(ref)
    if g == r:
        return
    gs, rs = set(g), set(r)
    only_g, only_r = [bson.decode(x) for x in g if x not in rs][:3], [bson.decode(x) for x in r if x not in gs][:3]
    raise AssertionError(f"{what}: {len(g)} vs {len(r)} statements, {len(gs - rs)} differ; "
                         f"sharded only: {only_g}; single only: {only_r}")


def _docs(stmts):
    import bson
    out = {}
    for s in stmts:
        d = bson.decode(s)
        out[d["q"]["_id"]] = d
    return out


def _same_docs(a, b):
    """tile statements (one per (cell, window) _id) as documents: averages within 1e-9 relative, the rest equal"""
    A, B = _docs(a), _docs(b)
    assert len(A) == len(a) and len(B) == len(b)
    assert set(A) == set(B)
    for k in A:
        x, y = A[k]["u"]["$set"], B[k]["u"]["$set"]
        assert set(x) == set(y)
        for f in x:
            if f == "avgSpeedKmh":
                assert abs(x[f] - y[f]) <= 1e-9 * abs(y[f]), (k, f)
            elif f == "centroid":
                for p, q in zip(x[f]["coordinates"], y[f]["coordinates"]):
                    assert abs(p - q) <= 1e-9 * abs(q), (k, f)
            else:
                assert x[f] == y[f], (k, f)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_foreach_batch_func_writes_single_gpu_statements(world, tmp_path, monkeypatch):
    """Dyadic inputs: every batch's tiles and positions_latest statements from `world` ranks equal the single-GPU
    path's byte for byte (as multisets: the reference's bulks are unordered); then a cut after batch 2 and a restart
    of the process resumes from the ranks' checkpoints (once into the same and once into another rank count) and writes
    the rest of the uninterrupted stream's statements."""
    from mobheat import stream
    frames = _frames(11)
    _set(monkeypatch, stream, tmp_path, 1, "n1")
    ref = _run(stream, frames, range(5))
    stream.reset_engine()
    _set(monkeypatch, stream, tmp_path, world, "nw")
    got = _run(stream, frames, range(5))
    for e in range(5):
        for coll in ("tiles", "positions_latest"):
            _assert_same_statements(got[e][coll], ref[e][coll], f"epoch {e} {coll}")
        assert len(ref[e]["tiles"]) > 1000 and len(ref[e]["positions_latest"]) > 1500
    # cut after batch 2: a new process (workers and state gone) resumes at epoch 3 from the checkpoints
    for world2 in (world, 3 if world != 3 else 2):
        _set(monkeypatch, stream, tmp_path, world, f"cut{world2}")
        _run(stream, frames, range(3))
        stream.close_sharded()
        monkeypatch.setattr(stream, "N_GPUS", world2)
        rest = _run(stream, frames, range(3, 5))
        for k, e in enumerate(range(3, 5)):
            for coll in ("tiles", "positions_latest"):
                _assert_same_statements(rest[k][coll], ref[e][coll], f"resumed into {world2} ranks, epoch {e} {coll}")
    stream.close_sharded()


def test_sharded_foreach_batch_func_general_inputs_and_replay(tmp_path, monkeypatch):
    """General (non-dyadic) inputs over 3 ranks: the same documents as one GPU (averages within 1e-9 relative); a
    batch whose writes fail is re-run by Spark and writes the same statements without merging twice; an epoch that
    was already committed, re-run, rebuilds the state of the epoch before it from the checkpoints."""
    from mobheat import stream
    frames = _frames(5, n_batches=4, dyadic=False)
    _set(monkeypatch, stream, tmp_path, 1, "g1")
    ref = _run(stream, frames, range(4))
    stream.reset_engine()
    _set(monkeypatch, stream, tmp_path, 3, "g3")
    got = _run(stream, frames, range(2))

    class Failing(Capture):
        def update_raw(self, collection, statements):
            raise IOError("mongo down")
    monkeypatch.setattr(stream, "SINK_FACTORY", Failing)
    with pytest.raises(IOError):
        stream.foreach_batch_func(frames[2], 2)
    monkeypatch.setattr(stream, "SINK_FACTORY", Capture)
    got += _run(stream, frames, [2])
    got += _run(stream, frames, [3])
    got += _run(stream, frames, [3])   # the committed epoch 3 re-run: restored from epoch 2's checkpoints
    for k, e in enumerate([0, 1, 2, 3, 3]):
        _same_docs(got[k]["tiles"], ref[e]["tiles"])
        # positions carry no sums: byte-identical (as multisets -- a vehicle's tied latest rows are several statements
        # for one _id, in no defined order, as in the reference's unordered bulk)
        _assert_same_statements(got[k]["positions_latest"], ref[e]["positions_latest"], f"epoch {e} positions_latest")
    stream.close_sharded()


def test_sharded_foreach_batch_func_on_kafka_values(tmp_path, monkeypatch):
    """The raw Kafka `value` column over 2 ranks (decoded on rank 0's GPU, records outside the device decoder spliced
    in from the host decode, the batch-wide dictionaries shared; every rank's slice of the decoded columns moved device
    to device, never through the host): the same statements as one GPU, byte for byte (dyadic coordinates: exact in
    JSON and in every sum)."""
    import datetime
    import json
    from mobheat import stream
    rng = np.random.default_rng(17)
    frames = []
    for b in range(3):
        n = 20_000
        vals = []
        for k in range(n):
            ts = datetime.datetime.fromtimestamp(T0 + b * 240 + int(rng.integers(0, 360)), datetime.timezone.utc)
            vals.append(json.dumps({"provider": "mbta" if k % 7 == 0 else "opensky",
                                    "vehicleId": f"v{int(rng.integers(0, 1500)):04d}",
                                    "lat": 42.0 + int(rng.integers(0, 1 << 14)) / 65536.0,
                                    "lon": -71.25 + int(rng.integers(0, 1 << 14)) / 65536.0,
                                    "speedKmh": None if k % 10 == 0 else int(rng.integers(0, 160)) * 0.5,
                                    "bearing": 90, "accuracyM": None,
                                    "ts": ts.strftime("%Y-%m-%dT%H:%M:%SZ")}).encode())
        vals[5] = b'{"provider":"mbta","vehicleId":1.5,"lat":42.25,"lon":-71.0,"ts":"2025-10-04T10:00:30Z"}'
        vals[9] = b'{"provider":{"a":1},"vehicleId":"v0001","lat":42.125,"lon":-71.125,"ts":"2025-10-04T10:01:00Z"}'
        frames.append(pd.DataFrame({"value": vals}))
    _set(monkeypatch, stream, tmp_path, 1, "k1")
    ref = _run(stream, frames, range(3))
    stream.reset_engine()
    _set(monkeypatch, stream, tmp_path, 2, "k2")

    def no_host_columns(*a, **k):
        raise AssertionError("the sharded writer copied decoded columns to the host")
    monkeypatch.setattr(stream, "_kafka_host_columns", no_host_columns)   # (rank 0 decodes, ranks take slices on-device)
    got = _run(stream, frames, range(3))
    for e in range(3):
        for coll in ("tiles", "positions_latest"):
            _assert_same_statements(got[e][coll], ref[e][coll], f"epoch {e} {coll}")
        assert len(ref[e]["positions_latest"]) > 1000
    assert any(b"mbta|1.5" in s for s in ref[0]["positions_latest"])
    stream.close_sharded()
