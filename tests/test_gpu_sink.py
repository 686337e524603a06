"""GPU: the tiles sink's update statements BSON-encoded on the MI355X.

Bar: bit-exact -- every statement equals the bytes pymongo encodes for the reference's UpdateOne
(reference heatmap_stream.py:164-196; pymongo/synchronous/bulk.py add_update builds {q, u, multi, upsert}).
"""
import os
import time

import numpy as np
import pytest

from test_stream_host import _reference_statements

pytestmark = pytest.mark.gpu


def _split(buf, offs):
    return [buf[offs[i]:offs[i + 1]].tobytes() for i in range(offs.size - 1)]


@pytest.mark.parametrize("city", ["ath", "greater-" * 40 + "αθήνα"])
def test_c1_batch_statements_match_pymongo(city):
    """C1 through the GPU encoder; a CITY of 330 bytes takes the unstaged encoder (k_tile_docs_direct)."""
    from mobheat import HeatmapEngine, synth
    eng = HeatmapEngine(h3_res=8)
    res = eng.process_batch(0, **synth.c1_boston())
    buf, offs = eng.encode_tile_updates(city, 45)
    assert offs.size == len(res.tiles) + 1 > 100
    assert _split(buf, offs) == _reference_statements(res.tiles, city, 8, 45)
    eng.close()


@pytest.mark.parametrize("tz", ["EET-2EEST,M3.5.0/3,M10.5.0/4", "UTC"])
def test_stream_statements_local_time_and_dst(tz):
    """Several batches around the EU DST change (2025-10-26 01:00 UTC), pyspark's naive local datetimes."""
    from mobheat import HeatmapEngine
    old = os.environ.get("TZ")
    os.environ["TZ"] = tz
    time.tzset()
    try:
        rng = np.random.default_rng(41)
        eng = HeatmapEngine(h3_res=10, tile_minutes=5)
        t0 = 1761440100 * 1_000_000 - 20 * 60_000_000
        for e in range(4):
            n = 30000
            b = dict(lat=rng.uniform(37.90, 38.05, n), lon=rng.uniform(23.60, 23.85, n),
                     ts_us=t0 + e * 10 * 60_000_000 + rng.integers(0, 15 * 60_000_000, n), speed=rng.uniform(0, 90, n),
                     speed_valid=rng.random(n) > 0.3, vkey=rng.integers(0, 300, n).astype(np.uint64), row_valid=None)
            res = eng.process_batch(e, **b)
            buf, offs = eng.encode_tile_updates("αθήνα", 45)
            assert _split(buf, offs) == _reference_statements(res.tiles, "αθήνα", 10, 45)
        eng.close()
    finally:
        if old is None:
            del os.environ["TZ"]
        else:
            os.environ["TZ"] = old
        time.tzset()


def test_large_batch_statements_and_device_copy():
    """2e6 events at res 8 (~2e6 tiles): every statement equals the host execution of the same encoder, a
    random sample equals pymongo's bytes, and the device-resident copy equals the host one."""
    import ctypes
    from mobheat import HeatmapEngine, _lib
    from mobheat.engine import TileRows
    rng = np.random.default_rng(42)
    n = 2_000_000
    eng = HeatmapEngine(h3_res=8)
    res = eng.process_batch(0, lat=np.degrees(np.arcsin(rng.uniform(-1, 1, n))), lon=rng.uniform(-180, 180, n),
                            ts_us=1759572000_000_000 + rng.integers(0, 15 * 60_000_000, n), speed=rng.uniform(0, 80, n),
                            speed_valid=rng.random(n) > 0.1, vkey=rng.integers(0, 50000, n).astype(np.uint64))
    buf, offs = eng.encode_tile_updates("ath", 45)
    hb, ho = _lib.tile_statements_selftest(res.tiles, "ath", 8, 45, eng.tile_us)
    np.testing.assert_array_equal(offs, ho)
    np.testing.assert_array_equal(buf, hb)
    pick = rng.choice(len(res.tiles), 2000, replace=False)
    sub = TileRows(**{f: getattr(res.tiles, f)[pick] for f in TileRows.__dataclass_fields__})
    assert [buf[offs[i]:offs[i + 1]].tobytes() for i in pick] == _reference_statements(sub, "ath", 8, 45)
    pb, po, nd = eng.encode_tile_updates_device("ath", 45)
    assert nd == len(res.tiles)
    dev_offs = np.zeros(nd + 1, np.int64)
    dev_buf = np.zeros(int(offs[-1]), np.uint8)
    _lib.check(_lib.load().hm_memcpy(dev_offs.ctypes.data, po, dev_offs.nbytes, 1))
    _lib.check(_lib.load().hm_memcpy(dev_buf.ctypes.data, pb, dev_buf.nbytes, 1))
    np.testing.assert_array_equal(dev_offs, offs)
    np.testing.assert_array_equal(dev_buf, buf)
    eng.close()
    del ctypes


def test_streamed_statements_land_in_pieces_and_feed_the_wire_sink():
    """HM_MEM_HOST_STREAM (hm_statements_wait): the offsets are there when the encode returns, the bytes land in pieces
    (>= 32 MiB, at most 64) -- after landed(offs[k]) statements [0, k) equal the synchronous encode's; a wait past the
    end or without a streamed encode is refused; a sink fed command by command as they land (wire.WireMongoSink, each
    command's bytes captured as send_statements is called) sends the synchronous encode's bytes."""
    from mobheat import HeatmapEngine
    rng = np.random.default_rng(44)
    n = 1_500_000
    eng = HeatmapEngine(h3_res=9)
    eng.process_batch(0, lat=np.degrees(np.arcsin(rng.uniform(-1, 1, n))), lon=rng.uniform(-180, 180, n),
                      ts_us=1759572000_000_000 + rng.integers(0, 15 * 60_000_000, n), speed=rng.uniform(0, 80, n),
                      speed_valid=rng.random(n) > 0.1, vkey=rng.integers(0, 50000, n).astype(np.uint64))
    ref_buf, ref_offs = eng.encode_tile_updates("ath", 45, copy=True)
    assert ref_buf.size > (64 << 20)   # (several pieces)
    buf, offs, landed = eng.encode_tile_updates_streamed("ath", 45)
    np.testing.assert_array_equal(offs, ref_offs)
    seen = []
    for k in np.linspace(0, offs.size - 1, 9).astype(int)[1:]:
        landed(int(offs[k]))
        seen.append(buf[: offs[k]].tobytes() == ref_buf[: ref_offs[k]].tobytes())
    assert all(seen)
    with pytest.raises(RuntimeError, match="bytes of"):
        landed(int(offs[-1]) + 1)
    # the wire sink, command by command: each command's bytes as send_statements sees them when it is called
    from mobheat import wire

    class Capture(wire.WireMongoSink):
        def __init__(self):
            self.sent = []

        def send_statements(self, collection, buf, lo, hi, n_statements, write_concern=None):
            self.sent.append(bytes(buf[lo:hi]))
            return {"ok": 1.0, "n": n_statements}
    buf, offs, landed = eng.encode_tile_updates_streamed("ath", 45)
    sink = Capture()
    sink.update_statements("tiles", buf, offs, landed=landed)
    assert len(sink.sent) > 10 and b"".join(sink.sent) == ref_buf.tobytes()
    eng.encode_tile_updates("ath", 45)   # (synchronous: nothing left to wait for)
    with pytest.raises(RuntimeError, match="without a streamed encode"):
        landed(1)
    eng.close()


def test_empty_batch_and_errors():
    from mobheat import HeatmapEngine
    eng = HeatmapEngine(h3_res=8)
    z = np.zeros(0)
    eng.process_batch(0, lat=z, lon=z, ts_us=np.zeros(0, np.int64))
    buf, offs = eng.encode_tile_updates("ath", 45)
    assert buf.size == 0 and offs.tolist() == [0]
    with pytest.raises(RuntimeError, match="city"):
        eng.encode_tile_updates("x" * (1 << 20 | 1), 45)   # (a CITY of more than 1 MiB)
    eng.close()


def test_position_statements_match_pymongo():
    """The positions half: a C5-like batch (vehicles with several updates and ties) through foreach's columns;
    the GPU statements equal pymongo's bytes for the reference's positions_latest UpdateOne ops."""
    import bson
    import pandas as pd
    from mobheat import HeatmapEngine, stream
    rng = np.random.default_rng(43)
    n = 200_000
    ts = 1759572000_000_000 + rng.integers(0, 60, n) * 1_000_000 + rng.integers(0, 3, n) * 1000
    df = pd.DataFrame({"provider": rng.choice(["mbta", "opensky"], n),
                       "vehicleId": [f"V{int(x)}" for x in rng.integers(0, 20000, n)],
                       "lat": rng.uniform(42.2, 42.45, n), "lon": rng.uniform(-71.2, -70.95, n),
                       "speedKmh": rng.uniform(0, 80, n), "eventTs": pd.to_datetime(ts, unit="us")})
    cols = stream.batch_columns(df)
    eng = HeatmapEngine(h3_res=8)
    res = eng.process_batch(0, cols["lat"], cols["lon"], cols["ts_us"], cols["speed"], cols["speed_valid"],
                            cols["vkey"], cols["row_valid"])
    rows = res.latest_rows
    assert rows.size > 20000   # ties: several rows for some vehicles
    t = cols["ts_us"][rows]
    buf, offs = eng.encode_position_updates(cols["provider_uniques"], cols["vehicle_uniques"], t)
    exp = [bson.encode({"q": op._filter, "u": op._doc, "multi": False, "upsert": True})
           for op in stream.position_ops(cols, rows)]
    assert _split(buf, offs) == exp
    with pytest.raises(RuntimeError, match="dictionaries"):
        eng.encode_position_updates(cols["provider_uniques"][:1], cols["vehicle_uniques"], t)
    eng.close()
