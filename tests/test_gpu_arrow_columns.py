"""GPU: hm_arrow_columns -- the boundary's frames (Spark's Arrow batches, Arrow tables, pandas frames) handed to the
device as their Arrow buffers, nulls resolved and provider / vehicleId factorised there (reference
heatmap_stream.py:51-61,96-106,150).  The device columns must give exactly what the host columns (stream.batch_columns)
give: the same tiles and latest rows through the engine, and the same statements through foreach_batch_func (dyadic
inputs: every fp64 sum exact, so no summation order shows)."""
import ctypes

import numpy as np
import pandas as pd
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu


def _tiles(r):
    """{(cell, window): (count, avg speed bits, null, avg lat bits, avg lon bits)} (bit patterns: NaN averages compare)"""
    t = r.tiles
    b = lambda a: np.asarray(a, np.float64).view(np.uint64)   # noqa: E731
    sp, la, lo = b(t.avg_speed), b(t.avg_lat), b(t.avg_lon)
    return {(int(t.cell[k]), int(t.window_start_us[k])): (int(t.count[k]), int(sp[k]), bool(t.speed_null[k]), int(la[k]),
                                                           int(lo[k]))
            for k in range(len(t))}


def _forms():
    from spark_standin import spark_table
    from test_spark_frame_host import spark_like_frames
    out = []
    for b, pdf in enumerate(spark_like_frames(n_batches=3, n=60_000, seed=31)):
        t = spark_table(pdf)
        out.append(("spark", t))
        out.append(("sliced", pa.concat_tables([t.slice(7, 20_000), t.slice(20_007, 39_000)])))
        out.append(("pandas", pdf))
    return out


def test_arrow_columns_equal_host_columns_through_the_engine():
    import mobheat
    from mobheat import stream
    eng_a = mobheat.HeatmapEngine(h3_res=8, device=0)
    eng_h = mobheat.HeatmapEngine(h3_res=8, device=0)
    try:
        for e, (form, df) in enumerate(_forms()):
            cols = stream.device_columns(df)
            assert "arrow" in cols, form
            ra, kb = eng_a.process_arrow(e, cols["arrow"].struct)
            h = stream.batch_columns(df)
            rh = eng_h.process_batch(e, h["lat"], h["lon"], h["ts_us"], h["speed"], h["speed_valid"], h["vkey"],
                                     h["row_valid"])
            assert _tiles(ra) == _tiles(rh), (e, form)
            np.testing.assert_array_equal(ra.latest_rows, rh.latest_rows)
            assert (ra.n_valid, ra.n_late, ra.watermark_ms, ra.n_state) == (rh.n_valid, rh.n_late, rh.watermark_ms,
                                                                            rh.n_state)
            # the dictionaries hold exactly the strings of the rows
            pn, po, pb = kb.providers
            names = {bytes(pb[po[k]:po[k + 1]]).decode() for k in range(pn)}
            assert names == set(x for x in h["provider_uniques"].to_pylist() if x is not None)
            assert kb.vehicles[0] == len(h["vehicle_uniques"])
            assert len(ra.tiles) > 1000
    finally:
        eng_a.close()
        eng_h.close()


def test_foreach_batch_func_device_columns_equal_host_columns(monkeypatch):
    from mobheat import stream
    from spark_standin import Spark35Frame
    from test_spark_frame_host import spark_like_frames

    class Capture:
        log = []

        def __init__(self):
            self.cur = {"tiles": [], "positions_latest": []}
            Capture.log.append(self.cur)

        def update_raw(self, collection, statements):
            self.cur[collection].extend(bytes(s.raw) for s in statements)

        def close(self):
            pass
    frames = spark_like_frames(n_batches=3, n=80_000, seed=41)
    monkeypatch.setattr(stream, "SINK_FACTORY", Capture)
    out = {}
    for mode in ("host", "device"):
        monkeypatch.setenv("MOBHEAT_COLUMNS", mode)
        stream.reset_engine()
        Capture.log.clear()
        for e, f in enumerate(frames):
            stream.foreach_batch_func(Spark35Frame(f) if e % 2 else f, e)
        out[mode] = [{k: sorted(v) for k, v in c.items()} for c in Capture.log]
    stream.reset_engine()
    assert out["host"] == out["device"]
    assert all(len(c["tiles"]) > 1000 and len(c["positions_latest"]) > 100 for c in out["device"])


def test_arrow_columns_rejects_bad_offsets():
    import mobheat
    from mobheat._lib import HmArrowIn
    n = 4
    offs = np.array([0, 3, 2, 5, 6], np.int32)   # not monotonic
    data = np.frombuffer(b"abcdefgh", np.uint8).copy()
    lat = np.zeros(n)
    a = HmArrowIn(n=n)
    a.lat.values = a.lon.values = lat.ctypes.data
    a.vehicle.values, a.vehicle.data, a.vehicle.offset_bytes = offs.ctypes.data, data.ctypes.data, 4
    eng = mobheat.HeatmapEngine(h3_res=8, device=0)
    try:
        with pytest.raises(RuntimeError, match="offsets out of order"):
            eng.arrow_columns(a)
        a.vehicle.offset_bytes = 3
        with pytest.raises(RuntimeError, match="string offsets of 3 bytes"):
            eng.arrow_columns(a)
    finally:
        eng.close()


def test_arrow_columns_nanosecond_timestamps():
    """A pandas frame's datetime64[ns] eventTs goes to the device as it is (hm_arrow_col.unit = 1) and is truncated
    toward zero to microseconds there -- equal to Arrow's unsafe ns -> us cast (the host path's), pre-1970 instants
    with a sub-microsecond part and NaT (-> a null eventTs: the row is invalid) included; a unit on any other column
    is refused."""
    import pyarrow.compute as pc
    import mobheat
    from mobheat import _lib, stream
    rng = np.random.default_rng(8)
    n = 5000
    ns = rng.integers(-2 * 10**18, 2 * 10**18, n)
    ns[::7] -= ns[::7] % 1000    # (whole microseconds too)
    ns[:4] = [-1, -999, -1000, -1001]
    ts = pd.Series(pd.to_datetime(ns, unit="ns"))
    ts[5::97] = pd.NaT
    pdf = pd.DataFrame({"provider": "p", "vehicleId": [f"v{k % 50}" for k in range(n)], "lat": rng.uniform(-60, 60, n),
                        "lon": rng.uniform(-180, 180, n), "speedKmh": rng.uniform(0, 50, n), "eventTs": ts})
    cols = stream.device_columns(pdf)
    a = cols["arrow"].struct
    assert a.ts_us.unit == 1
    exp = pc.cast(pa.array(ts), pa.timestamp("us"), safe=False)
    exp_v = exp.is_valid().to_numpy(zero_copy_only=False)
    exp_t = exp.cast(pa.int64()).fill_null(0).to_numpy()
    eng = mobheat.HeatmapEngine(h3_res=8, device=0)
    try:
        kb = eng.arrow_columns(a)
        lib = _lib.load()
        got_t, got_v = np.empty(n, np.int64), np.empty(n, np.uint8)
        _lib.check(lib.hm_memcpy(got_t.ctypes.data, kb.batch.ts_us, got_t.nbytes, 1), None, "hm_memcpy")
        _lib.check(lib.hm_memcpy(got_v.ctypes.data, kb.batch.row_valid, got_v.nbytes, 1), None, "hm_memcpy")
        np.testing.assert_array_equal(got_v.astype(bool), exp_v)
        np.testing.assert_array_equal(got_t[exp_v], exp_t[exp_v])
        assert list(got_t[:4]) == [0, 0, -1, -1]
        a.lat.unit = 1
        with pytest.raises(RuntimeError, match="only eventTs"):
            eng.arrow_columns(a)
    finally:
        eng.close()
