"""CPU: the Spark DataFrame input branch of the boundary (reference heatmap_stream.py:150 -- Spark hands
foreach_batch_func a pyspark DataFrame).  pyspark is not installed here, so tests/spark_standin.py stands in for it with
the Arrow surface mobheat.stream reads (pyspark 3.5's _collect_as_arrow, pyspark 4's toArrow) and Spark's Arrow types:
timestamp[us, tz=UTC], nullable doubles (null apart from NaN), strings with nulls, int32 columns the job does not use.

(1) stream.batch_columns of the stand-in equals that of the same micro-batch as a pandas frame (the path the rest of
the suite pins against the oracle); (2) foreach_batch_func over the stand-ins, through the sharded writer on the CPU
(gloo, the oracle's stages), writes the single-shard oracle's statements byte for byte.  tests/test_gpu_spark_frame.py
runs the stand-ins through the GPU path.
"""
import numpy as np
import pandas as pd
import pytest

from mobheat import stream
from spark_standin import Spark35Frame, Spark4Frame, spark_table

T0 = 1759572000


def spark_like_frames(n_batches=3, n=3000, seed=9):
    """dyadic micro-batches with every kind of null the Spark schema allows: provider / vehicleId / eventTs null (the row
    fails the filter, :99-103), lat null (fails between(), :101), speedKmh null (not averaged) or NaN (avg NaN)."""
    rng = np.random.default_rng(seed)
    out = []
    for b in range(n_batches):
        lat = pd.array(42.0 + rng.integers(0, 1 << 8, n) / 1024.0, dtype="Float64")
        lat[rng.random(n) < 0.01] = pd.NA
        lon = -71.25 + rng.integers(0, 1 << 8, n) / 1024.0
        sv = rng.integers(0, 160, n) * 0.5
        sv[rng.random(n) < 0.002] = np.nan   # (a NaN value, not a null: FloatingArray keeps the two apart)
        speed = pd.arrays.FloatingArray(sv, rng.random(n) < 0.1)
        ts = pd.Series(pd.to_datetime(T0 + b * 240 + rng.integers(0, 360, n), unit="s", utc=True))
        ts[rng.random(n) < 0.01] = pd.NaT
        veh = rng.integers(0, 300, n)
        vid = pd.Series([f"v{v}" for v in veh], dtype=object)
        vid[rng.random(n) < 0.01] = None
        prov = pd.Series(np.where(veh % 5 == 0, "mbta", "opensky"), dtype=object)
        prov[rng.random(n) < 0.005] = None
        out.append(pd.DataFrame({"provider": prov, "vehicleId": vid, "lat": lat, "lon": lon, "speedKmh": speed,
                                 "bearing": rng.integers(0, 360, n).astype(np.int32), "accuracyM": np.int32(5),
                                 "eventTs": ts}))
    return out


@pytest.mark.parametrize("kind", [Spark35Frame, Spark4Frame])
def test_batch_columns_of_spark_frame_equal_pandas(kind):
    pdf = spark_like_frames(1, n=5000)[0]
    t = spark_table(pdf)
    assert str(t.schema.field("eventTs").type) == "timestamp[us, tz=UTC]"
    assert t.column("speedKmh").null_count > 0 and t.column("vehicleId").null_count > 0
    a, b = stream.batch_columns(kind(pdf)), stream.batch_columns(pdf)
    assert a["n"] == b["n"] == len(pdf)
    for k in ("lat", "lon", "speed"):
        np.testing.assert_array_equal(a[k].view(np.uint64), b[k].view(np.uint64))
    for k in ("ts_us", "speed_valid", "row_valid"):
        np.testing.assert_array_equal(a[k], b[k])
    assert np.isnan(a["speed"][a["speed_valid"]]).any()   # NaN speeds stay NaN values, nulls are null
    # the vkeys name the same (provider, vehicleId) pair on every valid row
    def pairs(c):
        pu, vu = c["provider_uniques"].to_pylist(), c["vehicle_uniques"].to_pylist()
        nv = max(len(vu), 1)
        k = c["vkey"][c["row_valid"]].astype(np.int64)
        return [(pu[x // nv], vu[x % nv]) for x in k]
    assert pairs(a) == pairs(b)


def test_empty_spark_frame():
    pdf = spark_like_frames(1, n=10)[0].iloc[:0]
    for kind in (Spark35Frame, Spark4Frame):
        c = stream.batch_columns(kind(pdf))
        assert c["n"] == 0 and c["lat"].size == 0 and c["vkey"].size == 0


def test_foreach_batch_func_on_spark_frames_sharded_cpu(tmp_path, monkeypatch, oracle_h3):
    """foreach_batch_func(stand-in, epoch) through the sharded writer on the CPU: the oracle's statements."""
    from test_sharded_host import Capture, _expected
    from sharded_fake import OracleRunner
    frames = spark_like_frames()
    exp = _expected(frames)
    monkeypatch.setattr(stream, "SINK_FACTORY", Capture)
    monkeypatch.setattr(stream, "N_GPUS", 2)
    monkeypatch.setattr(stream, "DIST_BACKEND", "gloo")
    monkeypatch.setattr(stream, "STATE_CHECKPOINT", False)
    monkeypatch.setattr(stream, "SHARDED_EXTRA", {"cpu": True, "runner": "sharded_fake:OracleRunner"})
    stream.close_sharded()
    Capture.log.clear()
    OracleRunner.commits.clear()
    try:
        for e, f in enumerate(frames):
            stream.foreach_batch_func((Spark35Frame if e % 2 == 0 else Spark4Frame)(f), e)
    finally:
        stream.close_sharded()
    written = [c for c in Capture.log if c["tiles"] or c["positions_latest"]]
    assert len(written) == 3
    for e in range(3):
        for coll in ("tiles", "positions_latest"):
            assert sorted(written[e][coll]) == exp[e][coll], (e, coll)
        assert len(exp[e]["tiles"]) > 100 and len(exp[e]["positions_latest"]) > 100
