"""GPU: foreach_batch_func on the Spark DataFrame form of the micro-batch (reference heatmap_stream.py:150), through the
HIP library on one GPU.  tests/spark_standin.py's stand-ins expose pyspark's Arrow surface (3.5 _collect_as_arrow, 4
toArrow) with Spark's types (timestamp[us, tz=UTC], nullable doubles with NaN values apart from nulls, strings with
nulls); the statements written must be the single-shard oracle's (tests/test_sharded_host._expected: the oracle
restatement through the library's host encoders), byte for byte on dyadic inputs, batch after batch -- and, for a larger
batch, the statements of the same micro-batch handed over as a pandas frame.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class Capture:
    log = []

    def __init__(self):
        self.cur = {"tiles": [], "positions_latest": []}
        Capture.log.append(self.cur)

    def update_raw(self, collection, statements):
        self.cur[collection].extend(bytes(s.raw) for s in statements)

    def close(self):
        pass


def test_foreach_batch_func_on_spark_frames_matches_oracle(monkeypatch, oracle_h3):
    from mobheat import stream
    from spark_standin import Spark35Frame, Spark4Frame
    from test_sharded_host import _expected
    from test_spark_frame_host import spark_like_frames
    frames = spark_like_frames(n_batches=4, n=20000, seed=12)
    exp = _expected(frames)
    monkeypatch.setattr(stream, "SINK_FACTORY", Capture)
    stream.reset_engine()
    Capture.log.clear()
    for e, f in enumerate(frames):
        stream.foreach_batch_func((Spark35Frame if e % 2 == 0 else Spark4Frame)(f, parts=3 + e), e)
    stream.reset_engine()
    assert len(Capture.log) == 4
    for e in range(4):
        for coll in ("tiles", "positions_latest"):
            assert sorted(Capture.log[e][coll]) == exp[e][coll], (e, coll)
        assert len(exp[e]["tiles"]) > 1000


def test_foreach_batch_func_spark_frame_equals_pandas_frame(monkeypatch):
    """a 400k-row batch (general, non-dyadic values): the Spark form writes the pandas form's statements -- positions
    byte for byte, tiles as documents with averages within 1e-9 relative (the GPU sums a tile's rows in an order set by
    the device's scheduling, so two runs of the same batch may differ in the last bits of a sum)"""
    from test_gpu_sharded_stream import _same_docs
    import pandas as pd
    from mobheat import stream
    from spark_standin import Spark35Frame
    rng = np.random.default_rng(3)
    n = 400_000
    sv = rng.uniform(0, 90, n)
    pdf = pd.DataFrame({"provider": np.where(rng.random(n) < 0.3, "mbta", "opensky"),
                        "vehicleId": [f"v{v}" for v in rng.integers(0, 20000, n)],
                        "lat": rng.uniform(42.2, 42.45, n), "lon": rng.uniform(-71.2, -70.95, n),
                        "speedKmh": pd.arrays.FloatingArray(sv, rng.random(n) < 0.15),
                        "eventTs": pd.to_datetime(1759572000 + rng.integers(0, 600, n), unit="s", utc=True)})
    monkeypatch.setattr(stream, "SINK_FACTORY", Capture)
    monkeypatch.setattr(stream, "STATE_CHECKPOINT", False)
    out = []
    for df in (pdf, Spark35Frame(pdf, parts=8)):
        stream.reset_engine()
        Capture.log.clear()
        stream.foreach_batch_func(df, 0)
        out.append({k: sorted(v) for k, v in Capture.log[0].items()})
    stream.reset_engine()
    assert out[0]["positions_latest"] == out[1]["positions_latest"]
    _same_docs(out[1]["tiles"], out[0]["tiles"])
    assert len(out[0]["tiles"]) > 1000 and len(out[0]["positions_latest"]) > 10000
