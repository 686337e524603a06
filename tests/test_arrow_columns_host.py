"""CPU: stream.ArrowColumns, the zero-copy hm_arrow_in over a micro-batch's Arrow columns (the boundary's device
column path, hm_arrow_columns; reference heatmap_stream.py:51-61,150).  The struct's raw pointers -- values, validity
bitmaps with their bit offsets, string offsets and bytes -- read back here exactly the columns batch_columns extracts on
the host (lat / lon null -> NaN, speed null -> invalid, row_valid, the strings of every valid row), for Spark-typed
tables, pandas frames, and sliced tables whose arrays start at a nonzero offset.  tests/test_gpu_arrow_columns.py runs
the device side."""
import ctypes

import numpy as np
import pandas as pd
import pyarrow as pa
import pytest

from mobheat import stream
from spark_standin import spark_table
from test_spark_frame_host import spark_like_frames


def _bits(addr, off, n):
    if not addr:
        return np.ones(n, bool)
    nb = (off + n + 7) // 8
    raw = np.ctypeslib.as_array(ctypes.cast(addr, ctypes.POINTER(ctypes.c_uint8)), shape=(nb,))
    return np.unpackbits(raw, bitorder="little")[off:off + n].astype(bool)


def _vals(col, n, dt):
    if not col.values:
        return None
    return np.ctypeslib.as_array(ctypes.cast(col.values, ctypes.POINTER(dt)), shape=(n,)).copy()


def _strings(col, n):
    if not col.values:
        return [None] * n
    ot = ctypes.c_int32 if col.offset_bytes == 4 else ctypes.c_int64
    o = np.ctypeslib.as_array(ctypes.cast(col.values, ctypes.POINTER(ot)), shape=(n + 1,)).astype(np.int64)
    total = int(o[-1])
    data = bytes(np.ctypeslib.as_array(ctypes.cast(col.data, ctypes.POINTER(ctypes.c_uint8)), shape=(max(total, 1),))) \
        if col.data else b""
    v = _bits(col.validity, col.validity_offset, n)
    return [data[o[i]:o[i + 1]].decode() if v[i] else None for i in range(n)]


def _readback(ac):
    """the columns hm_arrow_columns would build, from the struct's pointers (numpy restatement of k_arrow_prep)"""
    a, n = ac.struct, ac.n
    out = {}
    for k, name in (("lat", "lat"), ("lon", "lon")):
        c = getattr(a, k)
        v = _vals(c, n, ctypes.c_double)
        out[name] = np.where(_bits(c.validity, c.validity_offset, n), v, np.nan) if v is not None else np.full(n, np.nan)
    v = _vals(a.speed, n, ctypes.c_double)
    sv = _bits(a.speed.validity, a.speed.validity_offset, n) if v is not None else np.zeros(n, bool)
    out["speed_valid"], out["speed"] = sv, np.where(sv, v, 0.0) if v is not None else np.zeros(n)
    t = _vals(a.ts_us, n, ctypes.c_int64)
    if t is not None and a.ts_us.unit == 1:   # (nanoseconds: truncated toward zero to microseconds on the device)
        t = np.where(t < 0, -((-t) // 1000), t // 1000)
    tv = _bits(a.ts_us.validity, a.ts_us.validity_offset, n) if t is not None else np.zeros(n, bool)
    out["ts_us"] = np.where(tv, t, 0)
    p, v = _strings(a.provider, n), _strings(a.vehicle, n)
    out["row_valid"] = tv & np.array([x is not None for x in p]) & np.array([x is not None for x in v])
    out["pairs"] = [(x, y) for x, y, ok in zip(p, v, out["row_valid"]) if ok]
    return out


def _host(df):
    c = stream.batch_columns(df)
    pu, vu = c["provider_uniques"].to_pylist(), c["vehicle_uniques"].to_pylist()
    nv = max(len(vu), 1)
    k = c["vkey"][c["row_valid"]].astype(np.int64)
    c["pairs"] = [(pu[x // nv], vu[x % nv]) for x in k]
    return c


def _same(dev, host):
    for k in ("lat", "lon"):
        np.testing.assert_array_equal(dev[k].view(np.uint64), np.asarray(host[k], np.float64).view(np.uint64), err_msg=k)
    np.testing.assert_array_equal(dev["speed_valid"], host["speed_valid"])
    sv = dev["speed_valid"]   # (a null speed's value is unused: the host path leaves NaN there, the device 0)
    np.testing.assert_array_equal(dev["speed"][sv].view(np.uint64), np.asarray(host["speed"])[sv].view(np.uint64))
    np.testing.assert_array_equal(dev["row_valid"], host["row_valid"])
    np.testing.assert_array_equal(dev["ts_us"][dev["row_valid"]], host["ts_us"][host["row_valid"]])
    assert dev["pairs"] == host["pairs"]


@pytest.mark.parametrize("form", ["spark", "pandas", "sliced", "large_string"])
def test_arrow_columns_pointers_read_back_host_columns(form):
    pdf = spark_like_frames(1, n=4000, seed=21)[0]
    if form == "spark":
        df = spark_table(pdf)
    elif form == "pandas":
        df = pdf
    elif form == "sliced":   # arrays at offset 13 (and a chunked column)
        t = spark_table(pdf)
        df = pa.concat_tables([t.slice(13, 1000), t.slice(1013, 2000)])
        pdf = pdf.iloc[13:3013].reset_index(drop=True)
    else:
        t = spark_table(pdf)
        df = t.set_column(t.schema.get_field_index("vehicleId"), "vehicleId", t.column("vehicleId").cast(pa.large_string()))
    cols = stream.device_columns(df)
    assert "arrow" in cols and cols["n"] == len(pdf)
    _same(_readback(cols["arrow"]), _host(df if form != "pandas" else pdf))


def test_arrow_columns_absent_and_string_ts_columns():
    """absent columns (no speedKmh, no provider) and raw ISO `ts` strings (to_timestamp on the host, then a bitmap)"""
    n = 50
    df = pd.DataFrame({"vehicleId": [f"v{i}" for i in range(n)], "lat": np.linspace(-10, 10, n), "lon": 1.0,
                       "ts": ["2025-10-04T10:00:00Z"] * (n - 2) + ["bad", None]})
    cols = stream.device_columns(df)
    dev = _readback(cols["arrow"])
    assert not dev["speed_valid"].any() and not dev["row_valid"].any()   # (no provider column: every row null)
    df["provider"] = "mbta"
    dev = _readback(stream.device_columns(df)["arrow"])
    assert dev["row_valid"].tolist() == [True] * (n - 2) + [False, False]
    assert dev["ts_us"][0] == 1759572000 * 1_000_000


def test_device_columns_host_switch_and_kafka(monkeypatch):
    df = pd.DataFrame({"value": [b'{"a": 1}']})
    assert "kafka" in stream.device_columns(df)
    monkeypatch.setenv("MOBHEAT_COLUMNS", "host")
    c = stream.device_columns(spark_like_frames(1, n=10)[0])
    assert "vkey" in c and "arrow" not in c


def test_object_strings_to_arrow():
    """_strcols (threads copying compact-ASCII str bytes) + the host's handling of the rest: equal to pyarrow's own
    conversion, None / NaN / pd.NA null, non-ASCII encoded, a non-string value -> None (the caller's fallback)"""
    vals = np.array(["mbta", None, "v0001", float("nan"), "vé", "", pd.NA, "x" * 300, "日本"] * 20000, dtype=object)
    got = stream._object_strings(vals)
    exp = pa.array([None if (v is None or v is pd.NA or (isinstance(v, float) and v != v)) else v for v in vals],
                   pa.large_string())
    assert got.equals(exp)
    assert stream._object_strings(np.array(["a", 3, "b"], dtype=object)) is None
    assert len(stream._object_strings(np.array([], dtype=object))) == 0


@pytest.mark.parametrize("n", [1, 63, 64, 65, 65536 + 37, 300_001])
def test_object_strings_fused_pass(n):
    """The fused _strcols.measure/fill form (compact-ASCII str and None only): offsets, bytes and the validity bitmap
    written per block of whole 64-row groups by up to 16 threads -- equal to pyarrow's conversion at block edges, with
    and without nulls."""
    rng = np.random.default_rng(n)
    words = np.array(["", "a", "v00017", "mbta", "x" * 70], dtype=object)
    vals = words[rng.integers(0, words.size, n)]
    for nulls in (False, True):
        v = vals.copy()
        if nulls:
            v[rng.random(n) < 0.3] = None
            v[-1] = None
        got = stream._object_strings(v)
        assert got.equals(pa.array(list(v), pa.large_string())), (n, nulls)
        assert got.null_count == sum(x is None for x in v)


def test_object_floats_to_arrow():
    """_strcols.floats + the host's handling of the rest: float objects as values (NaN stays a value), None / pd.NA
    null, ints converted, a non-number -> None"""
    vals = np.array([1.5, None, float("nan"), pd.NA, 3, -0.0, np.float64(2.25)] * 20000, dtype=object)
    got = stream._object_floats(vals)
    want_valid = np.array([True, False, True, False, True, True, True] * 20000)
    assert got.type == pa.float64() and got.null_count == int((~want_valid).sum())
    v = got.to_numpy(zero_copy_only=False)
    assert np.isnan(v[2]) and v[0] == 1.5 and v[4] == 3.0 and np.signbit(v[5]) and v[6] == 2.25
    assert not got.is_valid().to_numpy(zero_copy_only=False)[1]
    assert stream._object_floats(np.array([1.0, "x"], dtype=object)) is None


def test_pandas_object_speed_column_reads_back_host_columns():
    pdf = spark_like_frames(1, n=3000, seed=22)[0]
    pdf["speedKmh"] = pdf["speedKmh"].astype(object).where(pdf["speedKmh"].notna(), None)
    pdf["lat"] = pdf["lat"].astype(object)
    cols = stream.device_columns(pdf)
    _same(_readback(cols["arrow"]), _host(pdf))
