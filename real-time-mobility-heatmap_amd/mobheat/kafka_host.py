"""Host decode of the Kafka records the GPU decoder does not handle (spliced into the device batch).

hm_decode_json (row f1, csrc/json_decode.h) decodes the producer's records on the device and, for the rare record
outside its scope (a non-string JSON value in a StringType field, a >19-digit number on a rounding boundary), does not
silently differ: with HM_JSON_SPLICE it leaves that row all-null and lists it.  The reference never rejects such a
record: Spark's from_json (heatmap_stream.py:88-93, PERMISSIVE, Spark 3.5) keeps it, turning e.g. a numeric vehicleId
into that value's JSON text.  So the engine (engine.py decode_json) decodes just the listed records here, on the host,
with the same rules as the device decoder plus the cases it leaves out, and writes them into the device batch with
hm_json_patch -- a batch with one odd record costs one record's host decode, not the whole batch's.

Rules (Spark 3.5 JacksonParser, schema heatmap_stream.py:51-60):
  * a value that is not a JSON object (or not UTF-8 / not JSON) -> an all-null record;
  * absent / null field -> null; a field of the wrong type -> the whole record null (PERMISSIVE from_json);
  * DoubleType: JSON numbers (correctly rounded), the strings NaN, Infinity, +Infinity, +INF, -Infinity, -INF;
  * IntegerType (bearing, accuracyM): 32-bit integers;
  * StringType: a JSON string as is; any other value as Jackson re-serialises it (copyCurrentStructure: compact JSON,
    integers as written, floating-point numbers as Java's Double.toString);
  * ts: to_timestamp of YYYY-MM-DD[( |T)HH:MM[:SS[.f{1,9}]][Z|(+|-)HH[[:]MM]]] (UTC when no zone), null otherwise.
Parity: the device decoder's records decode identically (tests/test_kafka_decode_host.py); re-serialised doubles use
the shortest round-trip digits in Double.toString's layout, which is what Java 19+ prints -- where the reference's
Java 17 printed a longer digit string (the pre-JDK-19 algorithm occasionally does) the result is parity-unpinned.
"""
import decimal
import json
import math
import re

import numpy as np

SCHEMA = {"provider": "s", "vehicleId": "s", "lat": "d", "lon": "d", "speedKmh": "d", "bearing": "i", "accuracyM": "i",
          "ts": "s"}
_SPECIAL = {"NaN": math.nan, "Infinity": math.inf, "+Infinity": math.inf, "+INF": math.inf, "-Infinity": -math.inf,
            "-INF": -math.inf}
_TS_RE = re.compile(r"^\s*\d{4}-\d{2}-\d{2}(?:[T ]\d{2}:\d{2}(?::\d{2}(?:\.\d{1,9})?)?(?:Z|[+-]\d{2}(?::?\d{2})?)?)?\s*$")
_ZONE_RE = re.compile(r"[T ]\d{2}:\d{2}.*(?:Z|[+-]\d{2}(?::?\d{2})?)$")   # a zone only after a time


def java_double(d):
    """Java's Double.toString of d (shortest round-trip digits): plain for 1e-3 <= |d| < 1e7, else d.dddE[-]n."""
    if d != d:
        return "NaN"
    if math.isinf(d):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    sign, digits, exp = decimal.Decimal(repr(d)).as_tuple()
    ds = "".join(map(str, digits)).rstrip("0") or "0"
    e10 = exp + len(digits) - 1            # d = 0.ds... * 10^(e10 + 1) -> leading digit's power of ten
    s = "-" if sign else ""
    if 1e-3 <= abs(d) < 1e7:
        if e10 >= 0:
            ip, fp = ds[:e10 + 1].ljust(e10 + 1, "0"), ds[e10 + 1:]
        else:
            ip, fp = "0", "0" * (-e10 - 1) + ds
        return f"{s}{ip}.{fp or '0'}"
    return f"{s}{ds[0]}.{ds[1:] or '0'}E{e10}"


def _jackson_text(v):
    """A non-string JSON value as Jackson's generator writes it (copyCurrentStructure, default features)."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return java_double(v)
    if isinstance(v, _Pairs):   # every pair, duplicates included, in input order (copyCurrentStructure copies tokens)
        return "{" + ",".join(json.dumps(k, ensure_ascii=False) + ":" + _jackson_value(x) for k, x in v) + "}"
    if isinstance(v, list):
        return "[" + ",".join(_jackson_value(x) for x in v) + "]"
    raise TypeError(type(v))


def _jackson_value(v):
    if v is None:
        return "null"
    if isinstance(v, str):
        return json.dumps(v, ensure_ascii=False)
    return _jackson_text(v)


class _Pairs(list):
    """A JSON object as its (key, value) pairs in input order: nested objects are re-serialised token for token."""


def _pairs(pairs):
    return _Pairs(pairs)


def decode_record(raw):
    """One Kafka value (bytes) -> {field: value or None}, or None for from_json's all-null record."""
    try:
        text = raw.decode("utf-8")
        i = 0
        while i < len(text) and text[i] in " \t\n\r":
            i += 1
        obj, _ = json.JSONDecoder(object_pairs_hook=_pairs).raw_decode(text, i)
    except (UnicodeDecodeError, ValueError):
        return None
    if not isinstance(obj, _Pairs):
        return None
    obj = dict(obj)   # the record's own fields: the last duplicate wins, as the device decoder and from_json's parser
    out = {}
    for f, kind in SCHEMA.items():
        v = obj.get(f)
        if v is None:
            out[f] = None
        elif kind == "d":
            if isinstance(v, bool):
                return None
            if isinstance(v, int):
                try:
                    out[f] = float(v)
                except OverflowError:
                    out[f] = math.inf if v > 0 else -math.inf
            elif isinstance(v, float):
                out[f] = v
            elif isinstance(v, str) and v in _SPECIAL:
                out[f] = _SPECIAL[v]
            else:
                return None
        elif kind == "i":
            if isinstance(v, bool) or not isinstance(v, int) or not -2 ** 31 <= v < 2 ** 31:
                return None
            out[f] = v
        else:
            out[f] = v if isinstance(v, str) else _jackson_text(v)
    return out


def _to_timestamp_us(strings):
    import pandas as pd
    out = np.zeros(len(strings), np.int64)
    ok = np.zeros(len(strings), bool)
    idx = [k for k, s in enumerate(strings) if s is not None and _TS_RE.match(s)]
    for zoned in (False, True):   # parsed apart: pandas would apply a seen offset to the naive strings
        grp = [k for k in idx if bool(_ZONE_RE.search(strings[k].strip())) == zoned]
        if not grp:
            continue
        ser = pd.to_datetime(pd.Series([strings[k].strip() for k in grp]), utc=True, format="ISO8601", errors="coerce")
        ns = ser.astype("int64").to_numpy()
        for j, k in enumerate(grp):
            if not pd.isna(ser.iloc[j]):
                out[k], ok[k] = ns[j] // 1000, True
    return out, ok


def decode_columns(values, offsets, rows=None):
    """Records `rows` (int indices; all by default) of the batch's values (bytes uint8 + offsets int64[n+1], Arrow
    binary layout) -> columns as Python lists: provider / vehicleId (str or None, as the UTF-8 Spark stores), lat /
    lon / speedKmh (float or None), ts (the raw string), plus ts_us int64 / ts_ok bool (to_timestamp) and malformed
    (from_json's all-null record)."""
    offs = np.asarray(offsets, np.int64)
    buf = np.asarray(values, np.uint8)
    if rows is None:
        rows = range(offs.size - 1)
    recs = [decode_record(buf[offs[k]:offs[k + 1]].tobytes()) for k in rows]
    col = {f: [None if r is None else r[f] for r in recs] for f in ("provider", "vehicleId", "lat", "lon", "speedKmh", "ts")}
    for f in ("provider", "vehicleId"):   # the UTF-8 Spark stores: Java's encoder writes '?' for a lone surrogate
        col[f] = [None if v is None else v.encode("utf-8", "replace").decode("utf-8") for v in col[f]]
    col["ts_us"], col["ts_ok"] = _to_timestamp_us(col["ts"])
    col["malformed"] = [r is None for r in recs]
    return col


def decode_table(values, offsets):
    """The whole batch decoded on the host -> a pyarrow Table with the columns stream.batch_columns takes (provider,
    vehicleId, lat, lon, speedKmh, eventTs: null where from_json / to_timestamp give null; NaN speeds stay NaN)."""
    import pyarrow as pa
    col = decode_columns(values, offsets)
    ts_us, ts_ok = col["ts_us"], col["ts_ok"]
    return pa.table({
        "provider": pa.array(col["provider"], pa.string()),
        "vehicleId": pa.array(col["vehicleId"], pa.string()),
        "lat": pa.array(col["lat"], pa.float64(), from_pandas=False),
        "lon": pa.array(col["lon"], pa.float64(), from_pandas=False),
        "speedKmh": pa.array(col["speedKmh"], pa.float64(), from_pandas=False),
        "eventTs": pa.array(ts_us, pa.timestamp("us", tz="UTC"), mask=~ts_ok),
    })
