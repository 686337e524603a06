"""CPU restatement of the reference's decode step -- TEST INFRASTRUCTURE ONLY (the checker of hm_decode_json,
never called by the product path):

    events = raw.select(from_json(col("value").cast("string"), schema).alias("j")).select("j.*")
                .withColumn("eventTs", to_timestamp(col("ts")))            (reference heatmap_stream.py:51-61, 88-93)

restated with Python's json module (the producer's own codec: mbta_to_kafka.py:35 json.dumps) and
pandas.to_datetime(format="ISO8601", utc=True), the host parser the drop-in used before row f1.  Spark's JSON rules
(PERMISSIVE from_json, Jackson's token types; Spark 3.5) are restated field by field below; parity against Spark
itself is unpinned (no pyspark/JVM here), against Python json + pandas it is exact.

Not restated (the device decoder's documented scope, csrc/json_decode.h): Jackson-only tokens +Infinity, +INF, -INF
(Python's json rejects them: tests pin them separately), and timestamp strings outside
YYYY-MM-DD[( |T)HH:MM[:SS[.f{1,9}]][Z|(+|-)HH[[:]MM]]] (null here and on the device).
"""
import json
import math
import re

import numpy as np

SCHEMA = {"provider": "s", "vehicleId": "s", "lat": "d", "lon": "d", "speedKmh": "d", "bearing": "i", "accuracyM": "i",
          "ts": "s"}                                     # heatmap_stream.py:51-60
SPECIAL = {"NaN": math.nan, "Infinity": math.inf, "+Infinity": math.inf, "+INF": math.inf, "-Infinity": -math.inf,
           "-INF": -math.inf}                            # Spark's DoubleType strings (allowNonNumericNumbers)
TS_RE = re.compile(r"^\s*\d{4}-\d{2}-\d{2}(?:[T ]\d{2}:\d{2}(?::\d{2}(?:\.\d{1,9})?)?(?:Z|[+-]\d{2}(?::?\d{2})?)?)?\s*$")

ZONE_RE = re.compile(r"(?:Z|[+-]\d{2}(?::?\d{2})?)$")   # (after a time: TS_RE)

MALFORMED = "malformed"
UNSUPPORTED = "unsupported"


def decode_record(raw):
    """One Kafka value (bytes) -> {field: value or None}, MALFORMED (from_json's null record) or UNSUPPORTED."""
    try:
        text = raw.decode("utf-8")
        i = 0
        while i < len(text) and text[i] in " \t\n\r":
            i += 1
        obj, _ = json.JSONDecoder().raw_decode(text, i)   # (content after the first value is ignored, as Jackson's)
    except (UnicodeDecodeError, ValueError):
        return MALFORMED
    if not isinstance(obj, dict):
        return MALFORMED
    out = {}
    for f, kind in SCHEMA.items():
        v = obj.get(f)
        if v is None:
            out[f] = None
        elif kind == "d":
            if isinstance(v, bool):
                return MALFORMED
            if isinstance(v, int):
                try:
                    out[f] = float(v)
                except OverflowError:
                    out[f] = math.inf if v > 0 else -math.inf
            elif isinstance(v, float):
                out[f] = v
            elif isinstance(v, str) and v in SPECIAL:
                out[f] = SPECIAL[v]
            else:
                return MALFORMED
        elif kind == "i":
            if isinstance(v, bool) or not isinstance(v, int) or not -2 ** 31 <= v < 2 ** 31:
                return MALFORMED
            out[f] = v
        else:
            if isinstance(v, str):
                out[f] = v
            elif isinstance(v, bool):
                out[f] = "true" if v else "false"
            elif isinstance(v, int):
                out[f] = str(v)
            else:
                return UNSUPPORTED   # (Jackson re-serialises floats / objects / arrays; not decoded on the device)
    return out


def utf8(s):
    """A decoded JSON string as the bytes Spark stores (Java's UTF-8 encoder writes '?' for a lone surrogate)."""
    return s.encode("utf-8", "replace")


def to_timestamp_us(strings):
    """to_timestamp(ts) of each string (None -> None) as int64 microseconds UTC, None where it is null."""
    import pandas as pd
    out = [None] * len(strings)
    idx = [k for k, s in enumerate(strings) if s is not None and TS_RE.match(s)]
    # strings with and without a zone are parsed apart: in one mixed Series pandas applies an offset it saw to the
    # naive strings, where to_timestamp reads them in the session time zone (UTC, heatmap_stream.py:45)
    for zoned in (False, True):
        grp = [k for k in idx if bool(ZONE_RE.search(strings[k].strip())) == zoned]
        if not grp:
            continue
        ser = pd.to_datetime(pd.Series([strings[k].strip() for k in grp]), utc=True, format="ISO8601", errors="coerce")
        ns = ser.astype("int64").to_numpy()
        for j, k in enumerate(grp):
            if not pd.isna(ser.iloc[j]):
                out[k] = int(ns[j] // 1000)
    return out


def decode_values(values):
    """The batch's values (list of bytes) -> columns as batch_columns builds them (mobheat/stream.py) + the decoded
    strings: dict(lat, lon, ts_us, speed, speed_valid, row_valid, provider, vehicleId, n_malformed, n_unsupported)."""
    recs = [decode_record(v) for v in values]
    n = len(recs)
    lat, lon, speed = np.full(n, np.nan), np.full(n, np.nan), np.zeros(n)
    sv, rv = np.zeros(n, bool), np.zeros(n, bool)
    prov, veh, ts_s = [None] * n, [None] * n, [None] * n
    n_bad = n_unsup = 0
    for k, r in enumerate(recs):
        if r == MALFORMED:
            n_bad += 1
            continue
        if r == UNSUPPORTED:
            n_unsup += 1
            continue
        if r["lat"] is not None:
            lat[k] = r["lat"]
        if r["lon"] is not None:
            lon[k] = r["lon"]
        if r["speedKmh"] is not None:
            speed[k] = r["speedKmh"]
            sv[k] = True
        prov[k] = None if r["provider"] is None else utf8(r["provider"])
        veh[k] = None if r["vehicleId"] is None else utf8(r["vehicleId"])
        ts_s[k] = r["ts"]
    ts = to_timestamp_us(ts_s)
    ts_us = np.array([t if t is not None else 0 for t in ts], np.int64)
    for k in range(n):
        rv[k] = prov[k] is not None and veh[k] is not None and ts[k] is not None
    return dict(lat=lat, lon=lon, ts_us=ts_us, ts_valid=np.array([t is not None for t in ts]), speed=speed,
                speed_valid=sv, row_valid=rv, provider=prov, vehicleId=veh, n_malformed=n_bad, n_unsupported=n_unsup)
