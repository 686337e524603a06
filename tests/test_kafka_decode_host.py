"""CPU: row f1's decoder (csrc/json_decode.h: from_json + to_timestamp of the Kafka values, reference
heatmap_stream.py:51-61, 88-93) executed on the host, against the oracle (Python json + pandas.to_datetime,
oracle/kafka_oracle.py) and the committed fixture tests/golden/kafka_values.npz (tests/golden/make_kafka_golden.py).
"""
import json
import math
import os
import random
import struct

import numpy as np
import pytest

from mobheat import _lib
from oracle import kafka_oracle

HERE = os.path.dirname(os.path.abspath(__file__))
F = _lib.JF


def _golden():
    z = np.load(os.path.join(HERE, "golden", "kafka_values.npz"))
    buf, offs = z["bytes"].tobytes(), z["offsets"]
    return [buf[offs[i]:offs[i + 1]] for i in range(offs.size - 1)], z


def _strings(present, raw, lens):
    out, o = [], 0
    for p, n in zip(present, lens):
        out.append(raw[o:o + n].tobytes() if p else None)
        o += int(n)
    return out


def _same_f64(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))


def _compare(o, exp, values):
    """the host-run device decoder's per-record output vs the oracle's columns (every field, bit for bit)"""
    n = len(values)
    fl = o["flags"]
    lat = np.where(fl & F["LAT"], o["lat"], np.nan)
    lon = np.where(fl & F["LON"], o["lon"], np.nan)
    sv = (fl & F["SPEED"]) != 0
    sp = np.where(sv, o["speed"], 0.0)
    tv = (fl & F["TS"]) != 0
    rv = ((fl & F["PROV"]) != 0) & ((fl & F["VEH"]) != 0) & tv
    for name, ok in (("lat", _same_f64(lat, exp["lat"])), ("lon", _same_f64(lon, exp["lon"])),
                     ("speed", _same_f64(sp, exp["speed"]) & (sv == exp["speed_valid"])),
                     ("ts", (tv == exp["ts_valid"]) & (~tv | (o["ts_us"] == exp["ts_us"]))),
                     ("row_valid", rv == exp["row_valid"])):
        bad = np.flatnonzero(~ok)
        assert bad.size == 0, (name, [values[i] for i in bad[:3]])
    for k in range(n):
        assert o["provider"][k] == exp["provider"][k], (values[k], o["provider"][k], exp["provider"][k])
        assert o["vehicleId"][k] == exp["vehicleId"][k], (values[k], o["vehicleId"][k], exp["vehicleId"][k])
    assert int(((fl & F["MALFORMED"]) != 0).sum()) == exp["n_malformed"]


def test_oracle_reproduces_golden():
    values, z = _golden()
    exp = kafka_oracle.decode_values(values)
    for k in ("lat", "lon", "speed"):
        assert _same_f64(exp[k], z[k]).all()
    for k in ("ts_us", "ts_valid", "speed_valid", "row_valid"):
        assert np.array_equal(exp[k], z[k])
    assert exp["provider"] == _strings(z["provider_present"], z["provider_bytes"], z["provider_len"])
    assert exp["vehicleId"] == _strings(z["vehicle_present"], z["vehicle_bytes"], z["vehicle_len"])
    assert exp["n_malformed"] == int(z["n_malformed"]) > 10


def test_decoder_matches_golden_fixture():
    """producer records + edge records (NaN/Infinity tokens, non-Z and invalid timestamps, escapes, surrogates,
    invalid UTF-8, wrong types, repeated/unknown fields, malformed JSON): identical to the fixture's columns."""
    values, z = _golden()
    o = _lib.json_records_selftest(values)
    exp = dict(lat=z["lat"], lon=z["lon"], speed=z["speed"], speed_valid=z["speed_valid"], ts_us=z["ts_us"],
               ts_valid=z["ts_valid"], row_valid=z["row_valid"], n_malformed=int(z["n_malformed"]),
               provider=_strings(z["provider_present"], z["provider_bytes"], z["provider_len"]),
               vehicleId=_strings(z["vehicle_present"], z["vehicle_bytes"], z["vehicle_len"]))
    _compare(o, exp, values)


def test_unsupported_records_are_flagged():
    z = np.load(os.path.join(HERE, "golden", "kafka_values.npz"))
    ub, uo = z["unsupported_bytes"].tobytes(), z["unsupported_offsets"]
    o = _lib.json_records_selftest([ub[uo[i]:uo[i + 1]] for i in range(uo.size - 1)])
    assert np.all(o["flags"] & F["UNSUPPORTED"])


def test_random_producer_and_garbled_records_match_oracle():
    """20k records: the producer's json.dumps output with random floats (17 significant digits), escaped
    non-ASCII ids, random timestamps with zones and fractions, plus byte-level corruptions of them."""
    rng = random.Random(11)
    values = []
    for k in range(20000):
        msg = {"provider": rng.choice(["mbta", "opensky", "Αθήνα"]),
               "vehicleId": rng.choice([f"y{rng.randint(0, 99999)}", f"ώ{rng.randint(0, 99)}", rng.randint(-5, 5)]),
               "lat": rng.choice([rng.uniform(-95, 95), rng.randint(-90, 90), math.nan, None]),
               "lon": rng.uniform(-185, 185) * 10 ** rng.randint(-5, 5),
               "speedKmh": rng.choice([None, rng.uniform(0, 200) * 3.6, math.inf, -0.0]),
               "bearing": rng.choice([None, rng.randint(-2 ** 31, 2 ** 31 - 1)]), "accuracyM": None,
               "ts": (f"{rng.randint(1970, 2100):04d}-{rng.randint(1, 12):02d}-{rng.randint(1, 31):02d}"
                      + rng.choice(["", f"T{rng.randint(0, 23):02d}:{rng.randint(0, 59):02d}",
                                    f" {rng.randint(0, 23):02d}:{rng.randint(0, 59):02d}:{rng.randint(0, 59):02d}"
                                    f".{rng.randint(0, 10 ** 6 - 1):06d}"])
                      + rng.choice(["", "Z", f"+{rng.randint(0, 14):02d}:{rng.choice([0, 30, 45]):02d}",
                                    f"-{rng.randint(0, 12):02d}"]))}
        v = json.dumps(msg, ensure_ascii=rng.random() < 0.5).encode("utf-8")
        if rng.random() < 0.1:   # corrupt one byte
            i = rng.randrange(len(v))
            v = v[:i] + bytes([rng.randrange(256)]) + v[i + 1:]
        values.append(v)

    def in_scope(v):   # (the oracle's pandas parses years 1678-2261 only: datetime64[ns])
        r = kafka_oracle.decode_record(v)
        if r == kafka_oracle.UNSUPPORTED:
            return False
        ts = r["ts"] if isinstance(r, dict) else None
        return not (ts and ts.strip()[:4].isdigit() and not 1678 <= int(ts.strip()[:4]) <= 2261)
    values = [v for v in values if in_scope(v)]
    exp = kafka_oracle.decode_values(values)
    o = _lib.json_records_selftest(values)
    _compare(o, exp, values)


def test_decimal_to_double_is_correctly_rounded():
    """Eisel-Lemire with the 128-bit product (json_decode.h) against Python's correctly rounded float() on 200k
    random significands of 1-19 digits and decimal exponents -360..320 (under/overflow included)."""
    rng = random.Random(5)
    w, q = [], []
    for _ in range(200_000):
        nd = rng.randint(1, 19)
        w.append(rng.randrange(10 ** (nd - 1), 10 ** nd))
        q.append(rng.randint(-360, 320))
    # exact halfway cases between neighbouring doubles (round half to even): (2^53 + 2j + 1) 2^t
    for j in range(2000):
        for t in (0, 3, 9):
            w.append((2 ** 53 + 2 * j + 1) << t)
            q.append(0)
    got = _lib.decimal_to_double_selftest(np.array(w, np.uint64), np.array(q, np.int64))
    exp = np.array([struct.unpack("<Q", struct.pack("<d", float(f"{a}e{b}")))[0] for a, b in zip(w, q)], np.uint64)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("tok,val", [("+Infinity", math.inf), ("+INF", math.inf), ("-INF", -math.inf),
                                     ('"+INF"', math.inf), ('"-Infinity"', -math.inf), ('"NaN"', math.nan)])
def test_jackson_only_non_numeric_tokens(tok, val):
    """Tokens Jackson accepts for DoubleType under allowNonNumericNumbers that Python's json does not."""
    o = _lib.json_records_selftest([('{"provider":"p","vehicleId":"v","lat":%s,"lon":1,"ts":"2025-10-04"}' % tok).encode()])
    assert o["flags"][0] & F["LAT"] and not o["flags"][0] & F["MALFORMED"]
    assert (math.isnan(val) and math.isnan(o["lat"][0])) or o["lat"][0] == val


def _table_columns(t):
    """kafka_host.decode_table's Arrow table -> the fixture's column form"""
    lat = np.array([np.nan if v is None else v for v in t.column("lat").to_pylist()], np.float64)
    lon = np.array([np.nan if v is None else v for v in t.column("lon").to_pylist()], np.float64)
    spl = t.column("speedKmh").to_pylist()
    ts = t.column("eventTs").cast("int64").to_pylist()
    prov = [None if v is None else v.encode("utf-8") for v in t.column("provider").to_pylist()]
    veh = [None if v is None else v.encode("utf-8") for v in t.column("vehicleId").to_pylist()]
    return dict(lat=lat, lon=lon, speed=np.array([0.0 if v is None else v for v in spl]),
                speed_valid=np.array([v is not None for v in spl]), ts_us=np.array([0 if v is None else v for v in ts]),
                ts_valid=np.array([v is not None for v in ts]), provider=prov, vehicleId=veh)


def test_host_fallback_decodes_the_fixture_like_the_device():
    """mobheat.kafka_host (the product's host decode for batches with records outside the device decoder's scope)
    gives every fixture record the columns the device decoder and the oracle give it."""
    from mobheat import kafka_host
    values, z = _golden()
    offs = np.cumsum([0] + [len(v) for v in values])
    c = _table_columns(kafka_host.decode_table(np.frombuffer(b"".join(values), np.uint8), offs))
    for k in ("lat", "lon", "speed"):
        assert _same_f64(c[k], z[k]).all(), k
    assert np.array_equal(c["speed_valid"], z["speed_valid"]) and np.array_equal(c["ts_valid"], z["ts_valid"])
    assert np.array_equal(np.where(c["ts_valid"], c["ts_us"], 0), np.where(z["ts_valid"], z["ts_us"], 0))
    assert c["provider"] == _strings(z["provider_present"], z["provider_bytes"], z["provider_len"])
    assert c["vehicleId"] == _strings(z["vehicle_present"], z["vehicle_bytes"], z["vehicle_len"])


def test_host_fallback_writes_non_string_values_as_jackson_text():
    """The records the device flags (a number or an object in a StringType field) become that value's JSON text as
    Spark's JacksonParser stores it (copyCurrentStructure: compact JSON, Double.toString for floating point)."""
    from mobheat import kafka_host
    z = np.load(os.path.join(HERE, "golden", "kafka_values.npz"))
    ub, uo = z["unsupported_bytes"].tobytes(), z["unsupported_offsets"]
    recs = [kafka_host.decode_record(ub[uo[i]:uo[i + 1]]) for i in range(uo.size - 1)]
    assert recs[0]["vehicleId"] == "1.5" and recs[1]["provider"] == '{"a":1}'
    for v, want in ((1e10, "1.0E10"), (123456.0, "123456.0"), (1e-4, "1.0E-4"), (0.001, "0.001"), (-2.5e-7, "-2.5E-7"),
                    (12345678.9, "1.23456789E7"), (9999999.0, "9999999.0"), (-0.0, "-0.0"), (100.0, "100.0")):
        assert kafka_host.java_double(v) == want, v
    r = kafka_host.decode_record(b'{"provider":[1,2.5,"x",null,true],"vehicleId":{"k":{"z":-3}},"lat":1,"lon":2,"ts":"2025-10-04"}')
    assert r["provider"] == '[1,2.5,"x",null,true]' and r["vehicleId"] == '{"k":{"z":-3}}'


def test_host_decode_keeps_nested_duplicate_keys():
    """A StringType field holding an object is its JSON text as Jackson's copyCurrentStructure writes it: every token,
    nested duplicate keys included, in input order; the record's own duplicate fields: the last one wins (from_json)."""
    from mobheat import kafka_host
    r = kafka_host.decode_record(b'{"provider":"x","vehicleId":{"a":1,"a":[2,{"d":2,"d":3.5}],"b":{"c":1,"c":true}},'
                                 b'"lat":1,"lat":2.5,"provider":{"x":1,"x":null}}')
    assert r["vehicleId"] == '{"a":1,"a":[2,{"d":2,"d":3.5}],"b":{"c":1,"c":true}}'
    assert r["provider"] == '{"x":1,"x":null}' and r["lat"] == 2.5
    assert kafka_host.decode_record(b'[{"provider":"x"}]') is None


def test_splice_dictionary_extension():
    """engine._extend_dictionary (the splice step's host half): strings the batch's dictionary holds keep their code,
    new ones are appended once each in Arrow layout, None -> -1."""
    from mobheat.engine import _extend_dictionary
    offs = np.array([0, 4, 7], np.int64)
    d = (2, offs, np.frombuffer(b"mbtay\xce\x8e", np.uint8).copy())
    (n, o, raw), codes = _extend_dictionary(d, ["yΎ", None, "1.5", "mbta", "1.5", '{"a":1}'])
    assert n == 4 and codes.tolist() == [1, -1, 2, 0, 2, 3]
    assert [raw[o[k]:o[k + 1]].tobytes() for k in range(n)] == [b"mbta", b"y\xce\x8e", b"1.5", b'{"a":1}']
    (n, o, raw), codes = _extend_dictionary((0, np.zeros(1, np.int64), np.zeros(1, np.uint8)), ["", None])
    assert n == 1 and codes.tolist() == [0, -1] and o.tolist() == [0, 0]
    assert _extend_dictionary(d, [None, "mbta"])[0] is d


def test_decode_columns_rows_subset():
    """kafka_host.decode_columns on a subset of rows decodes exactly those records (the splice decodes only the
    records hm_decode_json lists)."""
    vals = [b'{"provider":"a","vehicleId":1,"ts":"2025-10-04T10:00:00Z"}', b"garbage",
            b'{"provider":"b","vehicleId":"v","lat":1.5,"ts":"2025-10-04 10:00:01"}']
    offs = np.cumsum([0] + [len(v) for v in vals])
    buf = np.frombuffer(b"".join(vals), np.uint8)
    from mobheat import kafka_host
    c = kafka_host.decode_columns(buf, offs, [2, 0])
    assert c["provider"] == ["b", "a"] and c["vehicleId"] == ["v", "1"] and c["lat"] == [1.5, None]
    assert c["ts_ok"].tolist() == [True, True] and c["malformed"] == [False, False]
    assert kafka_host.decode_columns(buf, offs, [1])["malformed"] == [True]
