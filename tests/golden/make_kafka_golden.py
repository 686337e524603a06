#!/usr/bin/env python3
"""Generate tests/golden/kafka_values.npz: Kafka message values as the reference's producer writes them
(mbta_to_kafka.py:66-74, json.dumps of the vehicle dict) plus hand-written edge records, and their decoded columns.

Provenance: the expected columns come from oracle/kafka_oracle.py -- Python's json module + pandas.to_datetime, i.e.
a restatement of from_json + to_timestamp (reference heatmap_stream.py:51-61, 88-93), NOT Spark's output (pyspark /
a JVM are absent).  The values themselves are data: the producer's serializer applied to synthetic vehicles, and
literal edge strings.

Run: python tests/golden/make_kafka_golden.py
"""
import json
import math
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-mobility-heatmap_amd")]

from oracle import kafka_oracle  # noqa: E402


def producer_values(rng, n):
    """The producer's records: msg = {provider, vehicleId, lat, lon, speedKmh, bearing, accuracyM, ts} (:66-74)."""
    out = []
    for k in range(n):
        speed = rng.choice([None, rng.uniform(0, 30), float(rng.randint(0, 25))])
        msg = {
            "provider": "mbta",
            "vehicleId": rng.choice([f"y{rng.randint(1000, 2999)}", f"{rng.randint(1000, 9999)}",
                                     f"G-{rng.randint(10, 99)}ώ", "unknown"]),
            "lat": float(rng.uniform(42.2, 42.45)), "lon": float(rng.uniform(-71.2, -70.95)),
            "speedKmh": (float(speed) * 3.6 if isinstance(speed, (float, int)) else None),
            "bearing": rng.choice([None, rng.randint(0, 359)]),
            "accuracyM": None,
            "ts": f"2025-10-04T{rng.randint(0, 23):02d}:{rng.randint(0, 59):02d}:{rng.randint(0, 59):02d}Z",
        }
        out.append(json.dumps(msg).encode("utf-8"))
    return out


EDGE = [
    # special numbers (json.dumps writes NaN / Infinity / -Infinity), non-Z timestamps, nulls
    json.dumps({"provider": "opensky", "vehicleId": "a1", "lat": math.nan, "lon": 1.0, "speedKmh": math.inf,
                "ts": "2025-10-04T10:22:05+02:00"}),
    json.dumps({"provider": "opensky", "vehicleId": "a2", "lat": 10.0, "lon": -math.inf, "speedKmh": math.nan,
                "ts": "2025-10-04 10:22:05.123456789"}),
    '{"provider":"p","vehicleId":"v","lat":1,"lon":-0,"speedKmh":-0.0,"ts":"2025-10-04T10:22:05.5-05:30"}',
    '{"provider":"p","vehicleId":"v","lat":0.1e1,"lon":1E-2,"speedKmh":12345678901234567890123,"ts":"2025-10-04T10:22Z"}',
    '{"provider":"p","vehicleId":"v","lat":4.9e-324,"lon":2.2250738585072011e-308,"speedKmh":1e400,"ts":"2025-10-04"}',
    '{"provider":"p","vehicleId":"v","lat":1e-400,"lon":-1.7976931348623157e308,"speedKmh":3.14159265358979323846264,'
    '"ts":"2024-02-29T23:59:59.999999Z"}',
    '{"provider":"p","vehicleId":"v","lat":"NaN","lon":"-Infinity","speedKmh":"Infinity","ts":"2025-10-04T10:22:05+0530"}',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05-03"}',
    # invalid timestamps -> null eventTs (row dropped)
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":"2025-13-04T10:22:05Z"}',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":"2025-02-30T10:22:05Z"}',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":"2025-10-04T24:00:00Z"}',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:60:00Z"}',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":"not a time"}',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":""}',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":null}',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0}',
    # strings: escapes, non-ASCII (json.dumps escapes it), surrogate pairs, a lone surrogate, raw UTF-8
    json.dumps({"provider": "mb\"ta\\/\n", "vehicleId": "ώ-😀", "lat": 1.5, "lon": 2.5, "ts": "2025-10-04T10:22:05Z"}),
    '{"provider":"p\\ud800x","vehicleId":"\\u0041\\u00e9\\ud83d\\ude00","lat":1.5,"lon":2.5,"ts":"2025-10-04T10:22:05Z"}',
    json.dumps({"provider": "Αθήνα", "vehicleId": "bus 7", "lat": 37.98, "lon": 23.72, "ts": "2025-10-04T10:22:05Z"},
               ensure_ascii=False),
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":"\\u0032025-10-04T10:22:05Z"}',
    # string fields holding other JSON types; repeated and unknown fields; whitespace; content after the object
    '{"provider":true,"vehicleId":12345,"lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
    '{"provider":"p","vehicleId":-0,"lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lat":null,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
    '{"provider":"p","vehicleId":"v","lat":null,"lat":3.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
    '{"extra":{"a":[1,2.5,{"b":null,"c":"x\\"y"}],"d":true},"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,'
    '"ts":"2025-10-04T10:22:05Z","more":[]}',
    ' \t\n{ "provider" : "p" , "vehicleId" : "v" , "lat" : 1.0 , "lon" : 2.0 , "ts" : "2025-10-04T10:22:05Z" } \n',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"} {"x": 1} trailing',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"bearing":2147483647,"accuracyM":-2147483648,'
    '"ts":"2025-10-04T10:22:05Z"}',
    '{}',
    # malformed records -> every field null
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"bearing":2147483648,"ts":"2025-10-04T10:22:05Z"}',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"bearing":1.5,"ts":"2025-10-04T10:22:05Z"}',
    '{"provider":"p","vehicleId":"v","lat":"abc","lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
    '{"provider":"p","vehicleId":"v","lat":true,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
    '{"provider":"p","vehicleId":"v","lat":[1],"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
    '{"provider":"p","vehicleId":"v","lat":01,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
    '{"provider":"p","vehicleId":"v","lat":1.,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
    '{"provider":"p","vehicleId":"v","lat":.5,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z",}',
    '{"provider":"p","vehicleId":"v\tx","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
    "{'provider':'p'}",
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"',
    '[{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}]',
    '"just a string"',
    '42',
    '',
    'null',
    '{"provider":"p","vehicleId":"v","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z","x":tru}',
    '{"provider":"p","vehicleId":"\\x41","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
]
EDGE_BYTES = [e.encode("utf-8") for e in EDGE] + [
    b'{"provider":"p","vehicleId":"\xff\xfe","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',   # invalid UTF-8
    b'{"provider":"p","vehicleId":"\xc0\xaf","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',   # overlong
    b'{"provider":"p","vehicleId":"\xed\xa0\x80","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',   # surrogate
]
# records the device decoder does not handle (the call fails with HM_E_UNSUPPORTED)
UNSUPPORTED = [b'{"provider":"p","vehicleId":1.5,"lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}',
               b'{"provider":{"a":1},"vehicleId":"v","lat":1.0,"lon":2.0,"ts":"2025-10-04T10:22:05Z"}']


def main():
    rng = random.Random(7)
    values = producer_values(rng, 3000) + EDGE_BYTES
    rng.shuffle(values)
    exp = kafka_oracle.decode_values(values)
    assert exp["n_unsupported"] == 0
    for u in UNSUPPORTED:
        assert kafka_oracle.decode_record(u) == kafka_oracle.UNSUPPORTED
    lens = np.array([len(v) for v in values], np.int64)
    offs = np.zeros(len(values) + 1, np.int64)
    np.cumsum(lens, out=offs[1:])

    def strcol(col):
        present = np.array([s is not None for s in col])
        joined = b"".join(s for s in col if s is not None)
        lens = np.array([len(s) if s is not None else 0 for s in col], np.int64)
        return present, np.frombuffer(joined, np.uint8) if joined else np.zeros(0, np.uint8), lens
    pp, pb, pl = strcol(exp["provider"])
    vp, vb, vl = strcol(exp["vehicleId"])
    ub = b"".join(UNSUPPORTED)
    np.savez_compressed(os.path.join(HERE, "kafka_values.npz"), bytes=np.frombuffer(b"".join(values), np.uint8),
                        offsets=offs, lat=exp["lat"], lon=exp["lon"], ts_us=exp["ts_us"], ts_valid=exp["ts_valid"],
                        speed=exp["speed"], speed_valid=exp["speed_valid"], row_valid=exp["row_valid"],
                        provider_present=pp, provider_bytes=pb, provider_len=pl, vehicle_present=vp, vehicle_bytes=vb,
                        vehicle_len=vl, n_malformed=np.int64(exp["n_malformed"]),
                        unsupported_bytes=np.frombuffer(ub, np.uint8),
                        unsupported_offsets=np.array([0, len(UNSUPPORTED[0]), len(ub)], np.int64))
    print(f"kafka_values.npz: {len(values)} values, {exp['n_malformed']} malformed, "
          f"{int(exp['row_valid'].sum())} valid rows")


if __name__ == "__main__":
    main()
