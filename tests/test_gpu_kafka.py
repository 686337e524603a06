"""GPU: row f1 -- hm_decode_json (from_json + to_timestamp of the Kafka values on the device, reference
heatmap_stream.py:51-61, 88-93) against the committed fixture and the oracle (Python json + pandas,
oracle/kafka_oracle.py), and foreach_batch_func fed raw Kafka values against the same batch fed decoded columns."""
import json
import os
import random
import time

import numpy as np
import pandas as pd
import pytest

from mobheat import _lib

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _d2h(ptr, n, dtype):
    out = np.zeros(max(n, 1), dtype)
    if n:
        _lib.check(_lib.load().hm_memcpy(out.ctypes.data, ptr, n * out.itemsize, 1))
    return out[:n]


def _strings(present, raw, lens):
    out, o = [], 0
    for p, n in zip(present, lens):
        out.append(raw[o:o + n].tobytes() if p else None)
        o += int(n)
    return out


def _dict_strings(d):
    n, offs, raw = d
    return [raw[offs[k]:offs[k + 1]].tobytes() for k in range(n)]


def _host_expected(values, offsets, rows=None):
    """mobheat.kafka_host's decode of the batch in _check_decoded's layout."""
    from mobheat import kafka_host
    c = kafka_host.decode_columns(values, offsets, rows)
    f64 = lambda v: np.array([np.nan if x is None else x for x in v], np.float64)   # noqa: E731
    sv = np.array([x is not None for x in c["speedKmh"]], bool)
    enc = lambda v: [None if x is None else x.encode("utf-8") for x in v]   # noqa: E731
    prov, veh = enc(c["provider"]), enc(c["vehicleId"])
    rv = np.array([p is not None and v is not None for p, v in zip(prov, veh)], bool) & np.asarray(c["ts_ok"], bool)
    return dict(lat=f64(c["lat"]), lon=f64(c["lon"]), speed=np.where(sv, f64(c["speedKmh"]), 0.0), speed_valid=sv,
                ts_us=np.asarray(c["ts_us"], np.int64), row_valid=rv, provider=prov, vehicleId=veh)


def _check_decoded(kb, exp, n):
    b = kb.batch
    assert b.n == n and b.memory == _lib.HM_MEM_DEVICE
    lat, lon = _d2h(b.lat, n, np.float64), _d2h(b.lon, n, np.float64)
    ts, sp = _d2h(b.ts_us, n, np.int64), _d2h(b.speed, n, np.float64)
    sv, rv = _d2h(b.speed_valid, n, np.uint8).astype(bool), _d2h(b.row_valid, n, np.uint8).astype(bool)
    vkey = _d2h(b.vkey, n, np.uint64)

    def same(a, e):
        return ((a.view(np.uint64) == e.view(np.uint64)) | (np.isnan(a) & np.isnan(e))).all()
    assert same(lat, exp["lat"]) and same(lon, exp["lon"])
    assert np.array_equal(sv, exp["speed_valid"]) and same(np.where(sv, sp, 0.0), exp["speed"])
    assert np.array_equal(rv, exp["row_valid"])
    assert np.array_equal(ts[rv], exp["ts_us"][rv])
    # the vkey names the row's exact strings through the batch's dictionaries
    provs, vehs = _dict_strings(kb.providers), _dict_strings(kb.vehicles)
    nv = max(len(vehs), 1)
    for k in np.flatnonzero(rv):
        assert provs[int(vkey[k]) // nv] == exp["provider"][k] and vehs[int(vkey[k]) % nv] == exp["vehicleId"][k]
    assert len(set(provs)) == len(provs) and len(set(vehs)) == len(vehs)   # one code per distinct string
    assert set(vehs) == {v for v in exp["vehicleId"] if v is not None}
    assert set(provs) == {p for p in exp["provider"] if p is not None}


def test_decode_golden_fixture():
    from mobheat import HeatmapEngine
    z = np.load(os.path.join(HERE, "golden", "kafka_values.npz"))
    eng = HeatmapEngine(h3_res=8)
    kb = eng.decode_json(z["bytes"], z["offsets"])
    exp = dict(lat=z["lat"], lon=z["lon"], speed=z["speed"], speed_valid=z["speed_valid"], ts_us=z["ts_us"],
               row_valid=z["row_valid"], provider=_strings(z["provider_present"], z["provider_bytes"], z["provider_len"]),
               vehicleId=_strings(z["vehicle_present"], z["vehicle_bytes"], z["vehicle_len"]))
    _check_decoded(kb, exp, z["offsets"].size - 1)
    assert kb.n_malformed == int(z["n_malformed"])
    # the fixture's unsupported records: spliced in from the host decode (engine.decode_json, hm_json_patch)
    ub, uo = z["unsupported_bytes"], z["unsupported_offsets"]
    kb = eng.decode_json(ub, uo)
    assert kb.n_spliced == uo.size - 1
    _check_decoded(kb, _host_expected(ub, uo), uo.size - 1)
    kb = eng.decode_json(np.zeros(0, np.uint8), np.zeros(1, np.int64))   # an empty batch
    assert kb.batch.n == 0 and kb.providers[0] == 0
    eng.close()


def _producer_values(rng, n, n_vehicles):
    vals = []
    for k in range(n):
        msg = {"provider": rng.choice(["mbta", "opensky"]), "vehicleId": f"y{rng.randrange(n_vehicles)}ώ",
               "lat": rng.uniform(42.2, 42.45), "lon": rng.uniform(-71.2, -70.95),
               "speedKmh": rng.choice([None, rng.uniform(0, 30) * 3.6]), "bearing": rng.choice([None, 90]),
               "accuracyM": None,
               "ts": f"2025-10-04T10:{rng.randint(0, 14):02d}:{rng.randint(0, 59):02d}Z"}
        vals.append(json.dumps(msg).encode())
    return vals


def test_decode_large_batch_and_dictionary_growth():
    """2e5 producer records with 5e4 vehicles, after a small batch (the dictionary table is sized from the last
    batch's distinct strings, so this one overflows its probes and is rebuilt full size)."""
    from mobheat import HeatmapEngine
    from oracle import kafka_oracle
    rng = random.Random(3)
    eng = HeatmapEngine(h3_res=8)
    small = _producer_values(rng, 500, 20)
    buf, offs = _lib.pack_values(small)
    eng.decode_json(buf, offs)
    vals = _producer_values(rng, 200_000, 50_000)
    buf, offs = _lib.pack_values(vals)
    t = time.perf_counter()
    kb = eng.decode_json(buf, offs)
    dt = time.perf_counter() - t
    exp = kafka_oracle.decode_values(vals)
    _check_decoded(kb, exp, len(vals))
    print(f"decode_json: {len(vals)} records, {offs[-1] / 1e6:.1f} MB in {dt * 1e3:.1f} ms (incl. H2D)")
    eng.close()


def test_foreach_batch_func_kafka_values_equal_decoded_frame():
    """foreach_batch_func on the raw Kafka `value` column writes exactly the documents it writes for the same
    batch already decoded into columns (provider, vehicleId, lat, lon, speedKmh, eventTs)."""
    from mobheat import stream
    from oracle import kafka_oracle
    rng = random.Random(9)
    vals = _producer_values(rng, 30_000, 800) + [b"not json", b'{"provider":"x","vehicleId":"y","lat":1,"lon":2,'
                                                               b'"ts":"2025-10-04T10:05:00+02:00"}']
    exp = kafka_oracle.decode_values(vals)

    def run(df):
        ops = {}

        class Capture:
            def update_raw(self, coll, stmts):
                import bson
                for st in stmts:
                    d = bson.decode(st.raw)
                    ops.setdefault(coll, {})[d["q"]["_id"]] = d
                    assert d["multi"] is False and d["upsert"] is True

            def close(self):
                pass
        stream.reset_engine()
        stream.SINK_FACTORY = Capture
        try:
            stream.foreach_batch_func(df, 0)
        finally:
            stream.SINK_FACTORY = stream.MongoSink
            stream.reset_engine()
        return ops

    got = run(pd.DataFrame({"value": vals}))
    ts = pd.to_datetime(np.where(exp["row_valid"], exp["ts_us"], 0), unit="us").to_series().reset_index(drop=True)
    ts[~exp["row_valid"]] = pd.NaT
    dec = pd.DataFrame({"provider": [p.decode() if p is not None else None for p in exp["provider"]],
                        "vehicleId": [v.decode() if v is not None else None for v in exp["vehicleId"]],
                        "lat": exp["lat"], "lon": exp["lon"],
                        "speedKmh": pd.Series([float(x) if s else None for x, s in zip(exp["speed"], exp["speed_valid"])],
                                              dtype=object),
                        "eventTs": ts})
    want = run(dec)
    assert set(got) == {"tiles", "positions_latest"}
    assert got["positions_latest"] == want["positions_latest"] and len(got["positions_latest"]) > 100
    # tiles: identical documents, except the last bits of the fp64 averages (the sums' order is not fixed)
    assert got["tiles"].keys() == want["tiles"].keys() and len(got["tiles"]) > 100

    def close(a, b):
        return a == b or abs(a - b) <= 1e-12 * max(abs(a), abs(b))
    for k, g in got["tiles"].items():
        w = want["tiles"][k]
        gs, ws = dict(g["u"]["$set"]), dict(w["u"]["$set"])
        assert close(gs.pop("avgSpeedKmh"), ws.pop("avgSpeedKmh"))
        gc, wc = gs.pop("centroid")["coordinates"], ws.pop("centroid")["coordinates"]
        assert close(gc[0], wc[0]) and close(gc[1], wc[1])
        assert gs == ws and g["q"] == w["q"]


def test_splice_unsupported_records_into_device_batch():
    """Records outside the device decoder (a number / object / array as a string field, strings new to the batch and
    strings it already holds) in a large batch: hm_decode_json lists them, the engine decodes just those on the host
    and hm_json_patch writes them in, re-encoding every vkey for the grown vehicle dictionary -- the whole batch then
    equals the host decode row for row, strings through the dictionaries.  Without HM_JSON_SPLICE the call fails."""
    from mobheat import HeatmapEngine
    rng = random.Random(23)
    vals = _producer_values(rng, 40_000, 900)
    odd = [b'{"provider":"mbta","vehicleId":1.5,"lat":42.3,"lon":-71.1,"speedKmh":10,"ts":"2025-10-04T10:22:05Z"}',
           b'{"provider":{"a":[1,2]},"vehicleId":"v-0","lat":42.31,"lon":-71.11,"ts":"2025-10-04T10:22:05Z"}',
           b'{"provider":"mbta","vehicleId":[true,null],"lat":42.32,"lon":-71.12,"ts":"2025-10-04 10:22:06"}',
           b'{"provider":"mbta","vehicleId":12345678901234567890123,"lat":1,"lon":2}',
           b'{"provider":"mbta","vehicleId":{"x":"y"},"speedKmh":null,"ts":"2025-10-04T10:22:05+01:00"}']
    pos = sorted(rng.sample(range(len(vals) + len(odd)), len(odd)))
    for p, v in zip(pos, odd):
        vals.insert(p, v)
    buf = np.frombuffer(b"".join(vals), np.uint8)
    offs = np.cumsum([0] + [len(v) for v in vals]).astype(np.int64)
    eng = HeatmapEngine(h3_res=8)
    kb = eng.decode_json(buf, offs)
    assert kb.n_spliced == len(odd) - 1   # (an integer as a string field is the device decoder's own: its text)
    _check_decoded(kb, _host_expected(buf, offs), len(vals))
    assert b"mbta" in _dict_strings(kb.providers) and b"1.5" in _dict_strings(kb.vehicles)
    # the batch through hm_process_batch: the spliced rows are ordinary rows
    res, _ = eng.process_kafka(0, buf, offs)
    e = _host_expected(buf, offs)   # valid: row_valid and lat / lon in range (the sanity filter, :96-106)
    assert res.n_valid == int((e["row_valid"] & (np.abs(e["lat"]) <= 90) & (np.abs(e["lon"]) <= 180)).sum())
    lib = _lib.load()
    jin = _lib.HmJsonIn(n=offs.size - 1, memory=_lib.HM_MEM_HOST, flags=0, bytes=buf.ctypes.data,
                        offsets=offs.ctypes.data)
    jout = _lib.HmJsonOut()
    assert lib.hm_decode_json(eng._ctx, jin, jout) == _lib.HM_E_UNSUPPORTED and jout.n_unsupported == len(odd) - 1
    # hm_json_patch's argument checks: rows outside the batch, codes outside the dictionaries, dictionaries that shrink
    kb = eng.decode_json(buf, offs)
    def patch(row, pcode, np_, nv):
        a = [np.array([row], np.int64), np.array([1.0]), np.array([2.0]), np.array([0], np.int64), np.array([0.0]),
             np.array([0], np.uint8), np.array([1], np.uint8), np.array([pcode], np.int64), np.array([0], np.int64)]
        return lib.hm_json_patch(eng._ctx, 1, *[x.ctypes.data for x in a], np_, nv)   # (a keeps the arrays alive)
    n_p, n_v = kb.providers[0], kb.vehicles[0]
    assert patch(len(vals), 0, n_p, n_v) == _lib.HM_E_INVALID
    assert patch(0, n_p, n_p, n_v) == _lib.HM_E_INVALID
    assert patch(0, 0, n_p - 1, n_v) == _lib.HM_E_INVALID
    assert patch(0, 0, n_p, n_v) == 0
    eng.close()


def test_foreach_batch_func_kafka_values_with_unsupported_records():
    """A batch holding records outside the device decoder's scope (a number as vehicleId, an object as provider) does
    not fail (those records are decoded on the host and spliced into the device batch): it writes the documents of
    the same batch decoded on the host, the odd records' strings being their JSON text as Spark stores them."""
    import numpy as np
    import pandas as pd
    from mobheat import kafka_host, stream
    rng = random.Random(19)
    vals = _producer_values(rng, 5_000, 300) + [
        b'{"provider":"mbta","vehicleId":1.5,"lat":42.3,"lon":-71.1,"speedKmh":10,"ts":"2025-10-04T10:22:05Z"}',
        b'{"provider":{"a":1},"vehicleId":"v","lat":42.31,"lon":-71.11,"ts":"2025-10-04T10:22:05Z"}']

    def run(df):
        ops = {}

        class Capture:
            def update_raw(self, coll, stmts):
                import bson
                for st in stmts:
                    d = bson.decode(st.raw)
                    ops.setdefault(coll, {})[d["q"]["_id"]] = d

            def close(self):
                pass
        stream.reset_engine()
        stream.SINK_FACTORY = Capture
        try:
            stream.foreach_batch_func(df, 0)
        finally:
            stream.SINK_FACTORY = stream.MongoSink
            stream.reset_engine()
        return ops

    got = run(pd.DataFrame({"value": vals}))
    offs = np.cumsum([0] + [len(v) for v in vals])
    want = run(kafka_host.decode_table(np.frombuffer(b"".join(vals), np.uint8), offs))
    assert got["positions_latest"] == want["positions_latest"]
    assert "mbta|1.5" in got["positions_latest"] and '{"a":1}|v' in got["positions_latest"]
    assert got["tiles"].keys() == want["tiles"].keys() and len(got["tiles"]) > 100
