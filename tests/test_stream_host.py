"""CPU: the host side of the drop-in boundary (mobheat/stream.py) against the reference's document formats.

Expected documents are written out literally from reference heatmap_stream.py:164-188 (tiles) and :211-228
(positions_latest); BSON encoding uses the real pymongo/bson to pin datetime handling (naive datetimes are
encoded as UTC milliseconds, sub-millisecond digits dropped -- SURVEY.md App. A.7).
"""
import datetime
import json
import os

import bson
import numpy as np
import pandas as pd
import pyarrow as pa
import pytest

from mobheat import stream
from mobheat.engine import TileRows


def _tiles(**kw):
    n = len(kw["cell"])
    base = dict(cell=np.array(kw["cell"], np.uint64), window_start_us=np.array(kw["ws"], np.int64))
    base["window_end_us"] = base["window_start_us"] + 300_000_000
    base["count"] = np.array(kw.get("count", [1] * n), np.int64)
    base["avg_speed"] = np.array(kw.get("avg_speed", [0.0] * n), np.float64)
    base["speed_null"] = np.array(kw.get("speed_null", [False] * n), bool)
    base["avg_lon"] = np.array(kw.get("avg_lon", [0.0] * n), np.float64)
    base["avg_lat"] = np.array(kw.get("avg_lat", [0.0] * n), np.float64)
    return TileRows(**base)


def test_tile_document_matches_reference_format():
    ws = 1759573200 * 1_000_000          # 2025-10-04T10:20:00Z
    t = _tiles(cell=[0x882A1072B5FFFFF], ws=[ws], count=[7], avg_speed=[21.5], avg_lon=[-71.06], avg_lat=[42.355])
    ops = stream.tile_ops(t, city="ath", h3_res=8, ttl_min=45)
    assert len(ops) == 1
    op = ops[0]
    _id = "ath|h3r8|882a1072b5fffff|2025-10-04T10:20:00Z"
    start = datetime.datetime(2025, 10, 4, 10, 20)
    end = datetime.datetime(2025, 10, 4, 10, 25)
    assert op._filter == {"_id": _id}
    assert op._upsert is True
    assert op._doc == {"$set": {
        "_id": _id, "city": "ath", "grid": "h3r8", "cellId": "882a1072b5fffff",
        "windowStart": start, "windowEnd": end, "count": 7, "avgSpeedKmh": 21.5,
        "centroid": {"type": "Point", "coordinates": [-71.06, 42.355]},
        "staleAt": end + datetime.timedelta(minutes=45)}}
    # key order of the $set document is the reference's (:176-187)
    assert list(op._doc["$set"]) == ["_id", "city", "grid", "cellId", "windowStart", "windowEnd", "count",
                                     "avgSpeedKmh", "centroid", "staleAt"]


def test_tile_null_coercions_follow_reference():
    # count or 0; avg or 0.0 (null -> 0.0, NaN stays NaN because NaN is truthy; -0.0 -> 0.0 because falsy)
    t = _tiles(cell=[1, 2], ws=[0, 0], avg_speed=[0.0, float("nan")], speed_null=[True, False],
               avg_lat=[-0.0, 1.0], avg_lon=[2.0, -0.0])
    d0, d1 = (op._doc["$set"] for op in stream.tile_ops(t, "ath", 8, 45))
    assert d0["avgSpeedKmh"] == 0.0 and np.isnan(d1["avgSpeedKmh"])
    assert str(d0["centroid"]["coordinates"][1]) == "0.0" and str(d1["centroid"]["coordinates"][0]) == "0.0"


def test_position_document_matches_reference_format():
    cols = dict(provider=pd.Series(["mbta", "mbta"]), vehicleId=pd.Series(["y1", "BUS_1432"]),
                ts_us=np.array([0, 1759573325 * 1_000_000 + 123456]), lat=np.array([0.0, 42.355]),
                lon=np.array([0.0, -71.06]))
    (op,) = stream.position_ops(cols, [1])
    ts = datetime.datetime(2025, 10, 4, 10, 22, 5, 123456)
    assert op._filter == {"_id": "mbta|BUS_1432", "$or": [{"ts": {"$exists": False}}, {"ts": {"$lt": ts}}]}
    assert op._doc == {"$set": {"provider": "mbta", "vehicleId": "BUS_1432", "ts": ts,
                                "loc": {"type": "Point", "coordinates": [-71.06, 42.355]}}}
    assert op._upsert is True
    # BSON datetimes are UTC milliseconds: the microseconds are floored (bson/datetime_ms.py)
    enc = bson.decode(bson.encode({"ts": ts}))
    assert enc["ts"] == datetime.datetime(2025, 10, 4, 10, 22, 5, 123000)


def test_bulk_chunks_of_1000_tiles_first():
    calls = []

    class Sink:
        def bulk_write(self, coll, ops):
            calls.append((coll, len(ops)))

    t = _tiles(cell=list(range(1, 2501)), ws=[0] * 2500)
    stream._flush(Sink(), "tiles", stream.tile_ops(t, "ath", 8, 45))
    assert calls == [("tiles", 1000), ("tiles", 1000), ("tiles", 500)]


@pytest.mark.parametrize("kind", ["pandas", "arrow"])
def test_batch_columns_nulls_and_keys(kind):
    df = pd.DataFrame({
        "provider": ["mbta", "mbta", None, "opensky", "mbta"],
        "vehicleId": ["a", "b", "a", "a", None],
        "lat": [42.3, None, 42.3, 10.0, 42.3],
        "lon": [-71.0, -71.0, -71.0, 20.0, -71.0],
        "speedKmh": pd.Series([10.0, None, 3.0, float("nan"), 1.0], dtype=object),   # null != NaN
        "eventTs": pd.to_datetime(["2025-10-04T10:22:05Z", "2025-10-04T10:22:06Z", None, "2025-10-04T10:22:07.500Z",
                                   "2025-10-04T10:22:08Z"], utc=True, format="ISO8601"),
    })
    src = df if kind == "pandas" else stream._pandas_to_arrow(df)
    c = stream.batch_columns(src)
    assert c["n"] == 5
    assert c["row_valid"].tolist() == [True, True, False, True, False]
    assert np.isnan(c["lat"][1])
    # a null speed is not aggregated (speed_valid 0); a NaN speed is a value (avg -> NaN)
    assert c["speed_valid"].tolist() == [True, False, True, True, True]
    assert np.isnan(c["speed"][3])
    assert c["ts_us"][3] == 1759573327_500000
    k = c["vkey"]
    assert k[0] != k[1] and k[0] != k[3]       # (mbta,a) vs (mbta,b) vs (opensky,a)


def test_nan_speed_is_not_null_at_the_boundary():
    """pandas float64 NaN, Arrow NaN and Arrow null reach the engine as NaN / NaN / null (pa.Table.from_pandas would
    turn the NaNs into nulls, and avg would then skip them instead of yielding NaN)."""
    df = pd.DataFrame({"provider": ["p"] * 3, "vehicleId": ["a", "b", "c"], "lat": [1.0, 2.0, 3.0],
                       "lon": [1.0, 2.0, 3.0], "speedKmh": [np.nan, 5.0, np.nan],
                       "eventTs": pd.to_datetime([1759572000] * 3, unit="s")})
    c = stream.batch_columns(df)
    assert c["speed_valid"].tolist() == [True, True, True] and np.isnan(c["speed"][[0, 2]]).all()
    t = pa.table({"provider": ["p"] * 3, "vehicleId": ["a", "b", "c"], "lat": [1.0, 2.0, 3.0], "lon": [1.0, 2.0, 3.0],
                  "speedKmh": pa.array([float("nan"), None, 4.0], pa.float64()),
                  "eventTs": pa.array([1759572000_000_000] * 3, pa.timestamp("us", tz="UTC"))})
    c = stream.batch_columns(t)
    assert c["speed_valid"].tolist() == [True, False, True] and np.isnan(c["speed"][0])


def test_iso_ts_strings_parse_like_to_timestamp():
    df = pd.DataFrame({"provider": ["p", "p"], "vehicleId": ["v", "w"], "lat": [1.0, 2.0], "lon": [1.0, 2.0],
                       "speedKmh": [1.0, 2.0], "ts": ["2025-09-26T12:45:10Z", "not a time"]})
    c = stream.batch_columns(df)
    assert c["ts_us"][0] == 1758890710 * 1_000_000
    assert c["row_valid"].tolist() == [True, False]


def test_iso_ts_date_only_and_mixed_zones():
    """A date-only string is midnight (UTC session), not a string with a '-15'-style zone; naive, Z and +hh:mm
    strings in one frame each parse on their own (the zone test only after a time component)."""
    df = pd.DataFrame({"provider": ["p"] * 4, "vehicleId": ["v", "w", "x", "y"], "lat": [1.0] * 4, "lon": [1.0] * 4,
                       "speedKmh": [1.0] * 4,
                       "ts": ["2025-09-26T12:45:10Z", "2025-09-26", "2025-09-26T12:45:10+02:00", "2025-09-26T12:45:10"]})
    c = stream.batch_columns(df)
    assert c["ts_us"].tolist() == [1758890710_000_000, 1758844800_000_000, 1758883510_000_000, 1758890710_000_000]
    assert c["row_valid"].tolist() == [True] * 4


def test_state_checkpoint_files_and_resume_choice(tmp_path, monkeypatch):
    """CPU: the state checkpoint's file format round-trips (plain arrays, no pickles) and a restarted engine
    resumes from the state after the newest checkpointed epoch OLDER than the incoming one (Spark re-runs the first
    uncommitted epoch on the state of the one before it, reference heatmap_stream.py:37,244): the newest full
    snapshot before it plus the deltas since, the last-written record of each key winning and windows evicted by the
    last delta's watermark dropped (engine.merge_state)."""
    from mobheat import engine as eng_mod
    from mobheat._lib import STATE_REC_DTYPE
    recs = np.zeros(3, STATE_REC_DTYPE)
    recs["cell"] = [1, 2, 3]
    recs["sum_speed"] = [0.5, np.nan, -1.25]
    info = dict(epoch_id=7, n_keys=3, watermark_ms=11, prev_watermark_ms=10, tile_us=300_000_000,
                watermark_delay_ms=600_000, h3_res=8)
    p = str(tmp_path / "s.mhs")
    eng_mod.save_state_file(p, info, recs, meta='{"lineage": "L"}')
    info2, recs2 = eng_mod.load_state_file(p)
    assert info2 == info and eng_mod.read_state_meta(p) == '{"lineage": "L"}'
    np.testing.assert_array_equal(recs2.view(np.uint8), recs.view(np.uint8))
    # the .npz files of earlier versions still load (and an empty state round-trips)
    legacy = str(tmp_path / "old.npz")
    np.savez(legacy, info=np.array([info[k] for k in eng_mod._INFO_FIELDS], np.int64), recs=recs, meta=np.array("m"))
    info3, recs3 = eng_mod.load_state_file(legacy)
    assert info3 == info and eng_mod.read_state_meta(legacy) == "m"
    np.testing.assert_array_equal(recs3.view(np.uint8), recs.view(np.uint8))
    eng_mod.save_state_file(p, info, recs[:0])
    assert eng_mod.load_state_file(p)[1].size == 0 and eng_mod.read_state_meta(p) is None

    imported = []

    class FakeEngine:
        def __init__(self, **kw):
            pass

        def import_state(self, info, recs):
            imported.append((info, {(int(r["cell"]), int(r["window_start_us"])): int(r["count"]) for r in recs}))

        def close(self):
            pass

    monkeypatch.setattr(stream, "HeatmapEngine", FakeEngine)
    monkeypatch.setattr(stream, "CHECKPOINT_DIR", str(tmp_path))
    monkeypatch.setattr(stream, "STATE_CHECKPOINT", True)
    os.makedirs(stream._state_dir())
    T = 300_000_000
    w0, w1 = 100 * T, 101 * T

    def write(kind, epoch, keys, prev_wm_ms=0, prev=-1, base=None, lineage="A"):
        r = np.zeros(len(keys), STATE_REC_DTYPE)
        for k, (c, w, n) in enumerate(keys):
            r[k]["cell"], r[k]["window_start_us"], r[k]["count"] = c, w, n
        inf = dict(info, epoch_id=epoch, n_keys=len(keys), prev_watermark_ms=prev_wm_ms)
        meta = json.dumps({"lineage": lineage, "base": epoch if base is None else base, "prev": prev})
        name = f"{kind}-{epoch}.r0of1.npz"
        eng_mod.save_state_file(os.path.join(stream._state_dir(), name), inf, r, meta=meta)

    write("state", 3, [(1, w0, 1), (2, w0, 1)])
    write("delta", 4, [(2, w0, 5), (9, w1, 1)], prev=3, base=3)
    write("delta", 5, [(1, w0, 7)], prev=4, base=3)
    write("delta", 6, [(3, w1, 2)], prev_wm_ms=(w0 + T) // 1000, prev=5, base=3)   # w0 evicted by batch 6's watermark
    write("state", 12, [(4, w1, 4)])
    write("delta", 13, [(4, w1, 6), (5, w1, 1)], prev=12, base=12)
    open(os.path.join(stream._state_dir(), "state-x.npz"), "wb").close()
    assert [(e, k) for e, k, _ in stream._checkpoints()] == [(3, "full"), (4, "delta"), (5, "delta"), (6, "delta"),
                                                             (12, "full"), (13, "delta")]
    cases = [(14, {(4, w1): 6, (5, w1): 1}), (13, {(4, w1): 4}), (12, {(3, w1): 2, (9, w1): 1}),
             (6, {(1, w0): 7, (2, w0): 5, (9, w1): 1}), (5, {(1, w0): 1, (2, w0): 5, (9, w1): 1}),
             (4, {(1, w0): 1, (2, w0): 1}), (3, None)]
    for epoch, want in cases:
        stream.reset_engine()
        imported.clear()
        stream.get_engine(epoch)
        assert (imported[0][1] if imported else None) == want, epoch
        if imported:
            assert imported[0][0]["n_keys"] == len(want)
    stream.reset_engine()


def test_state_checkpoint_legacy_files_restore_and_continue(tmp_path, monkeypatch):
    """CPU: checkpoint files in the naming and format of the version before chains were recorded
    (``state-<E>.npz`` / ``delta-<E>.npz``, np.savez of info + recs, no chain record) are restored by that version's rule
    -- the newest snapshot plus every delta after it, in epoch order -- not only from the last snapshot; the stream then
    continues the same chain with the current format, and a restart resumes from the mixed chain."""
    from mobheat import checkpoint as ck
    from mobheat import engine as eng_mod
    from mobheat._lib import STATE_REC_DTYPE
    T = 300_000_000
    w0 = 100 * T
    info = dict(epoch_id=0, n_keys=0, watermark_ms=0, prev_watermark_ms=0, tile_us=T, watermark_delay_ms=600_000,
                h3_res=8)
    root = tmp_path / "mobheat-state"
    root.mkdir()

    def legacy(kind, epoch, keys):
        r = np.zeros(len(keys), STATE_REC_DTYPE)
        for k, (c, n) in enumerate(keys):
            r[k]["cell"], r[k]["window_start_us"], r[k]["count"] = c, w0, n
        inf = dict(info, epoch_id=epoch, n_keys=len(keys))
        np.savez(str(root / f"{kind}-{epoch}.npz"), info=np.array([inf[f] for f in eng_mod._INFO_FIELDS], np.int64),
                 recs=r)

    legacy("state", 0, [(1, 1), (2, 1)])
    legacy("delta", 1, [(2, 4)])
    legacy("delta", 2, [(3, 1)])
    legacy("state", 3, [(1, 1), (2, 4), (3, 1), (4, 2)])
    legacy("delta", 4, [(4, 9)])
    st = ck.StateCheckpoints(str(root))
    got = {}
    for before in (1, 2, 3, 4, 5, 9):
        pt = st.restore_point(before)
        _, recs = st.load(pt)
        got[before] = (pt.epoch, pt.lineage, {int(r["cell"]): int(r["count"]) for r in recs})
    assert got[1] == (0, ck.LEGACY, {1: 1, 2: 1})
    assert got[2] == (1, ck.LEGACY, {1: 1, 2: 4})
    assert got[3] == (2, ck.LEGACY, {1: 1, 2: 4, 3: 1})             # was: the snapshot of epoch 0 only
    assert got[5][2] == got[9][2] == {1: 1, 2: 4, 3: 1, 4: 9}

    class Eng:   # a state of {cell: count}; the batch of epoch 5 touched cell 5
        def export_state(self, reuse=False):
            raise AssertionError("the restored chain continues with a delta")

        def export_state_delta(self, reuse=False):
            r = np.zeros(1, STATE_REC_DTYPE)
            r[0]["cell"], r[0]["window_start_us"], r[0]["count"] = 5, w0, 3
            return dict(info, epoch_id=5, n_keys=1), r

    pt = st.restore_point(5)
    assert st.save(5, Eng(), pt.lineage, full_every=10) == "delta"
    pt = st.restore_point(6)
    _, recs = st.load(pt)
    assert pt.epoch == 5 and {int(r["cell"]): int(r["count"]) for r in recs} == {1: 1, 2: 4, 3: 1, 4: 9, 5: 3}


def test_state_checkpoint_chains_lineage_and_pruning(tmp_path, monkeypatch):
    """CPU: the checkpoint chains (mobheat.checkpoint).  (1) Saves with a snapshot every 2 deltas keep only
    the files from the second-newest snapshot on, and a restart before every epoch restores exactly the state after the
    epoch before it.  (2) A delta whose link is missing, or one of another lineage, is never merged: the restore falls
    back to the newest complete chain, and warns when none exists.  (3) A fresh stream over an older stream's files
    (epochs restarting at 0) deletes them at its first save, so their higher epochs are never resumed."""
    import warnings

    from mobheat import checkpoint as ck
    from mobheat._lib import STATE_REC_DTYPE

    class FakeEngine:
        """A state of {key: count}: export_state = every key, export_state_delta = the keys the last batch touched."""
        info = dict(epoch_id=0, n_keys=0, watermark_ms=0, prev_watermark_ms=0, tile_us=300_000_000,
                    watermark_delay_ms=600_000, h3_res=8)

        def __init__(self, state=None):
            self.state, self.touched = dict(state or {}), set()

        def batch(self, epoch):
            self.touched = {epoch % 5, 100 + epoch}
            for k in self.touched:
                self.state[k] = self.state.get(k, 0) + epoch + 1

        def _recs(self, keys):
            r = np.zeros(len(keys), STATE_REC_DTYPE)
            for i, k in enumerate(sorted(keys)):
                r[i]["cell"], r[i]["window_start_us"], r[i]["count"] = k, 0, self.state[k]
            return dict(self.info, n_keys=len(keys)), r

        def export_state(self, reuse=False):
            return self._recs(self.state)

        def export_state_delta(self, reuse=False):
            return self._recs(self.touched)

    root = str(tmp_path / "st")
    st = ck.StateCheckpoints(root)
    eng, lineage, history = FakeEngine(), ck.new_lineage(), {}
    for epoch in range(9):
        eng.batch(epoch)
        kinds = st.save(epoch, eng, lineage, full_every=2)
        history[epoch] = dict(eng.state)
        assert kinds == ("full" if epoch % 3 == 0 else "delta"), epoch
        files = [(e.epoch, e.kind) for e in st.scan()]
        fulls = [e for e, k in files if k == "full"]
        assert fulls == sorted(fulls)[-2:] and files[0][0] == fulls[0], (epoch, files)   # from the 2nd-newest snapshot
    for before in range(4, 10):
        pt = st.restore_point(before)
        assert pt.epoch == before - 1 and pt.lineage == lineage and pt.world == 1
        info, recs = st.load(pt)
        assert {int(r["cell"]): int(r["count"]) for r in recs} == history[before - 1] and info["n_keys"] == recs.size
    # (2) a broken link: delete delta 7 -> epoch 8's chain is broken, the restore before 9 uses the chain ending at 6
    os.remove(st.path("delta", 7))
    assert st.restore_point(9).epoch == 6
    # a foreign lineage's newer snapshot + delta (an abandoned stream's leftovers in the directory) are not mixed in:
    # only a complete chain of one lineage counts, the newest wins (here the foreign one, complete on its own)
    foreign = FakeEngine({1: 111})
    foreign.touched = {1}
    st2 = ck.StateCheckpoints(root)
    info, r = foreign.export_state()
    from mobheat import engine as eng_mod
    eng_mod.save_state_file(st2.path("full", 20), info, r, meta=json.dumps({"lineage": "B", "base": 20, "prev": -1}))
    eng_mod.save_state_file(st2.path("delta", 21), info, r, meta=json.dumps({"lineage": "C", "base": 20, "prev": 20}))
    pt = st2.restore_point(22)
    assert pt.epoch == 20 and pt.lineage == "B"   # delta 21 names another lineage: its chain is broken
    # (3) a fresh stream (epochs from 0 again) deletes the older files at its first save: no later restore sees them
    fresh, lin2 = FakeEngine(), ck.new_lineage()
    fresh.batch(0)
    st2.save(0, fresh, lin2, full_every=2)
    assert [(e.epoch, e.kind) for e in st2.scan()] == [(0, "full")]
    pt = st2.restore_point(30)
    assert pt.epoch == 0 and pt.lineage == lin2
    # files exist but no complete chain: a warning, and an empty start
    os.remove(st2.path("full", 0))
    eng_mod.save_state_file(st2.path("delta", 5), info, r, meta=json.dumps({"lineage": lin2, "base": 4, "prev": 4}))
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert st2.restore_point(9) is None
    assert any("no complete chain" in str(x.message) for x in w)


def test_state_checkpoint_reshard(tmp_path):
    """CPU: a 3-rank stream's chains restored into 1 and into 2 ranks: each new rank keeps the keys it owns
    (distributed.tile_owner), and the union over the new ranks is the old state exactly."""
    from mobheat import checkpoint as ck
    from mobheat import engine as eng_mod
    from mobheat._lib import STATE_REC_DTYPE
    from mobheat.distributed import tile_owner
    rng = np.random.default_rng(3)
    cells = rng.integers(1, 2 ** 60, 3000).astype(np.uint64)
    ws = (rng.integers(0, 4, 3000) * 300_000_000).astype(np.int64)
    info = dict(epoch_id=5, n_keys=0, watermark_ms=0, prev_watermark_ms=0, tile_us=300_000_000,
                watermark_delay_ms=600_000, h3_res=8)
    old_owner = tile_owner(cells, ws, 3)
    root = str(tmp_path / "st")
    for r in range(3):
        sel = old_owner == r
        recs = np.zeros(int(sel.sum()), STATE_REC_DTYPE)
        recs["cell"], recs["window_start_us"], recs["count"] = cells[sel], ws[sel], np.arange(sel.sum()) + 1
        st = ck.StateCheckpoints(root, r, 3)
        os.makedirs(root, exist_ok=True)
        eng_mod.save_state_file(st.path("full", 5), dict(info, n_keys=recs.size), recs,
                                meta=json.dumps({"lineage": "L", "base": 5, "prev": -1}))
    everything = None
    for world in (1, 2):
        got = []
        for r in range(world):
            st = ck.StateCheckpoints(root, r, world)
            pt = st.restore_point(6)
            assert pt == ck.RestorePoint(5, 3, "L")
            _, recs = st.load(pt, owner=lambda c, w: tile_owner(c, w, world) == r)
            assert (tile_owner(recs["cell"], recs["window_start_us"], world) == r).all()
            got.append(recs)
        u = np.sort(np.concatenate(got), order=["cell", "window_start_us"])
        assert u.size == 3000
        if everything is None:
            everything = u
        np.testing.assert_array_equal(u.view(np.uint8), everything.view(np.uint8))


def _reference_statements(tiles, city, h3_res, ttl_min):
    """What pymongo sends for the reference's tile UpdateOne ops: bson of {q, u, multi: False, upsert: True}
    (pymongo/synchronous/bulk.py add_update), the ops built as heatmap_stream.py:164-188 (stream.tile_ops)."""
    return [bson.encode({"q": op._filter, "u": op._doc, "multi": False, "upsert": True})
            for op in stream.tile_ops(tiles, city=city, h3_res=h3_res, ttl_min=ttl_min)]


def _edge_tiles(rng, n, tile_us, t0_us):
    ws = t0_us + tile_us * rng.integers(-3, 4, n)
    cnt = rng.integers(1, 5000, n)
    cnt[:3] = [2**31 - 1, 2**31, 2**40]                       # int32 / int64 boundary
    sp = rng.uniform(0, 120, n)
    sp[3:6] = [0.0, -0.0, np.nan]
    lon = rng.uniform(-180, 180, n)
    lat = rng.uniform(-90, 90, n)
    lon[6:8] = [-0.0, 0.0]
    lat[8:10] = [-0.0, np.nan]
    cell = rng.integers(0x08000000_00000000, 0x08ffffff_ffffffff, n, dtype=np.uint64)
    cell[10] = 0x1                                           # short hex (not a valid cell: formatting only)
    return TileRows(cell=cell, window_start_us=ws, window_end_us=ws + tile_us, count=cnt, avg_speed=sp,
                    speed_null=rng.random(n) < 0.2, avg_lon=lon, avg_lat=lat)


@pytest.mark.parametrize("tz", ["UTC", "EET-2EEST,M3.5.0/3,M10.5.0/4", "EST+5EDT,M3.2.0/2,M11.1.0/2"])
@pytest.mark.parametrize("h3_res,city,tile_min", [(8, "ath", 5), (12, "αθήνα-" + "x" * 40, 15), (0, "", 1),
                                                  (9, "greater-" * 40 + "αθήνα", 5)])
def test_gpu_statement_encoder_matches_pymongo(tz, h3_res, city, tile_min):
    """CPU: the GPU encoder's code (host execution, hm_selftest_tile_statements) writes exactly the bytes pymongo
    encodes for the reference's UpdateOne ops -- under local time zones with DST transitions inside windows
    (pyspark's naive local datetimes), int32/int64 counts, +-0.0 and NaN averages, null speeds, res 0-15."""
    import time
    from mobheat import _lib
    old = os.environ.get("TZ")
    os.environ["TZ"] = tz
    time.tzset()
    try:
        rng = np.random.default_rng(h3_res)
        tile_us = tile_min * 60_000_000
        # 2025-10-26 00:55 UTC: the EU DST change (01:00 UTC) falls inside a window; 2025-11-02 06:00 UTC: the US one
        t0 = (1761440100 if tz.startswith("EET") else 1762063200) * 1_000_000
        t0 -= t0 % tile_us
        tiles = _edge_tiles(rng, 400, tile_us, t0)
        buf, offs = _lib.tile_statements_selftest(tiles, city, h3_res, 45, tile_us)
        exp = _reference_statements(tiles, city, h3_res, 45)
        assert offs.size == len(exp) + 1
        for i, e in enumerate(exp):
            got = buf[offs[i]:offs[i + 1]].tobytes()
            assert got == e, (i, bson.decode(got), bson.decode(e))
    finally:
        if old is None:
            del os.environ["TZ"]
        else:
            os.environ["TZ"] = old
        time.tzset()


def test_statement_batches_and_update_command(monkeypatch):
    """CPU: GPU-encoded statements go out in unordered `update` commands of <= 1000 (reference :191-196); the
    command is the one pymongo's bulk_write sends, and write errors raise BulkWriteError like bulk_write does."""
    from bson.raw_bson import RawBSONDocument
    from pymongo.errors import BulkWriteError
    from mobheat import _lib
    t = _edge_tiles(np.random.default_rng(5), 2500, 300_000_000, 1759572000_000_000)
    buf, offs = _lib.tile_statements_selftest(t, "ath", 8, 45, 300_000_000)
    cmds = []

    class DB:
        reply = {"ok": 1, "n": 0}

        def command(self, cmd):
            cmds.append(bson.decode(bson.encode(cmd)))       # encodable with the raw statements inside
            return DB.reply

    sink = stream.MongoSink.__new__(stream.MongoSink)   # the pymongo path (a URI with options or credentials)
    sink._db = DB()
    sink._wire = sink._client = None
    stream._flush_statements(sink, "tiles", buf, offs)
    assert [len(c["updates"]) for c in cmds] == [1000, 1000, 500]
    assert all(list(c) == ["update", "updates", "ordered"] and c["update"] == "tiles" and c["ordered"] is False for c in cmds)
    exp = _reference_statements(t, "ath", 8, 45)
    got = [bson.encode(u) for c in cmds for u in c["updates"]]
    assert got == exp
    DB.reply = {"ok": 1, "n": 1, "writeErrors": [{"index": 0, "code": 11000, "errmsg": "dup"}]}
    with pytest.raises(BulkWriteError):
        sink.update_raw("tiles", [RawBSONDocument(exp[0])])


@pytest.mark.parametrize("tz", ["UTC", "EET-2EEST,M3.5.0/3,M10.5.0/4"])
def test_gpu_position_encoder_matches_pymongo(tz):
    """CPU: the positions statement encoder (host execution of the GPU code) writes the bytes pymongo encodes for
    the reference's positions_latest UpdateOne (heatmap_stream.py:211-228): string dictionaries from the batch's
    factorization (non-ASCII ids, two providers), naive local eventTs with microseconds across a DST change."""
    import time
    from mobheat import _lib
    old = os.environ.get("TZ")
    os.environ["TZ"] = tz
    time.tzset()
    try:
        rng = np.random.default_rng(9)
        n = 3000
        t0 = 1761440100 * 1_000_000 - 3 * 3600 * 1_000_000
        df = pd.DataFrame({"provider": rng.choice(["mbta", "opensky-ψ"], n),
                           "vehicleId": [f"v{int(x)}-ώ" if x % 7 == 0 else f"BUS_{int(x)}" for x in rng.integers(0, 800, n)],
                           "lat": rng.uniform(-90, 90, n), "lon": rng.uniform(-180, 180, n),
                           "speedKmh": rng.uniform(0, 90, n),
                           "eventTs": pd.to_datetime(t0 + rng.integers(0, 6 * 3600 * 1_000_000, n), unit="us")})
        df.loc[5, "lat"] = -0.0
        cols = stream.batch_columns(df)
        rows = np.sort(rng.choice(n, 500, replace=False))
        buf, offs = _lib.position_statements_selftest(cols["provider_uniques"], cols["vehicle_uniques"],
                                                      cols["vkey"][rows], cols["ts_us"][rows], cols["lat"][rows],
                                                      cols["lon"][rows])
        exp = [bson.encode({"q": op._filter, "u": op._doc, "multi": False, "upsert": True})
               for op in stream.position_ops(cols, rows)]
        assert offs.size == len(exp) + 1
        for i, e in enumerate(exp):
            got = buf[offs[i]:offs[i + 1]].tobytes()
            assert got == e, (i, bson.decode(got), bson.decode(e))
    finally:
        if old is None:
            del os.environ["TZ"]
        else:
            os.environ["TZ"] = old
        time.tzset()


@pytest.mark.parametrize("tz", ["UTC", "EST+5EDT,M3.2.0/2,M11.1.0/2"])
def test_position_encoder_wide_time_span(tz):
    """A batch whose latest rows mix a default GPS time (1970-01-01, before the epoch too) with current traffic
    and a far-future row: only the 900-s buckets the rows use are looked up (no dense span table), and every
    statement equals pymongo's bytes for the reference's positions_latest op (heatmap_stream.py:211-228)."""
    import time
    from mobheat import _lib
    old = os.environ.get("TZ")
    os.environ["TZ"] = tz
    time.tzset()
    try:
        ts = np.array([0, -1, 1_000_000 * 86400 * 20000 + 123456, 1759572000_000_000 + 999_999,
                       1759572000_000_000 + 7 * 900_000_000, 4102444800_000_000], np.int64)
        n = ts.size
        df = pd.DataFrame({"provider": ["mbta"] * n, "vehicleId": [f"v{i}" for i in range(n)],
                           "lat": np.linspace(-60, 60, n), "lon": np.linspace(-170, 170, n), "speedKmh": [1.0] * n,
                           "eventTs": pd.to_datetime(ts, unit="us")})
        cols = stream.batch_columns(df)
        rows = np.arange(n)
        ids, offs_s = _lib.time_buckets(cols["ts_us"][rows])
        assert ids.size == 6 and np.all(np.diff(ids) > 0)   # (-1 us lies in bucket -1)
        buf, offs = _lib.position_statements_selftest(cols["provider_uniques"], cols["vehicle_uniques"],
                                                      cols["vkey"][rows], cols["ts_us"][rows], cols["lat"][rows],
                                                      cols["lon"][rows])
        exp = [bson.encode({"q": op._filter, "u": op._doc, "multi": False, "upsert": True})
               for op in stream.position_ops(cols, rows)]
        assert [buf[offs[i]:offs[i + 1]].tobytes() for i in range(n)] == exp
    finally:
        if old is None:
            del os.environ["TZ"]
        else:
            os.environ["TZ"] = old
        time.tzset()


@pytest.mark.parametrize("checkpoint", [True, False])
def test_failed_writes_and_replays_do_not_merge_twice(tmp_path, monkeypatch, checkpoint):
    """CPU, host logic of foreach_batch_func (reference heatmap_stream.py:150-249: an exception fails the batch and
    Spark re-runs the epoch), with and without state checkpoints:
      * a batch whose Mongo writes fail keeps its merged state; the re-run of that epoch writes the same documents
        again without merging twice;
      * an error before the merge (the state version unchanged: a decode error, a bad argument) keeps the engine;
      * an error after the merge began drops the state; the retry rebuilds it from the checkpoints;
      * an epoch the live engine already committed is re-run on the state of the epoch before it."""
    from mobheat import engine as eng_mod
    from mobheat._lib import STATE_REC_DTYPE
    monkeypatch.setenv("MOBHEAT_COLUMNS", "host")   # (the fake engine takes host columns)
    created, merged = [], []
    mode = {"fail_write": False, "fail_before": False, "fail_during": False}

    class FakeEngine:
        def __init__(self, **kw):
            self.epochs = []
            self.version = 0
            created.append(self)

        def state_version(self):
            return self.version

        def import_state(self, info, recs):
            self.epochs.append(("restored", int(info["epoch_id"])))

        def process_batch(self, epoch_id, *a, **kw):
            if mode["fail_before"]:
                raise RuntimeError("bad input")
            self.version += 1
            if mode["fail_during"]:
                raise RuntimeError("device fault")
            self.epochs.append(epoch_id)
            merged.append(epoch_id)

            class R:
                latest_rows = np.zeros(0, np.int64)
                n_latest = 0
            return R()

        def encode_tile_updates(self, city, ttl):
            doc = np.frombuffer(bson.encode({"q": {"_id": "x"}}), np.uint8)
            return doc, np.array([0, doc.size], np.int64)

        def _info(self):
            return dict(epoch_id=self.epochs[-1] if self.epochs and isinstance(self.epochs[-1], int) else -1, n_keys=0,
                        watermark_ms=0, prev_watermark_ms=0, tile_us=300_000_000, watermark_delay_ms=600_000, h3_res=8)

        def export_state(self, reuse=False):
            return self._info(), np.zeros(0, STATE_REC_DTYPE)

        def export_state_delta(self, reuse=False):
            return self._info(), np.zeros(0, STATE_REC_DTYPE)

        def close(self):
            pass

    writes = []

    class Sink:
        def update_raw(self, coll, statements):
            if mode["fail_write"]:
                raise IOError("mongo down")
            writes.append(coll)

        def close(self):
            pass

    monkeypatch.setattr(stream, "HeatmapEngine", FakeEngine)
    monkeypatch.setattr(stream, "SINK_FACTORY", Sink)
    monkeypatch.setattr(stream, "CHECKPOINT_DIR", str(tmp_path))
    monkeypatch.setattr(stream, "STATE_CHECKPOINT", checkpoint)
    df = pd.DataFrame({"provider": ["p"], "vehicleId": ["v"], "lat": [1.0], "lon": [2.0], "speedKmh": [3.0],
                       "eventTs": pd.to_datetime([1759572000], unit="s")})
    stream.reset_engine()
    stream.foreach_batch_func(df, 0)
    stream.foreach_batch_func(df, 1)
    assert len(created) == 1 and created[0].epochs == [0, 1]
    # writes fail: the merged state stays, the re-run writes again without a second merge
    mode["fail_write"] = True
    with pytest.raises(IOError):
        stream.foreach_batch_func(df, 2)
    assert stream._ENGINE is created[0] and merged == [0, 1, 2]
    mode["fail_write"] = False
    n_w = len(writes)
    stream.foreach_batch_func(df, 2)
    assert merged == [0, 1, 2] and len(created) == 1 and len(writes) == n_w + 1
    # an error before the merge keeps the engine
    mode["fail_before"] = True
    with pytest.raises(RuntimeError):
        stream.foreach_batch_func(df, 3)
    assert stream._ENGINE is created[0]
    mode["fail_before"] = False
    stream.foreach_batch_func(df, 3)
    assert created[0].epochs == [0, 1, 2, 3] and len(created) == 1
    # an error during the merge drops the state; the retry rebuilds it
    mode["fail_during"] = True
    with pytest.raises(RuntimeError):
        stream.foreach_batch_func(df, 4)
    assert stream._ENGINE is None
    mode["fail_during"] = False
    stream.foreach_batch_func(df, 4)
    assert len(created) == 2
    assert created[1].epochs == ([("restored", 3), 4] if checkpoint else [4])
    # a replay of a committed epoch in the same process: the state of the epoch before it, then the batch once
    stream.foreach_batch_func(df, 4)
    assert len(created) == 3 and created[2].epochs == ([("restored", 3), 4] if checkpoint else [4])
    if checkpoint:
        kinds = [(e, k) for e, k, _ in stream._checkpoints()]
        assert kinds[0] == (0, "full") and all(k == "delta" for _, k in kinds[1:])
    stream.reset_engine()


def test_wire_op_msg_equals_pymongo_and_fake_server():
    """The wire sink's OP_MSG for a chunk of GPU-encoded statements is byte-identical to the message pymongo builds
    for the same update command (message._op_msg: section 0 {update, ordered, $db}, section 1 the `updates`
    sequence); through a fake server on a local socket, chunks of <= 1000 statements arrive intact and write errors
    raise BulkWriteError like bulk_write (reference heatmap_stream.py:191-196)."""
    import socket
    import struct
    import threading
    from bson.codec_options import DEFAULT_CODEC_OPTIONS
    from bson.raw_bson import RawBSONDocument
    from bson.son import SON
    from pymongo import message
    from pymongo.errors import BulkWriteError
    from mobheat import _lib, wire
    t = _edge_tiles(np.random.default_rng(6), 2300, 300_000_000, 1759572000_000_000)
    buf, offs = _lib.tile_statements_selftest(t, "ath", 8, 45, 300_000_000)
    exp = _reference_statements(t, "ath", 8, 45)
    docs = [RawBSONDocument(e) for e in exp[:1000]]
    rid, msg, _, _ = message._op_msg(0, SON([("update", "tiles"), ("updates", docs), ("ordered", False)]), "mobility",
                                     None, DEFAULT_CODEC_OPTIONS)
    mine = b"".join(bytes(p) for p in wire.op_msg_parts(rid, wire.command_doc("tiles", "mobility"),
                                                          memoryview(buf)[:int(offs[1000])]))
    assert mine == msg
    assert wire.chunks(offs, 10**9) == [(0, 1000), (1000, 2000), (2000, 2300)]
    assert wire.chunks(np.array([0, 10, 20, 30, 200]), 25, 1000) == [(0, 2), (2, 3), (3, 4)]
    assert wire.plain_uri("mongodb://127.0.0.1:27017") == ("127.0.0.1", 27017, None)
    assert wire.plain_uri("mongodb://u:p@h/db") is None and wire.plain_uri("mongodb://h/?tls=true") is None

    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    got, fail_on = [], {"chunk": None}

    def serve():
        c, _ = srv.accept()
        k = 0
        while True:
            h = c.recv(16, socket.MSG_WAITALL)
            if len(h) < 16:
                break
            length, rqid, _, op = struct.unpack("<iiii", h)
            body = c.recv(length - 16, socket.MSG_WAITALL)
            clen = struct.unpack_from("<i", body, 5)[0]
            cmd = bson.decode(body[5:5 + clen])
            p = 5 + clen
            assert body[p] == 1
            slen = struct.unpack_from("<i", body, p + 1)[0]
            ident_end = body.index(b"\x00", p + 5)
            assert body[p + 5:ident_end] == b"updates"
            seq = body[ident_end + 1:p + 1 + slen]
            n = 0
            while seq:
                dl = struct.unpack_from("<i", seq, 0)[0]
                got.append(seq[:dl])
                seq = seq[dl:]
                n += 1
            assert cmd == {"update": "tiles", "ordered": False, "$db": "mobility"} and n <= 1000
            reply = {"ok": 1, "n": n}
            if k == fail_on["chunk"]:
                reply["writeErrors"] = [{"index": 0, "code": 11000, "errmsg": "E11000 duplicate key"}]
            rb = bson.encode(reply)
            c.sendall(struct.pack("<iiiiI", 16 + 5 + len(rb), 99, rqid, 2013, 0) + b"\x00" + rb)
            k += 1
        c.close()

    th = threading.Thread(target=serve, daemon=True)
    th.start()
    sink = wire.WireMongoSink("127.0.0.1", srv.getsockname()[1], "mobility")
    sink.update_statements("tiles", buf, offs)
    assert got == exp
    fail_on["chunk"] = 3
    with pytest.raises(BulkWriteError):
        sink.update_statements("tiles", buf, offs[:11])
    sink.close()
    th.join(5)
    srv.close()


def test_batch_columns_nullable_float_keeps_nulls_apart_from_nan():
    """A pandas nullable Float64 speedKmh column: pd.NA is a null speed (not counted by avg, Spark's null) and a NaN is
    a NaN value (propagates into avg), as Spark's JSON reader gives them.  (Round 4: NA became NaN
    through to_numpy(), turning every avgSpeedKmh of a tile with a missing speed into NaN.)"""
    sp = pd.arrays.FloatingArray(np.array([1.5, 0.0, np.nan, 4.0]), np.array([False, True, False, False]))
    df = pd.DataFrame({"provider": ["p"] * 4, "vehicleId": ["a", "b", "c", "d"], "lat": [1.0] * 4, "lon": [2.0] * 4,
                       "speedKmh": sp, "eventTs": pd.to_datetime([1759572000] * 4, unit="s")})
    c = stream.batch_columns(df)
    assert c["speed_valid"].tolist() == [True, False, True, True]
    assert c["speed"][0] == 1.5 and np.isnan(c["speed"][2]) and c["speed"][3] == 4.0
    # nullable integer and string columns too (mask = null)
    df2 = df.assign(lat=pd.array([1, None, 3, 4], dtype="Int64"), vehicleId=pd.array(["a", None, "c", "d"], dtype="string"))
    c2 = stream.batch_columns(df2)
    assert np.isnan(c2["lat"][1]) and c2["lat"][2] == 3.0
    assert c2["row_valid"].tolist() == [True, False, True, True]
