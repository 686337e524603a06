"""GPU: tile-state checkpoint and restore.

The reference keeps the windowed aggregation's state in Spark's state store under
`.option("checkpointLocation", CHECKPOINT_DIR)` (reference heatmap_stream.py:37,244); after a restart Spark
re-runs the first uncommitted epoch on the state of the epoch before it.  Here the state lives on the GPU:
hm_state_export / hm_state_import (include/mobheat.h) dump and restore it.  Bar: a stream interrupted after
any batch and resumed from the checkpoint emits what the uninterrupted stream emits (keys, counts and rows exact,
averages within 1e-9 relative), and both agree with the oracle (tests/test_gpu_parity.py's tolerance on averages).
"""
import numpy as np
import pytest

from test_gpu_parity import _close, assert_batch_equal

pytestmark = pytest.mark.gpu

T0 = 1_759_572_000_000_000
MINUTE = 60_000_000


def _batches(seed=31):
    rng = np.random.default_rng(seed)
    out = []
    for start_min, span_min, n in [(0, 7, 20000), (5, 6, 20000), (0, 0, 0), (14, 9, 30000), (1, 30, 30000),
                                   (40, 3, 5000), (0, 0, 0), (55, 2, 5000)]:
        ts = T0 + start_min * MINUTE + rng.integers(0, max(span_min, 1) * MINUTE, n)
        out.append(dict(lat=rng.uniform(37.90, 38.05, n), lon=rng.uniform(23.60, 23.85, n), ts_us=ts,
                        speed=rng.uniform(0, 90, n), speed_valid=rng.random(n) > 0.2,
                        vkey=rng.integers(0, 500, n).astype(np.uint64), row_valid=rng.random(n) > 0.01))
    return out


def _same(a, b):
    """Two engine results: keys, counts, null flags, latest rows and watermarks exact; averages within the parity
    tolerance (k_ingest's LDS pre-aggregation adds a tile's rows in a scheduling-dependent order)."""
    ka = np.lexsort((a.tiles.window_start_us, a.tiles.cell))
    kb = np.lexsort((b.tiles.window_start_us, b.tiles.cell))
    for f in ("cell", "window_start_us", "count", "speed_null"):
        np.testing.assert_array_equal(getattr(a.tiles, f)[ka], getattr(b.tiles, f)[kb])
    for f in ("avg_speed", "avg_lon", "avg_lat"):
        x, y = getattr(a.tiles, f)[ka], getattr(b.tiles, f)[kb]
        bad = [i for i in range(x.size) if not _close(float(x[i]), float(y[i]))]
        assert not bad, (f, len(bad), x[bad[0]], y[bad[0]])
    np.testing.assert_array_equal(a.latest_rows, b.latest_rows)
    assert (a.n_state, a.watermark_ms, a.late_watermark_ms, a.n_late) == \
        (b.n_state, b.watermark_ms, b.late_watermark_ms, b.n_late)


@pytest.mark.parametrize("cut", [0, 1, 3, 4])
def test_resume_from_checkpoint_matches_uninterrupted(cut, tmp_path):
    from mobheat import HeatmapEngine
    from oracle.spark_oracle import SparkHeatmapOracle
    bs = _batches()
    full = HeatmapEngine(h3_res=9)
    ora = SparkHeatmapOracle(h3_res=9)
    ref = []
    for e, b in enumerate(bs):
        r = full.process_batch(e, **b)
        assert_batch_equal(r, ora.process_batch(**b))
        ref.append(r)
    full.close()

    first = HeatmapEngine(h3_res=9)
    for e in range(cut + 1):
        first.process_batch(e, **bs[e])
    path = str(tmp_path / f"state-{cut}.npz")
    info = first.save_state(path)
    assert info["epoch_id"] == cut and info["n_keys"] == ref[cut].n_state
    first.close()

    resumed = HeatmapEngine(h3_res=9)
    resumed.load_state(path)
    for e in range(cut + 1, len(bs)):
        _same(resumed.process_batch(e, **bs[e]), ref[e])
    resumed.close()


def test_export_matches_oracle_state_and_round_trips():
    from mobheat import HeatmapEngine
    from oracle.spark_oracle import SparkHeatmapOracle
    bs = _batches(seed=32)
    eng = HeatmapEngine(h3_res=9)
    ora = SparkHeatmapOracle(h3_res=9)
    for e in range(5):
        eng.process_batch(e, **bs[e])
        ora.process_batch(**bs[e])
    info, recs = eng.export_state()
    assert info["n_keys"] == len(ora.state) == recs.size > 0
    assert info["watermark_ms"] == ora.wm_cur and info["prev_watermark_ms"] == ora.wm_prev
    assert not recs["reserved"].any()
    for r in recs:
        c, nsp, ssp, sla, slo = ora.state[(int(r["cell"]), int(r["window_start_us"]))]
        assert (int(r["count"]), int(r["n_speed"])) == (c, nsp)
        assert _close(float(r["sum_speed"]), ssp) and _close(float(r["sum_lat"]), sla) and _close(float(r["sum_lon"]), slo)
    # import -> export gives the same records (another order)
    eng2 = HeatmapEngine(h3_res=9)
    eng2.import_state(info, recs)
    info2, recs2 = eng2.export_state()
    assert info2 == info
    np.testing.assert_array_equal(np.sort(recs), np.sort(recs2))
    eng.close()
    eng2.close()


def test_large_state_round_trip_res12():
    """~1.5e6 keys over 6 windows (tables of 2^22 slots): restore, then a batch on top, bit-exact."""
    from mobheat import HeatmapEngine
    rng = np.random.default_rng(33)
    n = 2_000_000

    def batch(k):
        return dict(lat=rng.uniform(37.90, 38.05, n), lon=rng.uniform(23.60, 23.85, n),
                    ts_us=T0 + k * 10 * MINUTE + rng.integers(0, 30 * MINUTE, n), speed=rng.uniform(0, 90, n),
                    speed_valid=rng.random(n) > 0.1, vkey=rng.integers(0, 100000, n).astype(np.uint64), row_valid=None)
    b0, b1 = batch(0), batch(1)
    a = HeatmapEngine(h3_res=12)
    a.process_batch(0, **b0)
    info, recs = a.export_state()
    assert recs.size > 1_000_000
    ra = a.process_batch(1, **b1)
    b = HeatmapEngine(h3_res=12)
    b.import_state(info, recs)
    _same(b.process_batch(1, **b1), ra)
    a.close()
    b.close()


def test_import_errors():
    from mobheat import HeatmapEngine
    bs = _batches(seed=34)
    a = HeatmapEngine(h3_res=9)
    a.process_batch(0, **bs[0])
    info, recs = a.export_state()
    with pytest.raises(RuntimeError, match="already processed"):
        a.import_state(info, recs)                       # not a fresh context
    with pytest.raises(RuntimeError, match="does not match"):
        HeatmapEngine(h3_res=8).import_state(info, recs)   # another resolution
    bad = recs.copy()
    bad["window_start_us"][0] += 1                        # not a window start
    with pytest.raises(RuntimeError, match="malformed"):
        HeatmapEngine(h3_res=9).import_state(info, bad)
    bad = recs.copy()
    bad["reserved"][-1] = 7
    with pytest.raises(RuntimeError, match="malformed"):
        HeatmapEngine(h3_res=9).import_state(info, bad)
    a.close()


def test_incremental_checkpoint_equals_full_export():
    """hm_state_export_touched after every batch (Spark's per-version delta files): a full export of batch 0 merged
    with the deltas since (engine.merge_state: last write wins, windows evicted by the watermark dropped) equals the
    full export after every later batch, record for record (cumulative counts and fp64 sums bit for bit)."""
    from mobheat import HeatmapEngine
    from mobheat.engine import merge_state
    eng = HeatmapEngine(h3_res=9)
    base, deltas = None, []

    def keyed(recs):
        o = np.lexsort((recs["window_start_us"], recs["cell"]))
        return recs[o]
    for e, b in enumerate(_batches(seed=37)):
        eng.process_batch(e, **b)
        if base is None:
            base = eng.export_state()
            continue
        deltas.append(eng.export_state_delta())
        info, recs = merge_state(base, deltas)
        finfo, frecs = eng.export_state()
        assert info == finfo, e
        assert keyed(recs).tobytes() == keyed(frecs).tobytes(), e
    assert sum(d[1].size for d in deltas) > 0
    eng.close()


@pytest.mark.parametrize("full_every", [10, 2])
def test_foreach_batch_func_restart_replays_epoch(tmp_path, monkeypatch, full_every):
    """foreach_batch_func with its default state checkpoints (a full snapshot, then per-batch deltas): a restart (new
    engine) resumes from the state after the newest checkpointed epoch older than the incoming one -- also when that
    epoch itself was already checkpointed (crash before Spark's commit log) -- and emits the same documents as the
    uninterrupted stream."""
    import pandas as pd
    from mobheat import stream

    class Capture:
        ops = []

        def bulk_write(self, coll, ops):
            Capture.ops.extend((coll, op._filter["_id"], op._doc) for op in ops)

        def update_raw(self, coll, stmts):
            import bson
            Capture.ops.extend((coll, d["q"]["_id"], d["u"]) for d in (bson.decode(st.raw) for st in stmts))

        def close(self):
            pass

    def frame(b):
        return pd.DataFrame({"provider": ["p"] * len(b["lat"]), "vehicleId": [f"v{int(v)}" for v in b["vkey"]],
                             "lat": b["lat"], "lon": b["lon"],
                             "speedKmh": np.where(b["speed_valid"], b["speed"], np.nan),
                             "eventTs": pd.to_datetime(b["ts_us"], unit="us")})
    raw = _batches(seed=35)
    bs = [frame(raw[i]) for i in (0, 1, 3, 4, 5)]   # (index 2 is an empty batch)
    monkeypatch.setattr(stream, "SINK_FACTORY", Capture)
    monkeypatch.setattr(stream, "CHECKPOINT_DIR", str(tmp_path))
    monkeypatch.setattr(stream, "STATE_CHECKPOINT", True)
    monkeypatch.setattr(stream, "STATE_FULL_EVERY", full_every)

    def run(epochs):
        out = []
        for e in epochs:
            Capture.ops = []
            stream.foreach_batch_func(bs[e], e)
            # exact fields: ids, cumulative counts, latest timestamps (averages: test_resume_from_checkpoint_*)
            out.append(sorted((c, i, d["$set"].get("count"), str(d["$set"].get("ts"))) for c, i, d in Capture.ops))
        return out

    stream.reset_engine()
    monkeypatch.setattr(stream, "STATE_CHECKPOINT", False)
    ref = run(range(5))
    monkeypatch.setattr(stream, "STATE_CHECKPOINT", True)
    stream.reset_engine()
    got = run(range(3))                                    # epochs 0..2 committed: a snapshot, then deltas
    assert [(e, k) for e, k, _ in stream._checkpoints()] == [(0, "full"), (1, "delta"), (2, "delta")]
    stream.reset_engine()                                  # restart; Spark replays epoch 2 (its commit was lost)
    got += run([2, 3, 4])
    stream.reset_engine()
    assert got[:3] == ref[:3] and got[3:] == ref[2:]


def test_foreach_batch_func_failed_writes_without_checkpoints(monkeypatch):
    """Checkpoints off: a batch whose writes fail keeps its merged GPU state, and Spark's re-run of the epoch writes the
    same documents again without merging the batch twice -- the stream then continues exactly like an uninterrupted
    one (one transient Mongo error no longer discards the tile state)."""
    import pandas as pd
    from mobheat import stream

    class Capture:
        ops = []
        fail = False

        def update_raw(self, coll, stmts):
            import bson
            if Capture.fail:
                raise IOError("mongo down")
            Capture.ops.extend((coll, d["q"]["_id"], d["u"]) for d in (bson.decode(st.raw) for st in stmts))

        def close(self):
            pass

    raw = _batches(seed=36)
    bs = [pd.DataFrame({"provider": ["p"] * len(b["lat"]), "vehicleId": [f"v{int(v)}" for v in b["vkey"]],
                        "lat": b["lat"], "lon": b["lon"], "speedKmh": np.where(b["speed_valid"], b["speed"], np.nan),
                        "eventTs": pd.to_datetime(b["ts_us"], unit="us")}) for b in (raw[0], raw[1], raw[3], raw[4])]
    monkeypatch.setattr(stream, "SINK_FACTORY", Capture)
    monkeypatch.setattr(stream, "STATE_CHECKPOINT", False)

    def run(plan):
        out = []
        for e, fail in plan:
            Capture.ops, Capture.fail = [], fail
            if fail:
                with pytest.raises(IOError):
                    stream.foreach_batch_func(bs[e], e)
                continue
            stream.foreach_batch_func(bs[e], e)
            out.append(sorted((c, i, d["$set"].get("count"), str(d["$set"].get("ts"))) for c, i, d in Capture.ops))
        return out
    stream.reset_engine()
    ref = run([(0, False), (1, False), (2, False), (3, False)])
    stream.reset_engine()
    got = run([(0, False), (1, True), (1, True), (1, False), (2, False), (3, False)])
    stream.reset_engine()
    assert got == ref


def test_shard_import_rejects_foreign_keys():
    """a shard context (rank r of W: tables over its own region fields only) refuses to import a record that
    another rank owns (distributed.tile_owner) -- its slot index would fall below the table -- and imports its own."""
    import mobheat
    from mobheat._lib import STATE_REC_DTYPE
    from mobheat.distributed import tile_owner
    W = 4
    ws = (T0 // 300_000_000) * 300_000_000
    cells = np.array([0x8828308281fffff + (k << 12) for k in range(64)], np.uint64)
    own = tile_owner(cells, np.full(cells.size, ws, np.int64), W)
    assert (own == 1).any() and (own != 1).any()
    info = dict(epoch_id=3, n_keys=0, watermark_ms=0, prev_watermark_ms=0, tile_us=300_000_000,
                watermark_delay_ms=600_000, h3_res=8)

    def recs(sel):
        r = np.zeros(int(sel.sum()), STATE_REC_DTYPE)
        r["cell"], r["window_start_us"], r["count"], r["n_speed"] = cells[sel], ws, 2, 1
        return r
    eng = mobheat.HeatmapEngine(h3_res=8, device=0, shard=(1, W))
    try:
        with pytest.raises(RuntimeError, match="belongs to rank"):
            eng.import_state(dict(info, n_keys=int(cells.size)), recs(np.ones(cells.size, bool)))
    finally:
        eng.close()
    eng = mobheat.HeatmapEngine(h3_res=8, device=0, shard=(1, W))
    try:
        mine = recs(own == 1)
        eng.import_state(dict(info, n_keys=mine.size), mine)
        _, back = eng.export_state()
        assert sorted(back["cell"].tolist()) == sorted(mine["cell"].tolist())
    finally:
        eng.close()


def test_export_begin_copy_equals_exports_and_runs_beside_encode(tmp_path):
    """hm_state_export_begin / _copy (the checkpoint writer's two halves): the dump copied slice by slice equals
    hm_state_export / hm_state_export_touched record for record (as sets), the copies (enqueued up front, waited for
    slice by slice -- and the synchronous hm_state_export_copy) landing on a thread while the batch's tile statements
    are encoded on this engine's stream give the same statements as an encode alone; a copy outside the dump, or
    after another batch, is refused; the streamed file (save_state_file with fill / raw, O_DIRECT where the file system
    takes it) reads back the same records."""
    import threading
    from mobheat import HeatmapEngine, _lib
    from mobheat.engine import STATE_REC_DTYPE, load_state_file, save_state_file
    lib = _lib.load()
    bs = _batches(seed=33)
    eng = HeatmapEngine(h3_res=9)
    try:
        for e in range(4):
            eng.process_batch(e, **bs[e])
        ref_full = eng.export_state()
        ref_delta = eng.export_state_delta()
        ref_stm, ref_offs = eng.encode_tile_updates("ath", 45, copy=True)
        for touched, (rinfo, rrecs) in ((False, ref_full), (True, ref_delta)):
            info, n, recs, raw, fill = eng.export_begin(touched_only=touched, slice_records=997)
            assert info == rinfo and n == rrecs.size > 0
            sync = np.zeros(n, STATE_REC_DTYPE)
            got = {}

            def copier():
                for lo in range(0, n, 1500):
                    fill(lo, min(1500, n - lo))
                    _lib.check(lib.hm_state_export_copy(eng._ctx, sync[lo:].ctypes.data, lo, min(1500, n - lo)),
                               eng._ctx, "hm_state_export_copy")
                got["done"] = True
            th = threading.Thread(target=copier)
            th.start()
            stm, offs = eng.encode_tile_updates("ath", 45, copy=True)
            th.join()
            assert got.get("done")
            np.testing.assert_array_equal(np.sort(recs), np.sort(rrecs))
            np.testing.assert_array_equal(sync, recs)
            assert stm.tobytes() == ref_stm.tobytes() and np.array_equal(offs, ref_offs)
            with pytest.raises(RuntimeError, match="outside the dump"):
                fill(n - 1, 2)
            with pytest.raises(RuntimeError, match="outside the dump"):
                _lib.check(lib.hm_state_export_copy(eng._ctx, sync.ctypes.data, n - 1, 2), eng._ctx, "x")
            path = str(tmp_path / f"s{int(touched)}.mhs")
            info, n, recs, raw, fill = eng.export_begin(touched_only=touched)
            save_state_file(path, info, recs, meta="{}", fill=fill, raw=raw)
            i2, r2 = load_state_file(path)
            assert i2 == rinfo
            np.testing.assert_array_equal(np.sort(r2), np.sort(rrecs))
        eng.process_batch(4, **bs[4])
        buf = np.zeros(1, STATE_REC_DTYPE)
        for call in (lambda: lib.hm_state_export_copy(eng._ctx, buf.ctypes.data, 0, 1),
                     lambda: lib.hm_state_export_copy_async(eng._ctx, buf.ctypes.data, 0, 1, 0)):
            with pytest.raises(RuntimeError, match="without an hm_state_export_begin"):
                _lib.check(call(), eng._ctx, "x")
    finally:
        eng.close()
