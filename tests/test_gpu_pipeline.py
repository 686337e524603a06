"""GPU parity of the pipelined micro-batch (csrc/host_pipe.h): a binned batch split into K chunks,
each chunk's k_ingest<true> overlapping the previous chunk's k_merge_owned on a second stream, a key touched by several
chunks rewriting its one update-mode row in place -- against the oracle (reference heatmap_stream.py:112-133,200-207,
243), and statement for statement against the same batches run unpipelined (MOBHEAT_PIPELINE=0).

MOBHEAT_PIPELINE=K forces K chunks on every binned batch (MOBHEAT_INGEST_MODE=binned bins batches of any size), so the
chunk boundaries, the per-chunk exception ranges, the first chunk's key sample, tables sized from a partial census
(a window first seen in a later chunk, a table grown inside the batch) and the slab-overflow fallback all run at
test sizes.
"""
import numpy as np
import pytest

from test_gpu_parity import _run, assert_batch_equal

pytestmark = pytest.mark.gpu
MINUTE = 60_000_000


def _engine(monkeypatch, res, chunks, sub=None, **kw):
    from mobheat import HeatmapEngine
    monkeypatch.setenv("MOBHEAT_INGEST_MODE", "binned")
    monkeypatch.setenv("MOBHEAT_PIPELINE", str(chunks))
    if sub is not None:
        monkeypatch.setenv("MOBHEAT_SUBBINS", sub)
    return HeatmapEngine(h3_res=res, **kw)


@pytest.mark.parametrize("chunks,sub", [(2, "0"), (4, "0"), (4, "1"), (7, "0")])
def test_pipelined_stream_matches_oracle(chunks, sub, monkeypatch):
    """A multi-batch stream with late rows, ties, null speeds, invalid rows, an empty batch, a batch spanning 300 minutes
    (60 windows) and hot-key batches (the first chunk's sample picks table mode, or a slab overflows: the rest of the
    batch re-partitioned) -- every batch equals the oracle; the uniform batches ran pipelined in `chunks` chunks."""
    from mobheat import synth
    from oracle.spark_oracle import SparkHeatmapOracle
    rng = np.random.default_rng(31)
    eng = _engine(monkeypatch, 10, chunks, sub)
    ora = SparkHeatmapOracle(h3_res=10)
    plan = [(0, 7, 40000, 500), (5, 6, 60000, 20), (0, 0, 0, 1), (14, 9, 30000, 500), (1, 300, 50000, 500),
            (320, 4, 80000, 3), (322, 3, 70000, 500)]
    piped = []
    for epoch, (start, span, n, ncells) in enumerate(plan):
        lat = 37.98 + rng.integers(0, ncells, n) * 2e-3 + rng.uniform(0, 1e-4, n)
        lon = 23.73 + rng.uniform(-0.1, 0.1, n) if ncells > 100 else np.full(n, 23.73)
        ts = synth.T0 + start * MINUTE + rng.integers(0, max(span, 1) * MINUTE, n)
        ts[: n // 50] = ts[n // 50: 2 * (n // 50)]
        b = dict(lat=lat, lon=lon, ts_us=ts, speed=rng.uniform(0, 90, n), speed_valid=rng.random(n) > 0.2,
                 vkey=rng.integers(0, 700, n).astype(np.uint64), row_valid=rng.random(n) > 0.01)
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
        piped.append(eng.last_counts()["pipe_chunks"])
    print(f"pipelined chunks per batch: {piped}", flush=True)
    assert piped[0] == chunks and piped[3] == chunks and piped[4] == chunks, piped
    assert piped[2] == 0   # (the empty batch)
    eng.close()


@pytest.mark.parametrize("chunks", [3, 4])
def test_pipelined_keys_span_chunks(chunks, monkeypatch):
    """Every key in every chunk: 1.2e6 rows over ~4.5e4 res-11 keys in random order (each key ~25 rows, so each chunk
    touches nearly every key again: its row is rewritten in place by every chunk's merge, its state line re-read), then
    a second batch in the same window re-touching every key -- counts and sums add up exactly."""
    from mobheat import synth
    from oracle.spark_oracle import SparkHeatmapOracle
    rng = np.random.default_rng(77)
    eng = _engine(monkeypatch, 11, chunks, "0")
    ora = SparkHeatmapOracle(h3_res=11)
    for epoch in range(2):
        n = 1_200_000
        b = dict(lat=37.9 + rng.uniform(0, 0.1, n), lon=23.6 + rng.uniform(0, 0.1, n),
                 ts_us=synth.T0 + epoch * MINUTE + rng.integers(0, MINUTE, n), speed=rng.uniform(0, 90, n),
                 speed_valid=rng.random(n) > 0.1, vkey=rng.integers(0, 5000, n).astype(np.uint64), row_valid=None)
        res, exp = _run(eng, ora, b, epoch)
        c = eng.last_counts()
        assert c["pipe_chunks"] == chunks and not c["table_mode"], c
        assert_batch_equal(res, exp)
        if epoch == 0:   # (the second batch emits the keys it touched, with the first batch's rows in their counts)
            assert int(res.tiles.count.sum()) == n
        assert len(res.tiles) < n // 20   # (keys repeat ~25x: most rows were duplicates of a chunk's or an earlier chunk's key)
    eng.close()


def test_pipelined_state_read_regime(monkeypatch):
    """The state-read leg in small, pipelined: the same points each minute into open windows (batches 1-4 create no key;
    their merges read and rewrite existing lines, the sub-bin variant chosen from the last batch's re-touch ratio)."""
    from oracle.spark_oracle import SparkHeatmapOracle
    rng = np.random.default_rng(29)
    n = 200_000
    lat = np.degrees(np.arcsin(rng.uniform(-1.0, 1.0, n)))
    lon = rng.uniform(-180.0, 180.0, n)
    base = 1_759_572_000_000_000 + rng.integers(0, MINUTE, n)
    speed = rng.uniform(0, 90, n)
    sv = rng.random(n) > 0.1
    vkey = rng.integers(0, 5000, n).astype(np.uint64)
    eng = _engine(monkeypatch, 3, 4)
    ora = SparkHeatmapOracle(h3_res=3)
    for epoch in range(7):
        b = dict(lat=lat, lon=lon, ts_us=base + epoch * MINUTE, speed=speed, speed_valid=sv, vkey=vkey,
                 row_valid=np.ones(n, bool))
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
        assert eng.last_counts()["pipe_chunks"] == 4
        if 0 < epoch < 5:
            assert eng.last_counts()["state_new"] == 0, "an existing key was created again"
    eng.close()


def test_pipelined_windows_appear_in_later_chunks(monkeypatch):
    """A time-ordered batch: its first chunk sees mostly one window, later chunks bring new windows (tables created after
    the first chunk's merge ran: the device's key counts read back before the window map is rewritten) and fill a
    window the first chunk saw only a few rows of (its table, sized from the scaled census, grows inside the batch:
    the keys the earlier merges created dumped and re-merged); then a second batch into the same windows."""
    from mobheat import synth
    from oracle.spark_oracle import SparkHeatmapOracle
    rng = np.random.default_rng(5)
    eng = _engine(monkeypatch, 12, 4, "0")
    ora = SparkHeatmapOracle(h3_res=12)
    for epoch in range(2):
        n = 600_000
        ts = np.sort(synth.T0 + rng.integers(0, 20 * MINUTE, n))
        # the first quarter in window 0 but for a few rows of window 1 that carry hardly any keys; the rest spread
        ts[: n // 4] = synth.T0 + rng.integers(0, 5 * MINUTE, n // 4)
        ts[: 50] = synth.T0 + 5 * MINUTE + 1
        b = dict(lat=37.9 + rng.uniform(0, 0.2, n), lon=23.6 + rng.uniform(0, 0.2, n), ts_us=ts,
                 speed=rng.uniform(0, 90, n), speed_valid=rng.random(n) > 0.1,
                 vkey=rng.integers(0, 9000, n).astype(np.uint64), row_valid=None)
        res, exp = _run(eng, ora, b, epoch)
        assert eng.last_counts()["pipe_chunks"] == 4
        assert_batch_equal(res, exp)
    eng.close()


@pytest.mark.parametrize("cap", [20, 150])
def test_pipelined_slab_overflow_fallback(cap, monkeypatch):
    """Slabs too small for the batch (MOBHEAT_TEST_SLAB_CAP): with 20 records a bin overflows in the first chunk (nothing
    merged pipelined), with 150 in a later one (the chunks before it merged, the rest of the batch partitioned from its
    keys and merged as one more segment group) -- the results equal the oracle either way."""
    from mobheat import synth
    from oracle.spark_oracle import SparkHeatmapOracle
    monkeypatch.setenv("MOBHEAT_TEST_SLAB_CAP", str(cap))
    rng = np.random.default_rng(13)
    eng = _engine(monkeypatch, 9, 4, "0")
    ora = SparkHeatmapOracle(h3_res=9)
    for epoch in range(2):
        n = 2_000_000
        b = dict(lat=np.degrees(np.arcsin(rng.uniform(-1, 1, n))), lon=rng.uniform(-180, 180, n),
                 ts_us=synth.T0 + epoch * MINUTE + rng.integers(0, 2 * MINUTE, n), speed=rng.uniform(0, 90, n),
                 speed_valid=rng.random(n) > 0.1, vkey=rng.integers(0, 50_000, n).astype(np.uint64), row_valid=None)
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
        c = eng.last_counts()
        assert c["pipe_chunks"] == 4 and not c["binned"], c   # (re-partitioned)
    eng.close()


def test_pipelined_statements_equal_unpipelined(monkeypatch):
    """foreach_batch_func's tile and position statements from a pipelined engine equal an unpipelined one's (the same
    dyadic batches: every fp64 sum exact in any order; statements compared as a multiset -- the bulk is unordered)."""
    from mobheat import HeatmapEngine, synth
    rng = np.random.default_rng(3)
    engs = []
    for chunks in ("0", "4"):
        monkeypatch.setenv("MOBHEAT_INGEST_MODE", "binned")
        monkeypatch.setenv("MOBHEAT_PIPELINE", chunks)
        engs.append(HeatmapEngine(h3_res=9))
    for epoch in range(3):
        n = 300_000
        b = dict(lat=37.875 + rng.integers(0, 1 << 12, n) / 16384.0, lon=23.5 + rng.integers(0, 1 << 12, n) / 16384.0,
                 ts_us=synth.T0 + epoch * 3 * MINUTE + rng.integers(0, 4 * MINUTE, n),
                 speed=rng.integers(0, 1 << 10, n) / 16.0, speed_valid=rng.random(n) > 0.1,
                 vkey=rng.integers(0, 3000, n).astype(np.uint64), row_valid=None)
        outs = []
        for eng in engs:
            res = eng.process_batch(epoch, **b)
            buf, offs = eng.encode_tile_updates("ath", 45, copy=True)
            stm = sorted(bytes(buf[offs[i]:offs[i + 1]]) for i in range(offs.size - 1))
            outs.append((stm, np.sort(res.latest_rows)))
        assert [e.last_counts()["pipe_chunks"] for e in engs] == [0, 4]
        assert outs[0][0] == outs[1][0]
        np.testing.assert_array_equal(outs[0][1], outs[1][1])
    for e in engs:
        e.close()
