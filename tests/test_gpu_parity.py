"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on identical seeded inputs.

Bar (BASELINE.json north_star): cell ids, counts, window starts and latest-position rows bit-exact;
averages within 1e-9 relative (fp64 sums in a different order than Spark's), centroid with an absolute
floor of 1e-12 degrees for groups whose coordinates cancel around 0.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REL = 1e-9
ABS_DEG = 1e-12


def _tiles_dict_gpu(t):
    return {(int(t.cell[k]), int(t.window_start_us[k])):
            (int(t.count[k]), None if t.speed_null[k] else float(t.avg_speed[k]), float(t.avg_lon[k]),
             float(t.avg_lat[k])) for k in range(len(t))}


def _tiles_dict_oracle(tiles):
    return {(x["cell"], x["window_start_us"]): (x["count"], x["avg_speed"], x["avg_lon"], x["avg_lat"]) for x in tiles}


def _close(a, b):
    if a is None or b is None:
        return a is None and b is None
    if np.isnan(a) or np.isnan(b):
        return bool(np.isnan(a) and np.isnan(b))
    return abs(a - b) <= max(REL * max(abs(a), abs(b)), ABS_DEG)


def assert_batch_equal(res, exp):
    g = _tiles_dict_gpu(res.tiles)
    o = _tiles_dict_oracle(exp["tiles"])
    assert len(g) == len(res.tiles), "duplicate keys emitted"
    go, oo = set(g) - set(o), set(o) - set(g)   # (a plain set assert's diff repr takes minutes on 1e5 keys)
    assert not go and not oo, f"key sets differ: gpu-only {len(go)} {sorted(go)[:3]}, oracle-only {len(oo)} {sorted(oo)[:3]}"
    bad = [k for k in g if g[k][0] != o[k][0] or not all(_close(g[k][i], o[k][i]) for i in (1, 2, 3))]
    assert not bad, f"{len(bad)} tiles differ, e.g. {bad[0]}: gpu {g[bad[0]]} oracle {o[bad[0]]}"
    np.testing.assert_array_equal(np.sort(res.latest_rows), exp["latest_rows"])
    assert res.n_valid == exp["n_valid"] and res.n_late == exp["n_late"]
    assert res.n_state == exp["n_state"]
    assert res.batch_max_event_ms == exp["batch_max_event_ms"]
    assert res.watermark_ms == exp["watermark_ms"] and res.late_watermark_ms == exp["late_watermark_ms"]


# ---------------------------------------------------------------------------------------------------------
# the UDF: h3.latlng_to_cell
# ---------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("res", range(16))
def test_latlng_to_cell_random_and_edges(oracle_h3, res):
    import mobheat
    from mobheat import synth
    rng = np.random.default_rng(500 + res)
    n = 1_000_000
    el, eo = synth.edge_points()
    lat = np.r_[np.degrees(np.arcsin(rng.uniform(-1, 1, n))), el]
    lon = np.r_[rng.uniform(-180, 180, n), eo]
    got = mobheat.latlng_to_cell(lat, lon, res)
    exp = oracle_h3.latlng_to_cell(lat, lon, res)
    with np.errstate(invalid="ignore"):
        exp = np.where((lat >= -90) & (lat <= 90) & (lon >= -180) & (lon <= 180), exp, 0)
    bad = got != exp
    assert not bad.any(), f"res {res}: {bad.sum()} / {lat.size} mismatches, e.g. {lat[bad][:3]}, {lon[bad][:3]}"


@pytest.mark.parametrize("res", range(16))
def test_ingest_cells_every_resolution(res):
    """k_ingest computes its cells with a kernel specialised per resolution: the tiles of one batch (one window)
    hold exactly the cells latlng_to_cell gives for its points, with the right counts, at every resolution
    (a miscompiled specialisation showed up only at some resolutions)."""
    import mobheat
    from mobheat import HeatmapEngine
    rng = np.random.default_rng(900 + res)
    n = 200_000
    lat = np.degrees(np.arcsin(rng.uniform(-1.0, 1.0, n)))
    lon = rng.uniform(-180.0, 180.0, n)
    ts = 1_759_572_000_000_000 + rng.integers(0, 60_000_000, n)
    eng = HeatmapEngine(h3_res=res)
    r = eng.process_batch(0, lat, lon, ts, rng.uniform(0, 90, n), np.ones(n, bool),
                          rng.integers(0, 5000, n).astype(np.uint64), np.ones(n, bool))
    cells, counts = np.unique(mobheat.latlng_to_cell(lat, lon, res), return_counts=True)
    got = dict(zip(r.tiles.cell.tolist(), r.tiles.count.tolist()))
    want = dict(zip(cells.tolist(), counts.tolist()))
    bad = set(got) ^ set(want)
    assert not bad, f"res {res}: {len(bad)} cells differ, e.g. {[hex(c) for c in sorted(bad)[:3]]}"
    assert got == want
    eng.close()


def test_latlng_to_cell_golden():
    import mobheat
    g = np.load(os.path.join(ROOT, "tests", "golden", "h3_cells.npz"))
    with np.errstate(invalid="ignore"):
        ok = (g["lat"] >= -90) & (g["lat"] <= 90) & (g["lon"] >= -180) & (g["lon"] <= 180)
    for res in range(16):
        np.testing.assert_array_equal(mobheat.latlng_to_cell(g["lat"], g["lon"], res), np.where(ok, g[f"cells_r{res}"], 0))


@pytest.mark.parametrize("res", [7, 8])
def test_latlng_to_cell_c2_scale_sample(oracle_h3, res):
    """10M uniform-sphere points (a C2-sized sample) bit-exact."""
    import mobheat
    rng = np.random.default_rng(77 + res)
    n = 10_000_000
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, n)))
    lon = rng.uniform(-180, 180, n)
    got = mobheat.latlng_to_cell(lat, lon, res)
    exp = oracle_h3.latlng_to_cell(lat, lon, res)
    assert np.count_nonzero(got != exp) == 0


# ---------------------------------------------------------------------------------------------------------
# the whole micro-batch
# ---------------------------------------------------------------------------------------------------------
def _run(engine, oracle, batch, epoch):
    res = engine.process_batch(epoch, **batch)
    exp = oracle.process_batch(**batch)
    return res, exp


def test_c1_boston_batch():
    from mobheat import HeatmapEngine, synth
    from oracle.spark_oracle import SparkHeatmapOracle
    b = synth.c1_boston()
    eng = HeatmapEngine(h3_res=8)
    res, exp = _run(eng, SparkHeatmapOracle(h3_res=8), b, 0)
    assert_batch_equal(res, exp)
    assert len(res.tiles) > 100 and len(set(res.tiles.window_start_us.tolist())) == 2
    # against the committed golden fixture too
    g = np.load(os.path.join(ROOT, "tests", "golden", "c1_batch.npz"))
    assert set(zip(g["t_cell"].tolist(), g["t_ws"].tolist())) == set(
        zip(res.tiles.cell.tolist(), res.tiles.window_start_us.tolist()))
    np.testing.assert_array_equal(np.sort(res.latest_rows), g["latest"])
    eng.close()


def test_multi_batch_watermark_and_eviction():
    """Several batches: cumulative update-mode aggregates, late rows dropped with the previous batch's
    watermark, eviction after emission, an empty (no-data) batch, out-of-order and tied timestamps."""
    from mobheat import HeatmapEngine
    from oracle.spark_oracle import SparkHeatmapOracle
    rng = np.random.default_rng(11)
    eng = HeatmapEngine(h3_res=9)
    ora = SparkHeatmapOracle(h3_res=9)
    t0 = 1_759_572_000_000_000
    minute = 60_000_000
    for epoch, (start_min, span_min, n) in enumerate([(0, 7, 20000), (5, 6, 20000), (0, 0, 0), (14, 9, 30000),
                                                      (1, 30, 30000), (40, 3, 5000), (0, 0, 0), (55, 2, 5000)]):
        lat = rng.uniform(37.90, 38.05, n)
        lon = rng.uniform(23.60, 23.85, n)
        ts = t0 + start_min * minute + rng.integers(0, max(span_min, 1) * minute, n)
        ts[: n // 50] = ts[n // 50: 2 * (n // 50)]               # ties within vehicles below
        speed = rng.uniform(0, 90, n)
        sv = rng.random(n) > 0.2
        vkey = rng.integers(0, 500, n).astype(np.uint64)
        rv = rng.random(n) > 0.01
        b = dict(lat=lat, lon=lon, ts_us=ts, speed=speed, speed_valid=sv, vkey=vkey, row_valid=rv)
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
    eng.close()


def test_state_read_regime_matches_oracle():
    """The bench's state_read_leg in small: the same points every batch, each batch one minute later, so batches 2-5
    of a 5-minute window update every existing key (the merge's whole-line loads of existing state, rows rewritten),
    then a new window.  Dense enough (res 3: 41k cells for 2e5 points) that keys repeat within a batch and chunk."""
    from mobheat import HeatmapEngine
    from oracle.spark_oracle import SparkHeatmapOracle
    rng = np.random.default_rng(29)
    n = 200_000
    lat = np.degrees(np.arcsin(rng.uniform(-1.0, 1.0, n)))
    lon = rng.uniform(-180.0, 180.0, n)
    base = 1_759_572_000_000_000 + rng.integers(0, 60_000_000, n)
    speed = rng.uniform(0, 90, n)
    sv = rng.random(n) > 0.1
    vkey = rng.integers(0, 5000, n).astype(np.uint64)
    rv = np.ones(n, bool)
    eng = HeatmapEngine(h3_res=3)
    ora = SparkHeatmapOracle(h3_res=3)
    for epoch in range(7):
        b = dict(lat=lat, lon=lon, ts_us=base + epoch * 60_000_000, speed=speed, speed_valid=sv, vkey=vkey, row_valid=rv)
        print(f"state-read regime: batch {epoch}", flush=True)
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
        if 0 < epoch < 5:
            assert eng.last_counts()["state_new"] == 0, "an existing key was created again"
    eng.close()


def test_steady_state_batches_allocate_nothing():
    """The state-read regime with window growth, 30 one-minute batches at res 7 (half the points repeat, half are new
    each minute, so a window's table grows during its life): after the first windows have been evicted, no batch
    allocates or frees device or pinned memory (a hipMalloc/hipFree inside a step stalls it --
    released window tables are pooled, the buffers only grow), and every batch still equals the oracle."""
    from mobheat import HeatmapEngine
    from oracle.spark_oracle import SparkHeatmapOracle
    rng = np.random.default_rng(41)
    n = 200_000
    lat0 = np.degrees(np.arcsin(rng.uniform(-1.0, 1.0, n // 2)))
    lon0 = rng.uniform(-180.0, 180.0, n // 2)
    eng = HeatmapEngine(h3_res=7)
    ora = SparkHeatmapOracle(h3_res=7)
    counts = []
    for epoch in range(30):
        lat = np.concatenate([lat0, np.degrees(np.arcsin(rng.uniform(-1.0, 1.0, n // 2)))])
        lon = np.concatenate([lon0, rng.uniform(-180.0, 180.0, n // 2)])
        b = dict(lat=lat, lon=lon, ts_us=1_759_572_000_000_000 + epoch * 60_000_000 + rng.integers(0, 60_000_000, n),
                 speed=rng.uniform(0, 90, n), speed_valid=rng.random(n) > 0.1,
                 vkey=rng.integers(0, 5000, n).astype(np.uint64), row_valid=np.ones(n, bool))
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
        c = eng.last_counts()
        counts.append((c["allocs"], c["frees"]))
    # steady state from the first eviction on: window [0, 5 min) is evicted in batch 15 (watermark = max ts - 10 min);
    # before that every batch may hold more live windows than any batch before it, whose tables cannot come from the
    # pool yet.  From there on each window still grows its table twice during its life (2^19 -> 2^21 slots), from
    # the pool of released tables, and the buffers grow with headroom: nothing is allocated or freed.
    changed = [(e, counts[e - 1], counts[e]) for e in range(16, len(counts)) if counts[e] != counts[e - 1]]
    assert not changed, f"batches that allocated or freed (epoch, before, after): {changed}; all: {counts}"
    print(f"allocations/frees since create after each batch: {counts}")
    eng.close()


def test_edge_semantics_batch():
    """Filter edges (+-90/+-180 inclusive, NaN, inf, null rows), window boundaries, negative timestamps,
    null and NaN speeds, duplicate vehicles with tied maxima."""
    from mobheat import HeatmapEngine
    from oracle.spark_oracle import SparkHeatmapOracle
    tile = 300_000_000
    t0 = 1_759_572_000_000_000
    lat = np.array([90.0, -90.0, 0.0, 45.0, np.nan, 10.0, 10.0, 10.0, 10.0, 10.0, 10.0, 10.0, np.inf, 10.0, 10.0])
    lon = np.array([180.0, -180.0, 0.0, 45.0, 0.0, 180.0000001, 20.0, 20.0, 20.0, 20.0, 20.0, 20.0, 0.0, -np.inf, 20.0])
    ts = np.array([t0, t0 + tile - 1, t0 + tile, t0 - 1, t0, t0, t0 + 5, t0 + 5, t0 + 5, t0 + 7, t0 + 7, -1, t0, t0,
                   -tile - 3], dtype=np.int64)
    speed = np.array([1.0, 2.0, 3.0, np.nan, 5.0, 6.0, 7.0, 8.0, 9.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0])
    sv = np.array([1, 1, 1, 1, 1, 1, 0, 0, 0, 1, 1, 1, 1, 1, 1], bool)
    vkey = np.array([1, 1, 2, 3, 4, 5, 6, 6, 6, 7, 7, 8, 9, 10, 11], np.uint64)
    rv = np.array([1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 1, 1, 1, 1], bool)
    b = dict(lat=lat, lon=lon, ts_us=ts, speed=speed, speed_valid=sv, vkey=vkey, row_valid=rv)
    for late_prev in (True, False):
        eng = HeatmapEngine(h3_res=5, late_uses_prev_watermark=late_prev)
        res, exp = _run(eng, SparkHeatmapOracle(h3_res=5, late_uses_prev_watermark=late_prev), b, 0)
        assert_batch_equal(res, exp)
        eng.close()


def test_dedup_ties_c5_sample():
    from mobheat import HeatmapEngine, synth
    from oracle.spark_oracle import SparkHeatmapOracle
    b = synth.c5_dedup(n_vehicles=200_000, updates=10)
    eng = HeatmapEngine(h3_res=8)
    res, exp = _run(eng, SparkHeatmapOracle(h3_res=8), b, 0)
    assert_batch_equal(res, exp)
    assert len(res.latest_rows) > 200_000          # the tie subset adds rows
    eng.close()


@pytest.mark.parametrize("dense", ["1", "0"])
def test_dedup_more_vehicles_than_fused_table(dense, monkeypatch):
    """k_ingest's fused dedup: dense vkeys below the dense table's size (2^20 on a first batch, then sized from the
    last batch's largest vkey) keep their max in it, the others in the hash table, which is sized from the previous
    batch's distinct vehicles (>= 2^18 keys) -- the first batch's 1.2M vehicles (vkeys 0 .. 1.2M: 2^20 of them dense)
    overflow its bounded probes without the dense table (dense "0": MOBHEAT_DEDUP_DENSE=0), so the max pass reruns on
    a full-size table.  The second batch takes the fused path either way. Both must equal the oracle."""
    monkeypatch.setenv("MOBHEAT_DEDUP_DENSE", dense)
    from mobheat import HeatmapEngine, synth
    from oracle.spark_oracle import SparkHeatmapOracle
    eng = HeatmapEngine(h3_res=8)
    ora = SparkHeatmapOracle(h3_res=8)
    for epoch in range(2):
        b = synth.c5_dedup(seed=40 + epoch, n_vehicles=1_200_000, updates=2)
        b["ts_us"] = b["ts_us"] + epoch * 600_000_000
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
        assert len(res.latest_rows) >= 1_200_000
    eng.close()


def test_merge_many_duplicate_keys_per_chunk():
    """Every key of a 6M-row binned batch occurs 4 times (1.5M keys, ~183 per bin, one window): a merge chunk of 512
    records holds more keys with in-chunk duplicates than k_merge_owned's joiner accumulator pool (MO_ACC = 128), so
    the joiners left over wait for a second pass of the chunk.  Counts and averages against the oracle, then the same
    keys again in a second batch (every key existing)."""
    from mobheat import HeatmapEngine
    from oracle.spark_oracle import SparkHeatmapOracle
    rng = np.random.default_rng(77)
    m, rep = 1_500_000, 4
    lat0 = np.degrees(np.arcsin(rng.uniform(-1, 1, m)))
    lon0 = rng.uniform(-180, 180, m)
    eng = HeatmapEngine(h3_res=8)
    ora = SparkHeatmapOracle(h3_res=8)
    t0 = 1759572000 * 1_000_000
    for epoch in range(2):
        perm = rng.permutation(m * rep)
        idx = np.repeat(np.arange(m), rep)[perm]
        n = m * rep
        b = dict(lat=lat0[idx], lon=lon0[idx], ts_us=t0 + rng.integers(0, 240_000_000, n) + epoch * 1_000_000,
                 speed=rng.uniform(0, 80, n).round(0), speed_valid=rng.random(n) >= 0.1,
                 vkey=rng.integers(0, 40_000, n).astype(np.uint64), row_valid=np.ones(n, bool))
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
    eng.close()


def test_dedup_sparse_and_dense_vkeys():
    """vkeys that are not dense codes (64-bit values: the hash table only, and the next batch without a dense table),
    then dense ones (the dense table sized from scratch), then a mix of both in one batch."""
    from mobheat import HeatmapEngine, synth
    from oracle.spark_oracle import SparkHeatmapOracle
    eng = HeatmapEngine(h3_res=7)
    ora = SparkHeatmapOracle(h3_res=7)
    rng = np.random.default_rng(5)
    for epoch, kind in enumerate(("sparse", "sparse", "dense", "mixed", "dense")):
        b = synth.c5_dedup(seed=60 + epoch, n_vehicles=30_000, updates=4)
        b["ts_us"] = b["ts_us"] + epoch * 600_000_000
        v = b["vkey"].astype(np.uint64)
        big = (v * np.uint64(0x9E3779B97F4A7C15)) | np.uint64(1 << 40)
        if kind == "sparse":
            b["vkey"] = big
        elif kind == "mixed":
            b["vkey"] = np.where(rng.random(v.size) < 0.5, v, big).astype(np.uint64)
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
    eng.close()


def test_high_cardinality_res12_two_batches():
    from mobheat import HeatmapEngine, synth
    from oracle.spark_oracle import SparkHeatmapOracle
    b1, b2 = synth.c4_high_cardinality(n=2_000_000)
    eng = HeatmapEngine(h3_res=12)
    ora = SparkHeatmapOracle(h3_res=12)
    # Spark runs a no-data batch after batch 1 because the watermark advanced (MicroBatchExecution's
    # shouldRunAnotherBatch); the late filter of batch 3 then uses that batch's watermark.
    empty = {k: v[:0] for k, v in b1.items()}
    for e, b in enumerate((b1, empty, b2)):
        res, exp = _run(eng, ora, b, e)
        assert_batch_equal(res, exp)
    assert res.n_late > 0
    eng.close()


def test_clustered_city_res9():
    """C3-shaped batches (Zipf hot spots, res 9): every batch takes the table mode -- the first one because its key
    sample shows heavy hitters (k_sample_heavy: the hottest key holds ~3% of the rows), the next ones also from the
    last batch's cardinality -- which must collapse the partials to about the key count."""
    from mobheat import HeatmapEngine, synth
    from oracle.spark_oracle import SparkHeatmapOracle
    eng = HeatmapEngine(h3_res=9)
    ora = SparkHeatmapOracle(h3_res=9)
    for epoch in range(3):
        b = synth.c3_city(seed=2 + epoch, n=3_000_000, n_vehicles=5000)
        b["ts_us"] = b["ts_us"] + epoch * 600_000_000
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
        assert eng.last_counts()["table_mode"]
        assert res.n_partials <= 4 * len(res.tiles), (res.n_partials, len(res.tiles))
    eng.close()


def test_binned_ingest_then_table_mode():
    """A batch large enough to be binned in k_ingest (>= 2^22 rows) whose key sample then shows heavy hitters: the
    binned ingest wrote the event keys of its exception and sampled rows only, so the switch to table mode first
    completes every row's key (keys_complete: k_ingest's keys-only pass) -- results equal the oracle's, over two
    batches (the second chooses table mode from the first's cardinality, its keys written in full)."""
    from mobheat import HeatmapEngine, synth
    from oracle.spark_oracle import SparkHeatmapOracle
    eng = HeatmapEngine(h3_res=9)
    ora = SparkHeatmapOracle(h3_res=9)
    for epoch in range(2):
        b = synth.c3_city(seed=7 + epoch, n=4_400_000, n_vehicles=5000)
        b["ts_us"] = b["ts_us"] + epoch * 600_000_000
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
        assert eng.last_counts()["table_mode"]
    eng.close()


def test_full_size_properties_c2():
    """C2 size (1e8 events, res 8) through the device path: size-independent properties only."""
    import mobheat
    from mobheat import HeatmapEngine, synth
    b = synth.c2_global(n=100_000_000)
    eng = HeatmapEngine(h3_res=8)
    res = eng.process_batch(0, **b)
    assert not eng.last_counts()["table_mode"]                      # uniform keys: no heavy hitter in the sample
    t = res.tiles
    assert res.n_valid == b["lat"].size and res.n_late == 0
    assert int(t.count.sum()) == res.n_valid                       # every valid row lands in exactly one tile
    keys = t.cell.astype(np.uint64) ^ (t.window_start_us.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15))
    assert np.unique(keys).size == len(t)                           # no key emitted twice
    assert set(np.unique(t.window_start_us).tolist()) <= {synth.T0 + k * 300_000_000 for k in range(3)}
    # every latest row is a valid row and carries the max ts of its vehicle
    lr = res.latest_rows
    assert np.all(np.diff(lr) > 0)
    vk, ts = b["vkey"][lr], b["ts_us"][lr]
    order = np.lexsort((b["ts_us"], b["vkey"]))
    last = np.r_[b["vkey"][order][1:] != b["vkey"][order][:-1], True]
    vmax = dict(zip(b["vkey"][order][last].tolist(), b["ts_us"][order][last].tolist()))
    assert all(vmax[int(v)] == int(x) for v, x in zip(vk[:100000], ts[:100000]))
    assert len(set(vk.tolist())) == len(vmax)
    # sample parity of cells against the UDF
    idx = np.random.default_rng(0).choice(b["lat"].size, 200_000, replace=False)
    from oracle import h3_oracle
    c = h3_oracle.latlng_to_cell(b["lat"][idx], b["lon"][idx], 8)
    assert np.array_equal(c, mobheat.latlng_to_cell(b["lat"][idx], b["lon"][idx], 8))
    eng.close()


def test_rows_on_device_same_statements():
    """rows_on_device=True (what foreach_batch_func uses: the rows stay on the device and the statements are encoded
    from them) gives the same counts and byte-identical tile and position statements as the host-output path, over
    two batches that update the same windows."""
    import mobheat
    from mobheat import synth
    a, b = mobheat.HeatmapEngine(h3_res=9), mobheat.HeatmapEngine(h3_res=9)
    for epoch in range(2):
        x = synth.c1_boston(seed=30 + epoch, n=50_000)
        x["ts_us"] = x["ts_us"] + epoch * 30_000_000
        ra = a.process_batch(epoch, **x)
        rb = b.process_batch(epoch, **x, rows_on_device=True)
        assert rb.tiles is None and rb.latest_rows is None
        assert (rb.n_tiles, rb.n_latest) == (len(ra.tiles), ra.latest_rows.size)
        assert (rb.n_valid, rb.n_late, rb.n_state, rb.watermark_ms) == (ra.n_valid, ra.n_late, ra.n_state, ra.watermark_ms)
        ba, oa = a.encode_tile_updates("ath", 30)
        bb, ob = b.encode_tile_updates("ath", 30)
        # (tile order and the last bits of the fp64 sums may differ between two engines: compare by _id)
        import bson

        def docs(buf, offs):
            out = {}
            for k in range(offs.size - 1):
                d = bson.decode(bytes(buf[offs[k]:offs[k + 1]]))
                out[d["q"]["_id"]] = d["u"]["$set"]
            return out
        da, db = docs(ba, oa), docs(bb, ob)
        assert da.keys() == db.keys() and len(da) == rb.n_tiles
        for k, u in da.items():
            v = db[k]
            assert u.keys() == v.keys() and u["count"] == v["count"] and u["staleAt"] == v["staleAt"]
            assert u["avgSpeedKmh"] == pytest.approx(v["avgSpeedKmh"], rel=1e-12, abs=1e-12)
            assert u["centroid"]["coordinates"] == pytest.approx(v["centroid"]["coordinates"], rel=1e-12)
    a.close()
    b.close()


def test_foreach_batch_func_capture_sink():
    """The drop-in boundary end to end: a micro-batch frame in, the reference's UpdateOne ops out."""
    import pandas as pd
    from mobheat import stream, synth
    from oracle.spark_oracle import SparkHeatmapOracle

    class Capture:
        ops = {}

        def bulk_write(self, coll, ops):
            assert len(ops) <= 1000
            Capture.ops.setdefault(coll, []).extend(ops)

        def update_raw(self, coll, stmts):   # GPU-encoded statements: decoded back to (filter, update) pairs
            import types
            import bson
            assert len(stmts) <= 1000
            for st in stmts:
                d = bson.decode(st.raw)
                assert d["multi"] is False and d["upsert"] is True
                Capture.ops.setdefault(coll, []).append(types.SimpleNamespace(_filter=d["q"], _doc=d["u"]))

        def close(self):
            pass

    b = synth.c1_boston(n=3000)
    # a few NaN speeds (Spark's JSON reader accepts NaN tokens): avg(speedKmh) of their tiles is NaN, which the sink
    # keeps (float(NaN or 0.0) is NaN, heatmap_stream.py:169); null speeds (None) are skipped by avg
    nan_rows = np.flatnonzero(b["speed_valid"] & b["row_valid"])[:5]
    b["speed"] = b["speed"].copy()
    b["speed"][nan_rows] = np.nan
    df = pd.DataFrame({
        "provider": ["mbta"] * len(b["lat"]),
        "vehicleId": [None if not v else f"v{i:05d}" for i, v in enumerate(b["row_valid"])],
        "lat": b["lat"], "lon": b["lon"],
        "speedKmh": pd.Series([float(x) if v else None for x, v in zip(b["speed"], b["speed_valid"])], dtype=object),
        "eventTs": pd.to_datetime(b["ts_us"], unit="us"),
    })
    stream.reset_engine()
    stream.SINK_FACTORY = Capture
    try:
        stream.foreach_batch_func(df, 0)
    finally:
        stream.SINK_FACTORY = stream.MongoSink
        stream.reset_engine()
    exp = SparkHeatmapOracle(h3_res=stream.H3_RES).process_batch(**b)
    tiles = {op._filter["_id"]: op._doc["$set"] for op in Capture.ops["tiles"]}
    assert len(tiles) == len(exp["tiles"])
    for x in exp["tiles"]:
        ws = stream._spark_datetime(x["window_start_us"])
        _id = f"{stream.CITY}|h3r{stream.H3_RES}|{x['cell']:x}|{ws.strftime('%Y-%m-%dT%H:%M:%SZ')}"
        d = tiles[_id]
        assert d["count"] == x["count"] and d["cellId"] == format(x["cell"], "x")
        assert _close(d["avgSpeedKmh"], x["avg_speed"] or 0.0)
    assert sum(np.isnan(d["avgSpeedKmh"]) for d in tiles.values()) >= 1   # the NaN rows' tiles
    pos = Capture.ops["positions_latest"]
    assert sorted(op._filter["_id"] for op in pos) == sorted(f"mbta|v{r:05d}" for r in exp["latest_rows"])


def test_window_tables_growth_many_windows_and_reuse():
    """Per-window state tables: a window whose keys outgrow its table across batches (dump + rehash merge),
    a hot window with few keys and many partials, a batch spanning 300 windows (300 tables), and a long run
    of advancing batches whose evicted windows' tables are reused uncleared by later windows."""
    from mobheat import HeatmapEngine, synth
    from oracle.spark_oracle import SparkHeatmapOracle
    rng = np.random.default_rng(21)
    eng = HeatmapEngine(h3_res=12)
    ora = SparkHeatmapOracle(h3_res=12)
    minute = 60_000_000
    plan = [
        # (n, lat/lon box km, start minute, span minutes): window [0,5) grows from ~5k to ~250k keys
        (5_000, 5.0, 0, 4), (60_000, 20.0, 0, 4), (400_000, 40.0, 1, 3),
        # 300 windows in one batch, then advancing batches that evict and reuse tables
        (300_000, 10.0, 2, 1500), (50_000, 10.0, 1500, 10), (50_000, 10.0, 1510, 10), (80_000, 30.0, 1520, 10),
        (80_000, 30.0, 1530, 10), (2_000, 0.5, 1540, 4),
    ]
    for epoch, (n, km, start, span) in enumerate(plan):
        lat = 37.98 + rng.uniform(-0.5, 0.5, n) * km / 111.0
        lon = 23.73 + rng.uniform(-0.5, 0.5, n) * km / 88.0
        ts = synth.T0 + start * minute + rng.integers(0, span * minute, n)
        b = dict(lat=lat, lon=lon, ts_us=ts, speed=rng.uniform(0, 90, n), speed_valid=rng.random(n) > 0.1,
                 vkey=rng.integers(0, 4000, n).astype(np.uint64), row_valid=None)
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
    # hot window: 200 keys, 2M events -> many partials of few keys
    n = 2_000_000
    lat = 37.98 + rng.integers(0, 200, n) * 1e-3
    b = dict(lat=lat, lon=np.full(n, 23.73), ts_us=synth.T0 + 1560 * minute + rng.integers(0, 4 * minute, n),
             speed=rng.uniform(0, 90, n), speed_valid=None, vkey=rng.integers(0, 4000, n).astype(np.uint64), row_valid=None)
    res, exp = _run(eng, ora, b, len(plan))
    assert_batch_equal(res, exp)
    eng.close()


@pytest.mark.parametrize("mode", ["direct", "table", "binned", "binned_whole"])
def test_ingest_modes_parity(mode, monkeypatch):
    """The aggregation paths pinned (MOBHEAT_INGEST_MODE): direct (every aggregated row a 32-B record through the
    partition and merge), binned (the same records written into their sub-bins by k_ingest itself, merged a bin's
    sub-slabs in order -- MOBHEAT_SUBBINS=1; a batch whose hot keys overflow a slab falls back to the partition;
    binned_whole: whole bins, MOBHEAT_SUBBINS=0) and table (k_agg's LDS table with hot-key retention + k_bin_reduce, picked adaptively for
    low-cardinality batches) give the oracle's results on a multi-batch stream with late rows, ties, nulls, an empty
    batch, many windows and few hot keys."""
    from mobheat import HeatmapEngine, synth
    from oracle.spark_oracle import SparkHeatmapOracle
    monkeypatch.setenv("MOBHEAT_SUBBINS", "0" if mode == "binned_whole" else "1")
    mode = "binned" if mode == "binned_whole" else mode
    monkeypatch.setenv("MOBHEAT_INGEST_MODE", mode)
    rng = np.random.default_rng(31)
    binned = []
    eng = HeatmapEngine(h3_res=10)
    ora = SparkHeatmapOracle(h3_res=10)
    minute = 60_000_000
    plan = [(0, 7, 40000, 500), (5, 6, 60000, 20), (0, 0, 0, 1), (14, 9, 30000, 500), (1, 300, 50000, 500),
            (320, 4, 80000, 3)]
    for epoch, (start, span, n, ncells) in enumerate(plan):
        lat = 37.98 + rng.integers(0, ncells, n) * 2e-3 + rng.uniform(0, 1e-4, n)
        lon = 23.73 + rng.uniform(-0.1, 0.1, n) if ncells > 100 else np.full(n, 23.73)
        ts = synth.T0 + start * minute + rng.integers(0, max(span, 1) * minute, n)
        ts[: n // 50] = ts[n // 50: 2 * (n // 50)]
        b = dict(lat=lat, lon=lon, ts_us=ts, speed=rng.uniform(0, 90, n), speed_valid=rng.random(n) > 0.2,
                 vkey=rng.integers(0, 700, n).astype(np.uint64), row_valid=rng.random(n) > 0.01)
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
        binned.append(eng.last_counts()["binned"])
    if mode == "binned":   # (uniform batches binned by the ingest; the hot-key batches overflowed and re-partitioned)
        assert binned == [True, False, False, True, True, False], binned
    eng.close()


@pytest.mark.parametrize("mode", ["direct", "binned", "binned_whole"])
def test_direct_merge_keys_repeated_across_chunks(mode, monkeypatch):
    """k_merge_owned with every key in several consecutive 512-record chunks of its bin (direct path forced: 1.2e7 rows
    over ~5e5 res-11 keys, ~1.5k rows per bin): a chunk's stores are only drained by the next chunk's full barrier, so
    a key the previous chunk wrote is deferred behind it (mobheat.hip: k_merge_owned step 4) -- counts and sums must
    still add up exactly; a second batch in the same window re-reads every key's state."""
    from mobheat import HeatmapEngine, synth
    from oracle.spark_oracle import SparkHeatmapOracle
    monkeypatch.setenv("MOBHEAT_SUBBINS", "0" if mode == "binned_whole" else "1")
    mode = "binned" if mode == "binned_whole" else mode
    monkeypatch.setenv("MOBHEAT_INGEST_MODE", mode)
    rng = np.random.default_rng(77)
    eng = HeatmapEngine(h3_res=11)
    ora = SparkHeatmapOracle(h3_res=11)
    minute = 60_000_000
    for epoch in range(2):
        n = 12_000_000
        b = dict(lat=37.9 + rng.uniform(0, 0.3, n), lon=23.6 + rng.uniform(0, 0.3, n),
                 ts_us=synth.T0 + epoch * minute + rng.integers(0, minute, n), speed=rng.uniform(0, 90, n),
                 speed_valid=rng.random(n) > 0.1, vkey=rng.integers(0, 5000, n).astype(np.uint64), row_valid=None)
        res, exp = _run(eng, ora, b, epoch)
        assert not eng.last_counts()["table_mode"]
        assert_batch_equal(res, exp)
        if epoch == 0:
            assert int(res.tiles.count.sum()) == n
    eng.close()


@pytest.mark.parametrize("arena_mb", [1, 48])
def test_state_arena_tables(arena_mb):
    """Window tables carved from a create-time arena (state_arena_bytes): a small arena runs out mid-stream and
    later tables come from hipMalloc; evicted arena tables are pooled and reused -- results equal the oracle."""
    from mobheat import HeatmapEngine
    from oracle.spark_oracle import SparkHeatmapOracle
    rng = np.random.default_rng(61)
    eng = HeatmapEngine(h3_res=10, state_arena_bytes=arena_mb << 20)
    ora = SparkHeatmapOracle(h3_res=10)
    t0 = 1_759_572_000_000_000
    for epoch in range(10):
        n = 40000
        b = dict(lat=rng.uniform(37.90, 38.05, n), lon=rng.uniform(23.60, 23.85, n),
                 ts_us=t0 + epoch * 7 * 60_000_000 + rng.integers(0, 12 * 60_000_000, n), speed=rng.uniform(0, 90, n),
                 speed_valid=rng.random(n) > 0.2, vkey=rng.integers(0, 800, n).astype(np.uint64), row_valid=None)
        res, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res, exp)
    eng.close()


@pytest.mark.parametrize("res", [0, 7, 15])
def test_global_batch_other_resolutions(res):
    """The whole pipeline at configs[1]'s res 7 and the extreme resolutions, on a global batch with edge points
    (poles, the antimeridian, pentagon centres), two batches so cumulative state is exercised."""
    from mobheat import HeatmapEngine, synth
    from oracle.spark_oracle import SparkHeatmapOracle
    rng = np.random.default_rng(70 + res)
    eng = HeatmapEngine(h3_res=res)
    ora = SparkHeatmapOracle(h3_res=res)
    el, eo = synth.edge_points()
    for epoch in range(2):
        n = 30000
        lat = np.r_[np.degrees(np.arcsin(rng.uniform(-1, 1, n))), el]
        lon = np.r_[rng.uniform(-180, 180, n), eo]
        m = lat.size
        b = dict(lat=lat, lon=lon, ts_us=1_759_572_000_000_000 + epoch * 300_000_000 + rng.integers(0, 600_000_000, m),
                 speed=rng.uniform(0, 900, m), speed_valid=rng.random(m) > 0.1,
                 vkey=rng.integers(0, 5000, m).astype(np.uint64), row_valid=rng.random(m) > 0.01)
        res_, exp = _run(eng, ora, b, epoch)
        assert_batch_equal(res_, exp)
    eng.close()
