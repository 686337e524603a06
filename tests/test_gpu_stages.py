"""GPU: the multi-GPU stage API (hm_stage_local / hm_stage_merge / hm_stage_finish) through the HIP library,
with W contexts ("virtual ranks") on one device and the all-to-all done on the host.  The union of the owners'
outputs must equal the single-shard result (oracle), batch after batch (state ownership is stable).
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class DevBuf:
    def __init__(self, lib, nbytes):
        self.lib = lib
        self.p = ctypes.c_void_p()
        assert lib.hm_device_alloc(0, max(int(nbytes), 16), ctypes.byref(self.p)) == 0
        self.nbytes = nbytes

    def put(self, arr):
        arr = np.ascontiguousarray(arr)
        if arr.nbytes:
            assert self.lib.hm_memcpy(self.p, arr.ctypes.data, arr.nbytes, 0) == 0

    def get(self, nbytes):
        out = np.empty(int(nbytes), np.uint8)
        if nbytes:
            assert self.lib.hm_memcpy(out.ctypes.data, self.p, int(nbytes), 1) == 0
        return out

    def free(self):
        self.lib.hm_device_free(0, self.p)


def _stage_batch(engines, lib, batches_per_rank, epoch):
    from mobheat._lib import HM_CAND_REC_BYTES, HM_MEM_HOST, HM_TILE_REC_BYTES, HmBatchIn, HmBatchOut, HmStageSizes, check
    W = len(engines)
    sends, tcounts, ccounts, maxes, bufs = [], [], [], [], []
    for r, (eng, b) in enumerate(zip(engines, batches_per_rank)):
        n = b["lat"].size
        tb, cb = DevBuf(lib, n * HM_TILE_REC_BYTES), DevBuf(lib, n * HM_CAND_REC_BYTES)
        bufs += [tb, cb]
        tc, cc = (ctypes.c_int64 * W)(), (ctypes.c_int64 * W)()
        sz = HmStageSizes()
        keep = {k: np.ascontiguousarray(v) for k, v in b.items()}
        sv = keep["speed_valid"].astype(np.uint8)
        rv = keep["row_valid"].astype(np.uint8)
        bi = HmBatchIn(n=n, memory=HM_MEM_HOST, lat=keep["lat"].ctypes.data, lon=keep["lon"].ctypes.data,
                       ts_us=keep["ts_us"].ctypes.data, speed=keep["speed"].ctypes.data, speed_valid=sv.ctypes.data,
                       vkey=keep["vkey"].ctypes.data, row_valid=rv.ctypes.data)
        check(lib.hm_stage_local(eng._ctx, epoch, ctypes.byref(bi), W, r, tb.p, n, tc, cb.p, n, cc, ctypes.byref(sz)),
              eng._ctx)
        tcounts.append(list(tc)); ccounts.append(list(cc)); maxes.append(sz.batch_max_event_ms)
        sends.append((tb.get(sum(tc) * HM_TILE_REC_BYTES), cb.get(sum(cc) * HM_CAND_REC_BYTES)))
    gmax = max(maxes)

    def route(r, kind, rec):
        parts = []
        for s in range(W):
            cnt = (tcounts if kind == 0 else ccounts)[s]
            off = sum(cnt[:r]) * rec
            parts.append(sends[s][kind][off: off + cnt[r] * rec])
        return np.concatenate(parts) if parts else np.zeros(0, np.uint8)

    outs, wsends, wcounts = [], [], []
    for r, eng in enumerate(engines):
        trecv, crecv = route(r, 0, HM_TILE_REC_BYTES), route(r, 1, HM_CAND_REC_BYTES)
        tb, cb, wb = DevBuf(lib, trecv.nbytes), DevBuf(lib, crecv.nbytes), DevBuf(lib, max(crecv.nbytes // 4, 8))
        bufs += [tb, cb, wb]
        tb.put(trecv); cb.put(crecv)
        nc = crecv.nbytes // HM_CAND_REC_BYTES
        out = HmBatchOut()
        wc = (ctypes.c_int64 * W)()
        check(lib.hm_stage_merge(eng._ctx, tb.p, trecv.nbytes // HM_TILE_REC_BYTES, cb.p, nc, gmax, HM_MEM_HOST,
                                 ctypes.byref(out), wb.p, max(nc, 1), wc), eng._ctx)
        res = eng._result_from_host(out)
        outs.append(res.tiles)
        wcounts.append(list(wc))
        wsends.append(wb.get(sum(wc) * 8).view(np.int64))
    latest = []
    for r, eng in enumerate(engines):
        rows = np.concatenate([wsends[s][sum(wcounts[s][:r]): sum(wcounts[s][:r + 1])] for s in range(W)])
        wb = DevBuf(lib, rows.nbytes + 8)
        bufs.append(wb)
        wb.put(rows)
        out = HmBatchOut()
        check(lib.hm_stage_finish(eng._ctx, wb.p, rows.size, HM_MEM_HOST, ctypes.byref(out)), eng._ctx)
        got = np.ctypeslib.as_array(ctypes.cast(out.latest_row, ctypes.POINTER(ctypes.c_int64)), shape=(out.n_latest,)) \
            if out.n_latest else np.zeros(0, np.int64)
        latest.append(got.copy())
    for b in bufs:
        b.free()
    return outs, latest, tcounts, ccounts


@pytest.mark.parametrize("world", [2, 3])
def test_stage_api_matches_single_shard(world):
    import mobheat
    from mobheat import synth
    from oracle.spark_oracle import SparkHeatmapOracle
    lib = mobheat.load()
    engines = [mobheat.HeatmapEngine(h3_res=9) for _ in range(world)]
    ora = SparkHeatmapOracle(h3_res=9)
    rng = np.random.default_rng(9)
    for epoch, (start, n) in enumerate(((0, 60000), (12, 60000), (0, 0), (30, 80000))):
        b = synth.c3_city(seed=epoch, n=max(n, 1), hotspots=300, n_vehicles=2000)
        b = {k: v[:n] for k, v in b.items()}
        b["ts_us"] = synth.T0 + start * 60_000_000 + rng.integers(0, 9 * 60_000_000, n)
        bounds = [i * n // world for i in range(world + 1)]
        shards = [{k: v[bounds[r]:bounds[r + 1]] for k, v in b.items()} for r in range(world)]
        outs, latest, _, _ = _stage_batch(engines, lib, shards, epoch)
        exp = ora.process_batch(**b)
        got = {}
        for t in outs:
            for k in range(len(t)):
                key = (int(t.cell[k]), int(t.window_start_us[k]))
                assert key not in got
                got[key] = (int(t.count[k]), float(t.avg_lat[k]))
        o = {(x["cell"], x["window_start_us"]): (x["count"], x["avg_lat"]) for x in exp["tiles"]}
        assert set(got) == set(o)
        assert all(got[k][0] == o[k][0] and abs(got[k][1] - o[k][1]) <= 1e-9 * abs(o[k][1]) for k in got)
        rows = np.sort(np.concatenate([latest[r] + bounds[r] for r in range(world)]))
        np.testing.assert_array_equal(rows, exp["latest_rows"])
    for e in engines:
        e.close()


def _check_union(outs, latest, bounds, exp):
    got = {}
    for t in outs:
        for k in range(len(t)):
            key = (int(t.cell[k]), int(t.window_start_us[k]))
            assert key not in got, "a key emitted by two owners"
            got[key] = (int(t.count[k]), float(t.avg_lat[k]), float(t.avg_lon[k]))
    o = {(x["cell"], x["window_start_us"]): (x["count"], x["avg_lat"], x["avg_lon"]) for x in exp["tiles"]}
    assert set(got) == set(o)
    for k, g in got.items():
        assert g[0] == o[k][0]
        assert abs(g[1] - o[k][1]) <= 1e-9 * abs(o[k][1]) and abs(g[2] - o[k][2]) <= 1e-9 * abs(o[k][2])
    rows = np.sort(np.concatenate([latest[r] + bounds[r] for r in range(len(latest))]))
    np.testing.assert_array_equal(rows, exp["latest_rows"])


@pytest.mark.parametrize("world", [2, 4])
def test_stage_api_table_mode_c3(world, monkeypatch, capsys):
    """C3-shaped shards (Zipf hot spots, res 9) with the table-mode aggregation pinned: every rank sends exactly
    one 48-B partial per distinct (cell, window) key of its shard (what the exchange carries instead of rows), and
    the owners' union equals the single-shard oracle over two advancing batches.  Per-rank send counts and bytes
    are printed (C3's exchange scales with its keys, not with its 1e9 rows)."""
    monkeypatch.setenv("MOBHEAT_INGEST_MODE", "table")
    import mobheat
    from mobheat import synth
    from mobheat._lib import HM_CAND_REC_BYTES, HM_TILE_REC_BYTES
    from oracle.spark_oracle import SparkHeatmapOracle
    lib = mobheat.load()
    engines = [mobheat.HeatmapEngine(h3_res=9) for _ in range(world)]
    ora = SparkHeatmapOracle(h3_res=9)
    n = 400_000
    log = []
    for epoch in range(2):
        b = synth.c3_city(seed=20 + epoch, n=n, hotspots=300, n_vehicles=5000)
        b["ts_us"] = b["ts_us"] + epoch * 6 * 60_000_000
        bounds = [i * n // world for i in range(world + 1)]
        shards = [{k: v[bounds[r]:bounds[r + 1]] for k, v in b.items()} for r in range(world)]
        outs, latest, tc, cc = _stage_batch(engines, lib, shards, epoch)
        exp = ora.process_batch(**b)
        _check_union(outs, latest, bounds, exp)
        for r in range(world):
            keys_r = len(SparkHeatmapOracle(h3_res=9).process_batch(**shards[r])["tiles"])
            # one record per key (a key spills a second one only when an LDS probe or a bucket overflows: rare)
            assert keys_r <= sum(tc[r]) <= keys_r * 1.02 + 16, (r, sum(tc[r]), keys_r)
            tb, cb = sum(tc[r]) * HM_TILE_REC_BYTES, sum(cc[r]) * HM_CAND_REC_BYTES
            log.append((epoch, r, shards[r]["lat"].size, sum(tc[r]), tb, sum(cc[r]), cb))
            # a rank's tile exchange is bounded by its distinct keys, not by its rows (here ~30 rows per key)
            assert sum(tc[r]) * 8 <= shards[r]["lat"].size
    with capsys.disabled():
        for e, r, rows, nt, tb, nc, cb in log:
            print(f"\n[c3 table, world {world}] batch {e} rank {r}: {rows} rows -> {nt} tile partials ({tb} B), "
                  f"{nc} latest candidates ({cb} B); tile bytes per 1e6 rows {tb * 1e6 / rows:.0f}")
    for e in engines:
        e.close()


@pytest.mark.parametrize("world", [3, 4])
def test_stage_api_c5_vehicles_straddle_ranks(world, capsys):
    """C5-shaped batch: every vehicle's updates are permuted across all ranks and 5% of the vehicles have two rows
    tied at their max timestamp.  The owner of a vehicle must keep exactly the rows at the global max (both tied
    rows, whichever ranks they came from) and route them back to their origin ranks; tiles equal the oracle too."""
    import mobheat
    from mobheat import synth
    from mobheat._lib import HM_CAND_REC_BYTES
    from oracle.spark_oracle import SparkHeatmapOracle
    lib = mobheat.load()
    engines = [mobheat.HeatmapEngine(h3_res=9) for _ in range(world)]
    b = synth.c5_dedup(seed=40 + world, n_vehicles=30_000, updates=12, tie_frac=0.05)
    n = b["lat"].size
    bounds = [i * n // world for i in range(world + 1)]
    shards = [{k: v[bounds[r]:bounds[r + 1]] for k, v in b.items()} for r in range(world)]
    # every vehicle straddles the ranks (12 updates over `world` shards)
    owners_per_vehicle = np.zeros(30_000, np.int64)
    for r in range(world):
        owners_per_vehicle += np.bincount(shards[r]["vkey"].astype(np.int64), minlength=30_000) > 0
    assert (owners_per_vehicle >= 2).mean() > 0.99
    outs, latest, tc, cc = _stage_batch(engines, lib, shards, 0)
    exp = SparkHeatmapOracle(h3_res=9).process_batch(**b)
    _check_union(outs, latest, bounds, exp)
    n_ties = len(exp["latest_rows"]) - 30_000
    assert n_ties > 1000   # both tied rows of ~5% of the vehicles are kept
    with capsys.disabled():
        for r in range(world):
            print(f"\n[c5, world {world}] rank {r}: {bounds[r + 1] - bounds[r]} rows -> {sum(cc[r])} latest candidates "
                  f"({sum(cc[r]) * HM_CAND_REC_BYTES} B) to {world} owners {cc[r]}; tile partials {sum(tc[r])}")
    for e in engines:
        e.close()
