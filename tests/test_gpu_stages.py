"""GPU: the multi-GPU stage API (hm_stage_ingest / send / merge / finish) through the HIP library, with W contexts
("virtual ranks") on one device and the exchanges routed on the host, plus the product's ShardedHeatmap driver over
two gloo processes sharing the GPU (RCCL needs one GPU per rank).  The union of the owners' outputs must equal the
single-shard result (oracle), batch after batch (state ownership is stable).
"""
import ctypes
import os
import socket

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
    """One micro-batch through the stage API of W contexts, exchanges routed on the host.  Returns the owners' tiles,
    each rank's latest rows, per-rank tile/candidate send counts and whether table mode ran."""
    from mobheat._lib import HM_MEM_HOST, HM_STAGE_SUMMARY_WORDS, HmBatchIn, HmBatchOut, HmStageSizes, check
    W = len(engines)
    bufs, keep = [], []
    summaries = np.zeros((W, HM_STAGE_SUMMARY_WORDS), np.int64)
    for r, (eng, b) in enumerate(zip(engines, batches_per_rank)):
        n = b["lat"].size
        k = {kk: np.ascontiguousarray(v) for kk, v in b.items()}
        k["sv"], k["rv"] = k["speed_valid"].astype(np.uint8), k["row_valid"].astype(np.uint8)
        keep.append(k)
        bi = HmBatchIn(n=n, memory=HM_MEM_HOST, lat=k["lat"].ctypes.data, lon=k["lon"].ctypes.data,
                       ts_us=k["ts_us"].ctypes.data, speed=k["speed"].ctypes.data, speed_valid=k["sv"].ctypes.data,
                       vkey=k["vkey"].ctypes.data, row_valid=k["rv"].ctypes.data)
        check(lib.hm_stage_ingest(eng._ctx, epoch, ctypes.byref(bi), W, r, summaries[r].ctypes.data), eng._ctx)
    from stage_chunks import unpack
    sends, sbytes, tcounts, ccounts, table, self_recs = [], [], [], [], None, []
    for r, (eng, b) in enumerate(zip(engines, batches_per_rank)):
        n = b["lat"].size
        cap = lib.hm_stage_send_capacity(n, W)
        sb_ = DevBuf(lib, cap)
        bufs.append(sb_)
        sb = (ctypes.c_int64 * W)()
        sz = HmStageSizes()
        check(lib.hm_stage_send(eng._ctx, summaries.ctypes.data, sb_.p, cap, sb, ctypes.byref(sz)), eng._ctx)
        assert table is None or table == bool(sz.table_mode), "ranks disagree on the aggregation path"
        table = bool(sz.table_mode)
        assert sz.global_batch_max_event_ms == max(summaries[:, 4])
        raw = sb_.get(sum(sb))
        sends.append(raw)
        sbytes.append(list(sb))
        off, tc, cc = 0, [], []
        for d in range(W):   # each destination's chunk: its header's record and candidate counts
            h = raw[off: off + 64].view(np.int64)
            tc.append(int(h[1]))
            cc.append(int(h[2]))
            off += sb[d]
        tcounts.append(tc)
        ccounts.append(cc)
        if not table:   # one 32-B record per aggregated row of the rank (its own bins' ones may stay in its slabs)
            assert sum(tc) + sz.n_self_records == summaries[r][3] == sz.n_tile_records
            assert sz.n_self_records == 0 or tc[r] == 0
        self_recs.append(sz.n_self_records)

    outs, wsends, wcounts = [], [], []
    for r, eng in enumerate(engines):
        parts = [sends[s][sum(sbytes[s][:r]): sum(sbytes[s][:r + 1])] for s in range(W)]
        recv = np.concatenate(parts)
        rbytes = [p.size for p in parts]
        recs, cands, _ = unpack(recv, rbytes, direct=not table)
        nc = cands.size
        rb_, wb = DevBuf(lib, recv.nbytes), DevBuf(lib, max(nc, 1) * 8)
        bufs += [rb_, wb]
        rb_.put(recv)
        out = HmBatchOut()
        wc = (ctypes.c_int64 * W)()
        check(lib.hm_stage_merge(eng._ctx, rb_.p, (ctypes.c_int64 * W)(*rbytes), HM_MEM_HOST, ctypes.byref(out), wb.p,
                                 max(nc, 1), wc), eng._ctx)
        res = eng._result_from_host(out)
        outs.append(res.tiles)
        wcounts.append(list(wc))
        wsends.append(wb.get(sum(wc) * 8).view(np.int64))
        c = eng.last_counts()
        assert c["partials"] == recs.size + self_recs[r] and c["tiles"] == len(res.tiles)
        assert c["sent"] == sum(tcounts[r]) + self_recs[r]
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
    return outs, latest, tcounts, ccounts, table


@pytest.mark.parametrize("world,mode", [(2, "direct"), (3, "direct"), (2, "table"), (2, "binned"), (3, "binned")])
def test_stage_api_matches_single_shard(world, mode, monkeypatch):
    """Both aggregation paths pinned, four batches (one empty): on the direct path every aggregated row crosses as one
    32-B record (the key with the batch's global window slot) grouped by region field, and the owner merges each of its
    bins from the senders' segments with the single-GPU merge."""
    monkeypatch.setenv("MOBHEAT_INGEST_MODE", mode)
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
        outs, latest, _, _, _ = _stage_batch(engines, lib, shards, epoch)
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
        outs, latest, tc, cc, table = _stage_batch(engines, lib, shards, epoch)
        assert table
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
    outs, latest, tc, cc, _ = _stage_batch(engines, lib, shards, 0)
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


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def _batches_for_dist():
    from mobheat import synth
    rng = np.random.default_rng(77)
    out = []
    for start, n in ((0, 200_000), (7, 200_000), (0, 0), (20, 150_000)):
        b = synth.c2_global(seed=start + 3, n=max(n, 1))
        b = {k: v[:n] for k, v in b.items()}
        b["ts_us"] = synth.T0 + start * 60_000_000 + rng.integers(0, 9 * 60_000_000, n)
        out.append(b)
    return out


def _dist_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import mobheat
    from mobheat._lib import HM_MEM_HOST
    from mobheat.distributed import LibStages, ShardedHeatmap
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    eng = mobheat.HeatmapEngine(h3_res=8, device=0)
    sh = ShardedHeatmap(LibStages(eng), dev)
    res = []
    for e, b in enumerate(_batches_for_dist()):
        n = b["lat"].size
        lo, hi = rank * n // world, (rank + 1) * n // world
        cols = {}
        for k, v in b.items():
            a = np.ascontiguousarray(v[lo:hi])
            a = a.view(np.int64) if a.dtype == np.uint64 else a.astype(np.uint8) if a.dtype == bool else a
            cols[k] = torch.from_numpy(a).to(dev)
        ptrs = dict(n=hi - lo, **{k: v.data_ptr() for k, v in cols.items()})
        out = sh.process_batch(e, ptrs, out_memory=HM_MEM_HOST)
        r = eng._result_from_host(out)
        t = r.tiles
        tiles = {(int(t.cell[k]), int(t.window_start_us[k])): (int(t.count[k]), float(t.avg_lat[k])) for k in range(len(t))}
        res.append((tiles, (np.asarray(r.latest_rows) + lo).tolist(), eng.last_counts()))
        torch.cuda.synchronize()
    q.put((rank, res))
    dist.barrier()
    eng.close()
    dist.destroy_process_group()


def test_sharded_driver_two_processes_gloo_on_gpu():
    """The product's driver (mobheat.distributed: summaries all_gather, one counts all_to_all, the key/payload/candidate
    streams, winners back) over two processes that share the GPU, gloo moving the device tensors: every batch's union
    of the owners' tiles and latest rows equals the single-shard oracle, and hm_last_counts reports each rank's share
    (the bench's N>1 line prices its roofline on them)."""
    import torch.multiprocessing as mp
    from oracle.spark_oracle import SparkHeatmapOracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ora = SparkHeatmapOracle(h3_res=8)
    for e, b in enumerate(_batches_for_dist()):
        exp = ora.process_batch(**b)
        tiles = {}
        for r in range(world):
            assert not set(got[r][e][0]) & set(tiles), "a key emitted by two owners"
            tiles.update(got[r][e][0])
        o = {(x["cell"], x["window_start_us"]): (x["count"], x["avg_lat"]) for x in exp["tiles"]}
        assert set(tiles) == set(o)
        assert all(tiles[k][0] == o[k][0] and abs(tiles[k][1] - o[k][1]) <= 1e-9 * abs(o[k][1]) for k in tiles)
        assert sorted(got[0][e][1] + got[1][e][1]) == exp["latest_rows"].tolist()
        counts = [got[r][e][2] for r in range(world)]
        assert sum(c["tiles"] for c in counts) == len(o)
        assert sum(c["partials"] for c in counts) == sum(c["sent"] for c in counts)
        if b["lat"].size:
            assert all(c["tiles"] > 0 and c["partials"] > 0 for c in counts)
