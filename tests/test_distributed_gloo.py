"""CPU, world_size 2 over gloo: the sharded path (mobheat.distributed.ShardedHeatmap) -- local stage,
all-to-all of tile partials and latest candidates by owner rank, all-reduce(max) of the batch max event time,
owner merge, winners routed back -- must produce exactly the single-shard result.

The stages here are a numpy restatement of hm_stage_local / hm_stage_merge / hm_stage_finish built on the
oracle (test-only stand-in for the GPU); the orchestration, record layouts, owner functions and exchange
code under test are the product's.  tests/test_gpu_stages.py runs the same decomposition through the HIP
library on one GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

TILE_DT = np.dtype([("cell", "<u8"), ("ws", "<i8"), ("count", "<u4"), ("nsp", "<u4"), ("ssp", "<f8"), ("slat", "<f8"),
                    ("slon", "<f8")])   # HM_TILE_REC_BYTES = 48
CAND_DT = np.dtype([("vkey", "<u8"), ("ts", "<i8"), ("row", "<i8"), ("origin", "<i8")])


class OracleStages:
    def __init__(self, res, tile_us=300_000_000, delay_ms=600_000):
        from oracle.spark_oracle import SparkHeatmapOracle
        self.o = SparkHeatmapOracle(h3_res=res, tile_us=tile_us, watermark_delay_ms=delay_ms)
        self.res = res

    def local(self, epoch, b, world, rank):
        from mobheat.distributed import _owner as owner_of, tile_hash, vkey_owner
        from oracle import h3_oracle
        o = self.o
        valid = o.valid_mask(b["lat"], b["lon"], b["ts_us"], b["row_valid"])
        ts = b["ts_us"]
        ws = ts - np.mod(ts, o.tile)
        late = valid & (ws + o.tile <= o.wm_prev * 1000)
        agg = np.nonzero(valid & ~late)[0]
        cells = h3_oracle.latlng_to_cell(b["lat"][agg], b["lon"][agg], self.res)
        recs = np.zeros(0, TILE_DT)
        if agg.size:
            keys = np.rec.fromarrays([cells, ws[agg]], names="c,w")
            uq, inv = np.unique(keys, return_inverse=True)
            inv = inv.ravel()
            sv = b["speed_valid"][agg]
            recs = np.zeros(uq.size, TILE_DT)
            recs["cell"], recs["ws"] = uq["c"], uq["w"]
            recs["count"] = np.bincount(inv, minlength=uq.size)
            recs["nsp"] = np.bincount(inv, weights=sv.astype(float), minlength=uq.size)
            recs["ssp"] = np.bincount(inv[sv], weights=b["speed"][agg][sv], minlength=uq.size)
            recs["slat"] = np.bincount(inv, weights=b["lat"][agg], minlength=uq.size)
            recs["slon"] = np.bincount(inv, weights=b["lon"][agg], minlength=uq.size)
        own = owner_of(tile_hash(recs["cell"], recs["ws"]), world)
        order = np.argsort(own, kind="stable")
        tcounts = np.bincount(own, minlength=world).tolist()
        tile_send = torch.from_numpy(recs[order].view(np.uint8).copy())
        # local latest candidates: rows tied at the local max of their vehicle
        v = np.nonzero(valid)[0]
        cands = np.zeros(0, CAND_DT)
        if v.size:
            vk, tv = b["vkey"][v], ts[v]
            srt = np.lexsort((tv, vk))
            last = np.r_[vk[srt][1:] != vk[srt][:-1], True]
            grp = np.cumsum(np.r_[True, vk[srt][1:] != vk[srt][:-1]]) - 1
            win = srt[tv[srt] == tv[srt][last][grp]]
            cands = np.zeros(win.size, CAND_DT)
            cands["vkey"], cands["ts"], cands["row"], cands["origin"] = vk[win], tv[win], v[win], rank
        cown = vkey_owner(cands["vkey"], world)
        corder = np.argsort(cown, kind="stable")
        ccounts = np.bincount(cown, minlength=world).tolist()
        cand_send = torch.from_numpy(cands[corder].view(np.uint8).copy())
        bmax = int(np.max(np.where(ts[v] >= 0, ts[v] // 1000, -((-ts[v]) // 1000)))) if v.size else np.iinfo(np.int64).min
        return (tile_send if tile_send.numel() else torch.zeros(1, dtype=torch.uint8), tcounts,
                cand_send if cand_send.numel() else torch.zeros(1, dtype=torch.uint8), ccounts, bmax)

    def merge(self, tile_recv, n_tile, cand_recv, n_cand, global_max, out_memory):
        o = self.o
        recs = tile_recv.numpy()[: n_tile * TILE_DT.itemsize].view(TILE_DT)
        touched = []
        for r in recs:
            k = (int(r["cell"]), int(r["ws"]))
            st = o.state.setdefault(k, [0, 0, 0.0, 0.0, 0.0])
            if k not in touched:
                touched.append(k)
            st[0] += int(r["count"]); st[1] += int(r["nsp"]); st[2] += float(r["ssp"])
            st[3] += float(r["slat"]); st[4] += float(r["slon"])
        tiles = {}
        for k in touched:
            c, nsp, ssp, sla, slo = o.state[k]
            tiles[k] = (c, None if nsp == 0 else ssp / nsp, slo / c, sla / c)
        for k in [k for k in o.state if k[1] + o.tile <= o.wm_cur * 1000]:
            del o.state[k]
        nxt = o.wm_cur if global_max == np.iinfo(np.int64).min else max(o.wm_cur, global_max - o.delay)
        o.wm_prev, o.wm_cur = o.wm_cur, nxt
        cands = cand_recv.numpy()[: n_cand * CAND_DT.itemsize].view(CAND_DT)
        world = dist.get_world_size()
        rows_by_origin = [[] for _ in range(world)]
        if cands.size:
            srt = np.lexsort((cands["ts"], cands["vkey"]))
            vk = cands["vkey"][srt]
            last = np.r_[vk[1:] != vk[:-1], True]
            grp = np.cumsum(np.r_[True, vk[1:] != vk[:-1]]) - 1
            win = srt[cands["ts"][srt] == cands["ts"][srt][last][grp]]
            for w in win:
                rows_by_origin[int(cands["origin"][w])].append(int(cands["row"][w]))
        wcounts = [len(x) for x in rows_by_origin]
        flat = np.array([r for x in rows_by_origin for r in x], np.int64)
        send = torch.from_numpy(flat.view(np.uint8).copy()) if flat.size else torch.zeros(1, dtype=torch.uint8)
        return {"tiles": tiles}, send, wcounts

    def finish(self, winner_recv, n, out_memory, out):
        out["latest"] = np.sort(winner_recv.numpy()[: n * 8].view(np.int64))
        return out


def _worker(rank, world, port, batches, res, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mobheat.distributed import ShardedHeatmap
    sh = ShardedHeatmap(OracleStages(res), torch.device("cpu"))
    results = []
    for e, b in enumerate(batches):
        n = b["lat"].size
        lo, hi = rank * n // world, (rank + 1) * n // world
        part = {k: v[lo:hi] for k, v in b.items()}
        part["n"] = hi - lo
        out = sh.process_batch(e, part, sync=lambda: None)
        results.append((out["tiles"], (out["latest"] + lo).tolist()))
    q.put((rank, results))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_equals_single_shard(oracle_h3):
    from mobheat import synth
    from oracle.spark_oracle import SparkHeatmapOracle
    rng = np.random.default_rng(5)
    t0 = synth.T0
    batches = []
    for start, n in ((0, 6000), (12, 6000), (0, 0), (30, 8000)):
        b = synth.c1_boston(seed=start + 1, n=max(n, 100))
        b = {k: v[:n] for k, v in b.items()}
        b["ts_us"] = t0 + start * 60_000_000 + rng.integers(0, 9 * 60_000_000, n)
        b["vkey"] = rng.integers(0, 300, n).astype(np.uint64)
        b["ts_us"][: n // 40] = b["ts_us"][n // 40: 2 * (n // 40)]
        b["speed_valid"] = b["speed_valid"].astype(bool)
        b["row_valid"] = b["row_valid"].astype(bool)
        batches.append(b)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batches, 8, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ora = SparkHeatmapOracle(h3_res=8)
    for e, b in enumerate(batches):
        exp = ora.process_batch(**b)
        tiles = {}
        for r in range(world):
            t = got[r][e][0]
            assert not set(t) & set(tiles), "a key was emitted by two owners"
            tiles.update(t)
        o = {(x["cell"], x["window_start_us"]): x for x in exp["tiles"]}
        assert set(tiles) == set(o)
        for k, (c, sp, lon, lat) in tiles.items():
            assert c == o[k]["count"]
            assert (sp is None) == (o[k]["avg_speed"] is None)
            assert sp is None or abs(sp - o[k]["avg_speed"]) <= 1e-9 * abs(sp)
            assert abs(lat - o[k]["avg_lat"]) <= 1e-9 * abs(lat)
        latest = sorted(got[0][e][1] + got[1][e][1])
        assert latest == exp["latest_rows"].tolist()
