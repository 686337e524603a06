"""CPU, world_size 2 over gloo: the sharded path (mobheat.distributed.ShardedHeatmap) -- ingest, all_gather of the
ranks' summaries, the batch-wide decisions (global window registry, max event time), one chunk per destination
(direct path: 32-B records grouped by region field with per-field counts and a window census; table mode: 48-B tile
partials; 32-B latest candidates: tests/stage_chunks.py), one all_to_all of the chunk sizes then one of the chunks,
owner merge, winners routed back -- must produce exactly the single-shard result.

The stages here are a numpy restatement of hm_stage_ingest / send / merge / finish built on the oracle (test-only
stand-in for the GPU) that writes the library's wire formats; the orchestration, exchange code, owner functions and
the global registry rule (distributed.global_window_registry, the twin of the library's) are the product's.
tests/test_gpu_stages.py runs the same protocol through the HIP library on one GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from stage_chunks import CAND_DT, CENSUS_WORDS, EVENT_DT, TILE_DT, pack, unpack
CELL_LO = (1 << 52) - 1
SPEED_NULL = 0x7FF0000000000001
I64_MIN = np.iinfo(np.int64).min


def _wenc(ws):
    return (np.asarray(ws, np.int64).view(np.uint64) ^ np.uint64(1 << 63))


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()) if a.size else torch.zeros(8, dtype=torch.uint8)


class OracleStages:
    def __init__(self, res, table=False, tile_us=300_000_000, delay_ms=600_000):
        from oracle.spark_oracle import SparkHeatmapOracle
        self.o = SparkHeatmapOracle(h3_res=res, tile_us=tile_us, watermark_delay_ms=delay_ms)
        self.res = res
        self.table = table

    def ingest(self, epoch, b, world, rank):
        from mobheat import _lib
        from mobheat.distributed import SW_AGG, SW_MAX_MS, SW_N_IN, SW_NWIN, SW_VALID, SW_WIN0
        from oracle import h3_oracle
        o = self.o
        self.b, self.world, self.rank = b, world, rank
        valid = o.valid_mask(b["lat"], b["lon"], b["ts_us"], b["row_valid"])
        ts = b["ts_us"]
        ws = ts - np.mod(ts, o.tile)
        late = valid & (ws + o.tile <= o.wm_prev * 1000)
        self.valid = valid
        self.agg = agg = np.nonzero(valid & ~late)[0]
        self.cells = h3_oracle.latlng_to_cell(b["lat"][agg], b["lon"][agg], self.res)
        self.ws = ws[agg]
        v = np.nonzero(valid)[0]
        S = np.zeros(_lib.HM_STAGE_SUMMARY_WORDS, np.int64)
        S[SW_N_IN], S[SW_VALID], S[SW_AGG] = ts.size, v.size, agg.size
        S[SW_MAX_MS] = int(np.max(np.floor_divide(ts[v], 1000))) if v.size else I64_MIN
        wins = np.unique(self.ws)
        S[SW_NWIN] = wins.size
        S[SW_WIN0: SW_WIN0 + 2 * wins.size: 2] = np.arange(wins.size)          # this rank's slots
        S[SW_WIN0 + 1: SW_WIN0 + 2 * wins.size: 2] = _wenc(wins).view(np.int64)
        return S

    def send(self, summaries):
        from mobheat.distributed import SW_MAX_MS, global_window_registry, region_field, shard_lo, tile_hash, tile_owner
        o, b, world, rank = self.o, self.b, self.world, self.rank
        self.gmax = int(max(S[SW_MAX_MS] for S in summaries))
        self.reg = global_window_registry(summaries, o.tile)
        gslot = {we: i for i, we in enumerate(self.reg) if we}
        agg, cells, ws = self.agg, self.cells, self.ws
        if self.table:
            recs = np.zeros(0, TILE_DT)
            if agg.size:
                keys = np.rec.fromarrays([cells, ws], names="c,w")
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
            own = tile_owner(recs["cell"], recs["ws"], world)
            per_dest = [(recs[own == d], None, None, None) for d in range(world)]
        else:
            slot = np.array([gslot[int(w)] for w in _wenc(ws)], np.int64)
            recs = np.zeros(agg.size, EVENT_DT)
            recs["key"] = (cells & np.uint64(CELL_LO)) | ((slot + 1).astype(np.uint64) << np.uint64(52))
            sv, sp = b["speed_valid"][agg], b["speed"][agg]
            bits = np.where(np.isnan(sp), np.uint64(0x7FF8000000000000), sp.view(np.uint64))
            recs["sp"] = np.where(sv, bits, np.uint64(SPEED_NULL))
            recs["lat"], recs["lon"] = b["lat"][agg], b["lon"][agg]
            field = region_field(tile_hash(cells, ws))
            order = np.argsort(field, kind="stable")
            recs, field, slot = recs[order], field[order], slot[order]
            per_dest = []
            for d in range(world):
                lo, hi = shard_lo(d, world), shard_lo(d + 1, world)
                m = (field >= lo) & (field < hi)
                per_dest.append((recs[m], hi - lo, np.bincount(field[m] - lo, minlength=hi - lo).astype(np.uint32),
                                 np.bincount(slot[m], minlength=CENSUS_WORDS).astype(np.uint32)))
        # local latest candidates: rows tied at the local max of their vehicle
        v = np.nonzero(self.valid)[0]
        ts = b["ts_us"]
        cands = np.zeros(0, CAND_DT)
        if v.size:
            vk, tv = b["vkey"][v], ts[v]
            srt = np.lexsort((tv, vk))
            last = np.r_[vk[srt][1:] != vk[srt][:-1], True]
            grp = np.cumsum(np.r_[True, vk[srt][1:] != vk[srt][:-1]]) - 1
            win = srt[tv[srt] == tv[srt][last][grp]]
            cands = np.zeros(win.size, CAND_DT)
            cands["vkey"], cands["ts"], cands["row"], cands["origin"] = vk[win], tv[win], v[win], rank
        from mobheat.distributed import vkey_owner
        cown = vkey_owner(cands["vkey"], world)
        chunks = [pack(r, cands[cown == d], bins, cnt, cen) for d, (r, bins, cnt, cen) in enumerate(per_dest)]
        return _t(np.concatenate(chunks)), [c.size for c in chunks]

    def merge(self, recv, recv_bytes, out_memory):
        from mobheat.distributed import Stream
        o = self.o
        got, cands, _ = unpack(recv.numpy()[: sum(recv_bytes)], recv_bytes, direct=not self.table)
        if self.table:
            recs = got
        else:
            n = got.size
            key = got["key"]
            pay = got
            wenc = np.array(self.reg, np.uint64)[(key >> np.uint64(52)).astype(np.int64) - 1]
            recs = np.zeros(n, TILE_DT)
            recs["cell"] = (key & np.uint64(CELL_LO)) | np.uint64((1 << 59) | (self.res << 52))
            recs["ws"] = (wenc ^ np.uint64(1 << 63)).view(np.int64)
            recs["count"] = 1
            null = pay["sp"] == np.uint64(SPEED_NULL)
            recs["nsp"] = ~null
            recs["ssp"] = np.where(null, 0.0, pay["sp"].view(np.float64))
            recs["slat"], recs["slon"] = pay["lat"], pay["lon"]
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
        nxt = o.wm_cur if self.gmax == I64_MIN else max(o.wm_cur, self.gmax - o.delay)
        o.wm_prev, o.wm_cur = o.wm_cur, nxt
        world = self.world
        rows_by_origin = [[] for _ in range(world)]
        if cands.size:
            srt = np.lexsort((cands["ts"], cands["vkey"]))
            vk = cands["vkey"][srt]
            last = np.r_[vk[1:] != vk[:-1], True]
            grp = np.cumsum(np.r_[True, vk[1:] != vk[:-1]]) - 1
            win = srt[cands["ts"][srt] == cands["ts"][srt][last][grp]]
            for w in win:
                rows_by_origin[int(cands["origin"][w])].append(int(cands["row"][w]))
        flat = np.array([r for x in rows_by_origin for r in x], np.int64)
        return {"tiles": tiles}, Stream("winner", _t(flat), [len(x) for x in rows_by_origin], 8)

    def finish(self, winner_recv, n, out_memory, out):
        out["latest"] = np.sort(winner_recv.numpy()[: n * 8].view(np.int64))
        return out


def _worker(rank, world, port, batches, res, table, q, round_bytes=None, meta=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mobheat import distributed
    from mobheat.distributed import ShardedHeatmap
    if round_bytes:   # (the payload exchanged in rounds of at most this many bytes per rank pair)
        distributed.EXCHANGE_ROUND_BYTES = round_bytes
    if meta:   # (the host metadata over a group of its own, as under RCCL)
        distributed.META_BACKEND = "gloo"
    sh = ShardedHeatmap(OracleStages(res, table=table), torch.device("cpu"))
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


@pytest.mark.parametrize("table,round_bytes,meta,world", [(False, None, False, 2), (True, None, False, 2),
                                                           (False, 4096, False, 2), (False, None, True, 2),
                                                           (False, 4096, False, 3), (True, None, True, 3)])
def test_sharded_equals_single_shard(oracle_h3, table, round_bytes, meta, world):
    """world 2 and 3 over gloo, the payload exchanged in one call or in rounds of 4 KiB per rank pair (the chunked
    exchange), the host metadata over the same group or a separate one: the union of the shards equals one engine."""
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
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batches, 8, table, q, round_bytes, meta))
             for r in range(world)]
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
        latest = sorted(x for r in range(world) for x in got[r][e][1])
        assert latest == exp["latest_rows"].tolist()


def _scatter_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mobheat import distributed
    distributed.EXCHANGE_ROUND_BYTES = 64   # (rounds of 8 words per rank pair)
    if rank == 0:   # rank 0 alone sends: rank r gets words [sum(sizes[:r]), ...)
        sizes = [8 * (20 + 7 * r) for r in range(world)]
        buf = torch.arange(sum(sizes) // 8, dtype=torch.int64).view(torch.uint8)
        recv, rb = distributed.exchange_chunks(buf, sizes, torch.device("cpu"))
    else:
        recv, rb = distributed.exchange_chunks(None, [0] * world, torch.device("cpu"))
    q.put((rank, rb, recv.view(torch.int64)[: sum(rb) // 8].tolist()))
    dist.destroy_process_group()


def test_exchange_from_one_sender_in_rounds():
    """The sharded writer's device-column scatter pattern (sharded.ShardedStream.process_device): rank 0 alone sends,
    every rank (rank 0 too) receives its slice, moved in rounds (distributed.EXCHANGE_ROUND_BYTES)"""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (rb, w)) for r, rb, w in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    start = 0
    for r in range(world):
        n = 20 + 7 * r
        assert got[r][0] == [8 * n] + [0] * (world - 1)
        assert got[r][1] == list(range(start, start + n))
        start += n


def _cap_worker(rank, world, port, q):
    """exchange_chunks and exchange under round sizes the cap must clamp, every all_to_all call's per-pair element
    counts recorded"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mobheat import distributed
    calls = []
    real_single = distributed.dist.all_to_all_single

    def rec_single(out, inp, out_split=None, in_split=None, **kw):
        calls.append(max(list(out_split or [out.numel() // world]) + list(in_split or [inp.numel() // world])))
        return real_single(out, inp, out_split, in_split, **kw)

    distributed.dist.all_to_all_single = rec_single
    distributed.EXCHANGE_ROUND_CAP = 256   # (bytes per pair and call: 32 words)
    got = []
    try:
        for asked in (0, -8, 1 << 40, 100, 256):
            distributed.EXCHANGE_ROUND_BYTES = asked
            # chunk for rank r: 8 * (37 * (rank + 1) + 11 * r) bytes, words numbered by (sender, receiver, index)
            sizes = [8 * (37 * (rank + 1) + 11 * r) for r in range(world)]
            words = np.concatenate([(rank * 1000 + r * 100000) * 1000 + np.arange(s // 8) for r, s in enumerate(sizes)])
            first = len(calls)
            recv, rb = distributed.exchange_chunks(torch.from_numpy(words).view(torch.uint8), sizes, torch.device("cpu"))
            payload_calls = calls[first + 0:]   # (exchange_chunks' size matrix moves by all_gather: not recorded)
            # the winners' form: 8-B records
            st = distributed.Stream("w", torch.from_numpy(words).view(torch.uint8), [s // 8 for s in sizes], 8)
            first_w = len(calls)
            [(wrecv, wrc)] = distributed.exchange([st], torch.device("cpu"))
            got.append((asked, rb, recv.view(torch.int64)[: sum(rb) // 8].tolist(), payload_calls, wrc,
                        wrecv.view(torch.int64)[: sum(wrc)].tolist(), calls[first_w + 1:]))
    finally:
        distributed.dist.all_to_all_single = real_single
    q.put((rank, got))
    dist.destroy_process_group()


def test_exchange_round_cap():
    """no all_to_all call moves more than distributed.EXCHANGE_ROUND_CAP bytes per rank pair,
    whatever MOBHEAT_EXCHANGE_ROUND_BYTES asks (0, negative, above the cap: the cap; below it: that size), and the
    pieces land where one call would put them"""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cap_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        for asked, rb, words, calls, wrc, wwords, wcalls in got[rank]:
            cap_words = (256 if asked <= 0 or asked > 256 else asked) // 8
            assert calls and max(calls) <= cap_words, (asked, calls)
            assert wcalls and max(wcalls) <= cap_words, (asked, wcalls)
            # the biggest piece is 8 * (37 * 2 + 11) = 680 B: several rounds under the cap
            assert len(calls) >= 3 and len(wcalls) >= 3
            exp_rb = [8 * (37 * (s + 1) + 11 * rank) for s in range(world)]
            exp = [w for s in range(world) for w in ((s * 1000 + rank * 100000) * 1000 + np.arange(exp_rb[s] // 8))]
            assert rb == exp_rb and words == exp
            assert wrc == [b // 8 for b in exp_rb] and wwords == exp
