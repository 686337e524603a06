"""GPU: the multi-GPU code path over RCCL itself (torch.distributed backend "nccl"), at world size 1 on the box's one GPU.

RCCL refuses two ranks on one device, so the N>1 tests elsewhere move their exchanges with gloo; a world of ONE rank
runs every nccl-only line of the sharded path on one GPU: `init_process_group(..., device_id=...)`, the summaries'
all_gather, the uneven-split int64 `all_to_all_single` of the record chunks (a rank sending its whole share to itself),
the winners' exchange, and the ordering of RCCL's stream (torch's current stream) against the library's own
(distributed.py).  The results must equal the single-engine path on the same batches (reference heatmap_stream.py:44,
112-133,198-207: the shuffle this exchange replaces): tiles (cells, windows, counts bit-exact; dyadic inputs, so every
fp64 sum is exact and the averages bit-exact too) and latest rows; behind foreach_batch_func (MOBHEAT_SHARDED=1 runs the
sharded writer at one GPU), the statements byte for byte.  Each case runs in a spawned process of its own: it owns a
process group.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

T0 = 1759572000


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def _batches():
    """dyadic C2-like batches (exact fp64 sums): 300k rows, an empty batch, and 4.5M rows (k_ingest bins its records
    above 4M rows, so the sender's pack reads k_ingest's own bins)"""
    rng = np.random.default_rng(5)
    out = []
    for start, n in ((0, 300_000), (7, 0), (20, 4_500_000), (27, 300_000)):
        lat = np.degrees(np.arcsin(rng.integers(-(1 << 20), 1 << 20, n) / float(1 << 20)))
        lat = np.round(lat * 4096.0) / 4096.0
        lon = (rng.integers(0, 360 * 4096, n) / 4096.0) - 180.0
        ts = (T0 + start * 60) * 1_000_000 + rng.integers(0, 9 * 60_000_000, n)
        speed = rng.integers(0, 160, n) * 0.5
        sv = (rng.random(n) >= 0.1).astype(np.uint8)
        vkey = rng.integers(0, 50_000, n).astype(np.uint64)
        out.append(dict(lat=lat, lon=lon, ts_us=ts, speed=speed, speed_valid=sv, vkey=vkey,
                        row_valid=np.ones(n, np.uint8)))
    return out


def _tiles(r):
    t = r.tiles
    return {(int(t.cell[k]), int(t.window_start_us[k])): (int(t.count[k]), float(t.avg_speed[k]), bool(t.speed_null[k]),
                                                           float(t.avg_lat[k]), float(t.avg_lon[k]))
            for k in range(len(t))}


def _stage_worker(port, round_bytes, q):
    """ShardedHeatmap over RCCL at world 1 against HeatmapEngine.process_batch on the same batches."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as dist
        import mobheat
        from mobheat import distributed
        if round_bytes:   # (the record exchange in rounds of at most this many bytes per rank pair: RCCL's list form)
            distributed.EXCHANGE_ROUND_BYTES = round_bytes
        from mobheat._lib import HM_MEM_HOST
        from mobheat.distributed import LibStages, ShardedHeatmap
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        backend = dist.get_backend()
        eng = mobheat.HeatmapEngine(h3_res=8, device=0)
        ref = mobheat.HeatmapEngine(h3_res=8, device=0)
        sh = ShardedHeatmap(LibStages(eng), dev)
        res = []
        for e, b in enumerate(_batches()):
            n = b["lat"].size
            cols = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.int64) if v.dtype == np.uint64 else
                                        np.ascontiguousarray(v)).to(dev) for k, v in b.items()}
            ptrs = dict(n=n, **{k: v.data_ptr() for k, v in cols.items()})
            got = eng._result_from_host(sh.process_batch(e, ptrs, out_memory=HM_MEM_HOST))
            exp = ref.process_batch(e, b["lat"], b["lon"], b["ts_us"], b["speed"], b["speed_valid"], b["vkey"],
                                    b["row_valid"])
            c = eng.last_counts()
            same_tiles = _tiles(got) == _tiles(exp)
            same_latest = np.asarray(got.latest_rows).tolist() == np.asarray(exp.latest_rows).tolist()
            res.append(dict(epoch=e, n=n, tiles=len(got.tiles), exp_tiles=len(exp.tiles), same_tiles=same_tiles,
                            same_latest=same_latest, latest=len(got.latest_rows), binned=bool(c.get("binned")),
                            sent=int(c["sent"]), partials=int(c["partials"]),
                            watermark=(int(got.watermark_ms), int(exp.watermark_ms))))
            torch.cuda.synchronize()
        eng.close()
        ref.close()
        dist.destroy_process_group()
        q.put(("ok", backend, res))
    except BaseException as e:   # (the parent reports it)
        import traceback
        q.put(("err", repr(e), traceback.format_exc()))


def _frames():
    import pandas as pd
    rng = np.random.default_rng(23)
    out = []
    for b in range(4):
        n = 50_000
        lat = 42.0 + rng.integers(0, 1 << 14, n) / 65536.0
        lon = -71.25 + rng.integers(0, 1 << 14, n) / 65536.0
        sp = pd.array(rng.integers(0, 160, n) * 0.5, dtype="Float64")
        sp[rng.random(n) < 0.1] = pd.NA
        ts = T0 + b * 240 + rng.integers(0, 360, n)
        ts[: n // 50] = ts[n // 50: 2 * (n // 50)]
        veh = rng.integers(0, 2000, n)
        out.append(pd.DataFrame({"provider": np.where(veh % 7 == 0, "mbta", "opensky"),
                                 "vehicleId": [f"v{v:04d}" for v in veh], "lat": lat, "lon": lon, "speedKmh": sp,
                                 "eventTs": pd.to_datetime(ts, unit="s", utc=True)}))
    return out


class _Capture:
    log = []

    def __init__(self):
        self.cur = {"tiles": [], "positions_latest": []}
        _Capture.log.append(self.cur)

    def update_raw(self, collection, statements):
        self.cur[collection].extend(bytes(s.raw) for s in statements)

    def close(self):
        pass


def _stream_worker(ckdir, q):
    """foreach_batch_func: the single-GPU path, then the sharded writer forced at one GPU over RCCL."""
    try:
        import torch
        torch.cuda.init()   # (torch's runtime first: its init fails once the library's copy has been working, conftest)
        from mobheat import stream
        frames = _frames()
        stream.SINK_FACTORY = _Capture
        stream.CHECKPOINT_DIR = os.path.join(ckdir, "single")
        for e, f in enumerate(frames):
            stream.foreach_batch_func(f, e)
        ref = [sorted(c["tiles"]) + sorted(c["positions_latest"]) for c in _Capture.log]
        stream.reset_engine()
        _Capture.log.clear()
        stream.FORCE_SHARDED = True
        stream.DIST_BACKEND = "nccl"
        stream.CHECKPOINT_DIR = os.path.join(ckdir, "sharded")
        for e, f in enumerate(frames):
            stream.foreach_batch_func(f, e)
        import torch.distributed as dist
        backend = dist.get_backend()
        world = dist.get_world_size()
        got = [sorted(c["tiles"]) + sorted(c["positions_latest"]) for c in _Capture.log]
        stream.close_sharded()
        q.put(("ok", backend, world, [len(x) for x in ref], [g == r for g, r in zip(got, ref)]))
    except BaseException as e:
        import traceback
        q.put(("err", repr(e), traceback.format_exc()))


def _spawn(target, *args, timeout=300):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=target, args=args + (q,))
    p.start()
    try:
        m = q.get(timeout=timeout)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert m[0] == "ok", f"{m[1]}\n{m[2]}"
    assert p.exitcode == 0
    return m


@pytest.mark.parametrize("round_bytes", [0, 16 << 20])
def test_sharded_heatmap_over_rccl_world1_equals_single_engine(round_bytes):
    """ShardedHeatmap (summaries all_gather, chunk all_to_all, owner merge, winners back) over RCCL: every batch's tiles
    and latest rows equal the single-engine path's, including a 4.5M-row batch whose records k_ingest binned; with a
    16-MiB round size the 144-MB record exchange of that batch moves in rounds (distributed.EXCHANGE_ROUND_BYTES)."""
    m = _spawn(_stage_worker, _free_port(), round_bytes)
    _, backend, res = m
    assert backend == "nccl"
    for r in res:
        print(f"[rccl] {r}", flush=True)
        assert r["same_tiles"] and r["same_latest"], r
        assert r["tiles"] == r["exp_tiles"]
        assert r["watermark"][0] == r["watermark"][1]
        if r["n"]:
            assert r["tiles"] > 0 and r["latest"] > 0 and r["sent"] == r["partials"]
    assert any(r["binned"] for r in res)


def test_foreach_batch_func_sharded_writer_over_rccl_world1(tmp_path):
    """foreach_batch_func with the sharded writer (mobheat.sharded) forced at one GPU over RCCL writes the single-GPU
    path's tiles and positions_latest statements byte for byte, batch after batch."""
    m = _spawn(_stream_worker, str(tmp_path))
    _, backend, world, sizes, same = m
    print(f"[rccl] backend {backend} world {world} statements per batch {sizes}", flush=True)
    assert backend == "nccl" and world == 1
    assert all(s > 1000 for s in sizes)
    assert all(same), same
