"""CPU, world_size 2 over gloo: the sharded writer behind foreach_batch_func (mobheat.sharded, MOBHEAT_GPUS = 2;
reference heatmap_stream.py:150,159-235,244-245) -- a spawned worker rank, the batch's columns and string dictionaries
handed over in shared memory, every rank encoding the statements of what it owns, the driver writing them tiles first,
every rank's checkpoint written while the statements go out, and Spark's replay of a batch whose writes failed.

The ranks' stages are the oracle restatement (tests/sharded_fake.OracleRunner over test_distributed_gloo.OracleStages)
and their statements come from the library's host-executed encoders, so the written statements must equal those of
the single-shard oracle run through the same encoders, byte for byte (dyadic inputs: every fp64 sum is exact).
tests/test_gpu_sharded_stream.py runs the same writer on the GPU through the HIP library.
"""
import numpy as np
import pandas as pd
import pytest

from mobheat import stream


class Capture:
    log = []
    fail = False

    def __init__(self):
        self.cur = {"tiles": [], "positions_latest": []}
        Capture.log.append(self.cur)

    def update_raw(self, collection, statements):
        if Capture.fail:
            raise IOError("mongo down")
        self.cur[collection].extend(bytes(s.raw) for s in statements)

    def close(self):
        pass


def _frames(n_batches=3, n=3000, seed=2, grid=1 << 8):
    """dyadic micro-batches: lat/lon on a `grid` x `grid` lattice of 1/1024-degree steps"""
    rng = np.random.default_rng(seed)
    out = []
    for b in range(n_batches):
        lat = 42.0 + rng.integers(0, grid, n) / 1024.0
        lon = -71.25 + rng.integers(0, grid, n) / 1024.0
        speed = pd.array(rng.integers(0, 160, n) * 0.5, dtype="Float64")
        speed[rng.random(n) < 0.1] = pd.NA
        ts = 1759572000 + b * 240 + rng.integers(0, 360, n)
        ts[: n // 30] = ts[n // 30: 2 * (n // 30)]
        veh = rng.integers(0, 300, n)
        out.append(pd.DataFrame({"provider": np.where(veh % 5 == 0, "mbta", "opensky"),
                                 "vehicleId": [f"v{v}" for v in veh], "lat": lat, "lon": lon, "speedKmh": speed,
                                 "eventTs": pd.to_datetime(ts, unit="s", utc=True)}))
    return out


def _expected(frames):
    """The single-shard oracle through the same host encoders: per batch, sorted tile and position statements."""
    from mobheat import _lib
    from oracle.spark_oracle import SparkHeatmapOracle
    from sharded_fake import statements_of_tiles
    ora = SparkHeatmapOracle(h3_res=stream.H3_RES, tile_us=stream.TILE_MIN * 60_000_000)
    cfg = dict(city=stream.CITY, h3_res=stream.H3_RES, ttl_min=stream.TTL_MIN, tile_minutes=stream.TILE_MIN)
    out = []
    for df in frames:
        c = stream.batch_columns(df)
        e = ora.process_batch(c["lat"], c["lon"], c["ts_us"], c["speed"], c["speed_valid"], c["vkey"], c["row_valid"])
        tb, to = statements_of_tiles({(t["cell"], t["window_start_us"]): (t["count"], t["avg_speed"], t["avg_lon"],
                                                                         t["avg_lat"]) for t in e["tiles"]}, cfg)
        r = e["latest_rows"]
        pb, po = _lib.position_statements_selftest(c["provider_uniques"], c["vehicle_uniques"], c["vkey"][r],
                                                   c["ts_us"][r], c["lat"][r], c["lon"][r])
        out.append({"tiles": sorted(bytes(tb[to[k]:to[k + 1]]) for k in range(to.size - 1)),
                    "positions_latest": sorted(bytes(pb[po[k]:po[k + 1]]) for k in range(po.size - 1))})
    return out


def test_sharded_writer_world2_gloo(tmp_path, monkeypatch, oracle_h3):
    from sharded_fake import OracleRunner
    frames = _frames()
    exp = _expected(frames)
    monkeypatch.setattr(stream, "SINK_FACTORY", Capture)
    monkeypatch.setattr(stream, "N_GPUS", 2)
    monkeypatch.setattr(stream, "DIST_BACKEND", "gloo")
    monkeypatch.setattr(stream, "STATE_CHECKPOINT", True)
    monkeypatch.setattr(stream, "SHARDED_EXTRA", {"cpu": True, "runner": "sharded_fake:OracleRunner"})
    stream.close_sharded()
    Capture.log.clear()
    OracleRunner.commits.clear()
    try:
        stream.foreach_batch_func(frames[0], 0)
        stream.foreach_batch_func(frames[1], 1)
        # the writes of batch 2 fail: the epoch is not committed; Spark re-runs it and the same statements are written
        # without a second merge (the oracle's state would double-count the batch)
        Capture.fail = True
        with pytest.raises(IOError):
            stream.foreach_batch_func(frames[2], 2)
        Capture.fail = False
        res = stream.foreach_batch_func(frames[2], 2)
    finally:
        Capture.fail = False
        stream.close_sharded()
    written = [c for c in Capture.log if c["tiles"] or c["positions_latest"]]
    assert len(written) == 3
    for e in range(3):
        for coll in ("tiles", "positions_latest"):
            assert sorted(written[e][coll]) == exp[e][coll], (e, coll)
    assert len(exp[2]["tiles"]) > 100 and res.n_tiles == len(exp[2]["tiles"])
    # (rank 0's checkpoints are recorded here; the worker's in its own process) one per epoch, written while the
    # statements go out -- epoch 2 twice: its first writes failed, and the replay checkpoints it again (the same state)
    assert OracleRunner.commits == [(0, 0), (0, 1), (0, 2), (0, 2)]


def test_sharded_writer_growing_batches(tmp_path, monkeypatch, oracle_h3):
    """Batches that outgrow the shared-memory regions (3k, then 40k rows, then 3k): the regions holding the ranks'
    statements grow while the previous batch's views of them are still referenced (a region closed under
    live views raised BufferError after every rank had merged), and every batch still writes the oracle's statements."""
    frames = [_frames(n_batches=1, n=n, seed=sd, grid=1 << 12)[0] for n, sd in ((3000, 3), (40000, 4), (3000, 5))]
    for b, f in enumerate(frames):   # (consecutive batches of one stream: 4 minutes apart)
        f["eventTs"] = f["eventTs"] + pd.Timedelta(minutes=4 * b)
    exp = _expected(frames)
    monkeypatch.setattr(stream, "SINK_FACTORY", Capture)
    monkeypatch.setattr(stream, "N_GPUS", 2)
    monkeypatch.setattr(stream, "DIST_BACKEND", "gloo")
    monkeypatch.setattr(stream, "STATE_CHECKPOINT", True)
    monkeypatch.setattr(stream, "SHARDED_EXTRA", {"cpu": True, "runner": "sharded_fake:OracleRunner"})
    stream.close_sharded()
    Capture.log.clear()
    try:
        for e, f in enumerate(frames):
            stream.foreach_batch_func(f, e)
            # the views the driver kept for a replay read back exactly the statements it wrote
            last = stream._SHARDED.last
            assert sorted(bytes(b[o[k]:o[k + 1]]) for _, (b, o), _ in last for k in range(o.size - 1)) == \
                sorted(Capture.log[-1]["tiles"])
    finally:
        stream.close_sharded()
    written = [c for c in Capture.log if c["tiles"] or c["positions_latest"]]
    assert len(written) == 3
    for e in range(3):
        for coll in ("tiles", "positions_latest"):
            assert sorted(written[e][coll]) == exp[e][coll], (e, coll)
    # (40k rows over a 4-degree box: ~10 MB of tile statements, past the 3k-row batch's regions and their 1 MiB slack)
    assert len(exp[1]["tiles"]) > 30000 and len(exp[1]["tiles"]) > 10 * len(exp[0]["tiles"])


def test_shm_arena_keeps_replaced_regions_mapped_until_released():
    """ShmArena: a region replaced by a larger one stays mapped (the last batch's views read it) until close_retired;
    its name is unlinked at once."""
    from multiprocessing import shared_memory
    from mobheat.sharded import ShmArena
    a = ShmArena()
    try:
        name, lay = a.put({"x": np.arange(1000, dtype=np.int64)})
        v = np.ndarray(lay[0][2], np.dtype(lay[0][1]), buffer=a.shm.buf, offset=lay[0][3])
        a.put({"x": np.zeros(1 << 20, np.int64)})   # grows: a new region
        assert a.shm.name != name and len(a._retired) == 1
        assert int(v.sum()) == 499500                # the old view still reads the old region
        with pytest.raises(FileNotFoundError):
            shared_memory.SharedMemory(name=name)
        del v
        a.close_retired()
        assert not a._retired
    finally:
        a.close()


def test_run_device_orders_ingest_after_column_exchange(monkeypatch):
    """the device-column path (RankRunner.run_device) must make the library's stream wait for the
    all_to_all that delivered the rank's columns before hm_stage_ingest reads them -- exchange, then the stream wait
    (ShardedHeatmap.after_collective), then the stages; and the columns handed to the stages are the received slice."""
    from mobheat import distributed, sharded
    import torch
    order = []
    recv = torch.zeros(sharded.packed_bytes(5), dtype=torch.uint8)

    def fake_exchange(buf, sb, device, status=0):
        order.append("exchange")
        return recv, [sharded.packed_bytes(5)]

    class Stop(Exception):
        pass

    class FakeSharded:
        def after_collective(self):
            order.append("wait")

        def process_batch(self, epoch, batch, out_memory=None):
            order.append(("stages", batch["n"], batch["lat"] >= recv.data_ptr()))
            raise Stop

    class FakeEng:
        def state_version(self):
            return 0

    monkeypatch.setattr(distributed, "exchange_chunks", fake_exchange)
    r = sharded.RankRunner.__new__(sharded.RankRunner)
    r.rank, r.world, r.engine, r.sharded, r.device = 0, 1, FakeEng(), FakeSharded(), torch.device("cpu")
    with pytest.raises(Stop):
        r.run_device(3, {}, np.array([0, 5]), None)
    assert order == ["exchange", "wait", ("stages", 5, True)]
