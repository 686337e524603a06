"""Test helper (not a test module): a rank of the sharded writer (mobheat.sharded) whose stages are the oracle
restatement (test_distributed_gloo.OracleStages, the library's wire formats) and whose statements come from the
library's host-executed encoders -- so that the CPU suite runs the writer's whole protocol (spawned workers, gloo,
shared-memory hand-offs, statement flush, commit) without a GPU.  Spawned workers import it by name."""
import numpy as np
import torch

from mobheat import _lib
from mobheat.engine import TileRows
from mobheat.sharded import COLS, RankRunner


class _Eng:
    def close(self):
        pass


class OracleRunner(RankRunner):
    commits = []

    def _start(self, restore):
        from mobheat.distributed import ShardedHeatmap
        from test_distributed_gloo import OracleStages
        self.engine = _Eng()
        self.sharded = ShardedHeatmap(OracleStages(self.cfg["h3_res"]), torch.device("cpu"))
        self.lineage = "cpu"

    def run(self, epoch, views, lo, hi, restore):
        if self.engine is None:
            self._start(restore)
        self.began = True
        n = hi - lo
        b = {k: np.array(views[k][lo:hi]) for k in COLS}
        b["speed_valid"], b["row_valid"], b["n"] = b["speed_valid"].astype(bool), b["row_valid"].astype(bool), n
        out = self.sharded.process_batch(epoch, b, sync=lambda: None)
        c = self.cfg
        tb, to = statements_of_tiles(out["tiles"], c)
        tiles = self.out_t.put({"b": tb, "o": to})
        rows = np.asarray(out["latest"], np.int64) + lo
        pos = None
        if rows.size:
            prov = (int(views["prov_n"][0]), views["prov_offs"], views["prov_bytes"])
            veh = (int(views["veh_n"][0]), views["veh_offs"], views["veh_bytes"])
            pb, po = _lib.position_statements_selftest(prov, veh, views["vkey"][rows], views["ts_us"][rows],
                                                       views["lat"][rows], views["lon"][rows])
            pos = self.out_p.put({"b": pb, "o": po})
        o = self.sharded.stages.o
        stats = dict(n_in=n, n_valid=0, n_late=0, n_state=len(o.state), n_tiles=len(out["tiles"]), n_latest=int(rows.size),
                     watermark_ms=int(o.wm_cur), batch_max_event_ms=0, late_watermark_ms=0, n_partials=0)
        return stats, tiles, pos

    def commit_prepare(self, epoch):
        OracleRunner.commits.append((self.rank, int(epoch)))
        return None


def statements_of_tiles(tiles, cfg):
    """{(cell, ws): (count, avg_speed | None, avg_lon, avg_lat)} -> the library's host-encoded tile statements."""
    keys = sorted(tiles)
    n = len(keys)
    t = [tiles[k] for k in keys]
    tile_us = cfg["tile_minutes"] * 60_000_000
    ws = np.array([k[1] for k in keys], np.int64)
    rows = TileRows(cell=np.array([k[0] for k in keys], np.uint64), window_start_us=ws, window_end_us=ws + tile_us,
                    count=np.array([x[0] for x in t], np.int64),
                    avg_speed=np.array([0.0 if x[1] is None else x[1] for x in t], np.float64),
                    speed_null=np.array([x[1] is None for x in t], bool), avg_lon=np.array([x[2] for x in t], np.float64),
                    avg_lat=np.array([x[3] for x in t], np.float64))
    if n == 0:
        return np.zeros(0, np.uint8), np.zeros(1, np.int64)
    return _lib.tile_statements_selftest(rows, cfg["city"], cfg["h3_res"], cfg["ttl_min"], tile_us)
