"""Multi-GPU hot path: one process per GPU, torch.distributed (backend "nccl" = RCCL over xGMI).

Replaces Spark's shuffle of the two aggregations (spark.sql.shuffle.partitions = 4, reference
heatmap_stream.py:44): every rank snaps and pre-aggregates its own shard of the micro-batch, then ONE
all-to-all per record kind routes

  * tile partials  (48-B records: cell, windowStart, count, n_speed, sum speed/lat/lon) to owner rank
    hash(cell, windowStart) % world, which merges them into the persistent state it owns and emits them;
  * latest-position candidates (32-B records: vkey, ts, row, origin rank) to owner hash(vkey) % world,
    which keeps the rows tied at the global max and routes the winning row indices back to their origin;

plus an all-reduce(max) of the batch's max event time (the watermark's input, :107).  Ownership is a pure
function of the key, so the persistent state never moves between batches.  The exchange buffers are torch
tensors handed to RCCL directly; the library writes/reads them through plain device pointers.
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import HM_CAND_REC_BYTES, HM_MEM_DEVICE, HM_MEM_HOST, HM_TILE_REC_BYTES, HmBatchIn, HmBatchOut, HmStageSizes, check


def exchange(send, send_counts, rec_bytes, device):
    """all_to_all of variable-size record runs; send_counts[r] records go to rank r. Returns (recv, counts),
    recv a uint8 tensor.  The payload moves as 8-byte words (records are 48, 32 or 8 bytes): a rank's share at
    1e8 events per GPU is several GB, past 2^31 single-byte elements."""
    world = dist.get_world_size()
    assert rec_bytes % 8 == 0
    w = rec_bytes // 8
    sc = torch.tensor(send_counts, dtype=torch.int64, device=device)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc)
    recv_counts = rc.cpu().tolist()
    nrecv = int(sum(recv_counts))
    recv = torch.empty(max(nrecv * w, 2), dtype=torch.int64, device=device)
    nsend = int(sum(send_counts))
    dist.all_to_all_single(recv[: nrecv * w], send[: nsend * rec_bytes].view(torch.int64),
                           [c * w for c in recv_counts], [c * w for c in send_counts])
    assert len(recv_counts) == world
    return recv.view(torch.uint8), recv_counts


class LibStages:
    """The library's stage API (hm_stage_local / hm_stage_merge / hm_stage_finish) on torch device buffers."""

    def __init__(self, engine):
        self.engine = engine
        self.lib = _lib.load()
        self.dev = torch.device("cuda", engine.device)
        self._tile_send = self._cand_send = self._winner_send = None

    def _buf(self, name, nbytes):
        b = getattr(self, name)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=self.dev)
            setattr(self, name, b)
        return b

    def local(self, epoch, batch, world, rank):
        n = int(batch["n"])
        tile_send = self._buf("_tile_send", n * HM_TILE_REC_BYTES)
        cand_send = self._buf("_cand_send", n * HM_CAND_REC_BYTES)
        tc = (ctypes.c_int64 * world)()
        cc = (ctypes.c_int64 * world)()
        sizes = HmStageSizes()
        b = HmBatchIn(n=n, memory=HM_MEM_DEVICE, lat=batch["lat"], lon=batch["lon"], ts_us=batch["ts_us"],
                      speed=batch.get("speed"), speed_valid=batch.get("speed_valid"), vkey=batch["vkey"],
                      row_valid=batch.get("row_valid"))
        ctx = self.engine._ctx
        check(self.lib.hm_stage_local(ctx, int(epoch), ctypes.byref(b), world, rank, tile_send.data_ptr(), n, tc,
                                      cand_send.data_ptr(), n, cc, ctypes.byref(sizes)), ctx, "hm_stage_local")
        return tile_send, list(tc), cand_send, list(cc), int(sizes.batch_max_event_ms)

    def merge(self, tile_recv, n_tile, cand_recv, n_cand, global_max_ms, out_memory):
        world = dist.get_world_size()
        winner_send = self._buf("_winner_send", max(n_cand, 1) * 8)
        wc = (ctypes.c_int64 * world)()
        out = HmBatchOut()
        ctx = self.engine._ctx
        check(self.lib.hm_stage_merge(ctx, tile_recv.data_ptr(), n_tile, cand_recv.data_ptr(), n_cand, global_max_ms,
                                      out_memory, ctypes.byref(out), winner_send.data_ptr(), max(n_cand, 1), wc),
              ctx, "hm_stage_merge")
        return out, winner_send, list(wc)

    def finish(self, winner_recv, n_winner, out_memory, out):
        ctx = self.engine._ctx
        check(self.lib.hm_stage_finish(ctx, winner_recv.data_ptr(), n_winner, out_memory, ctypes.byref(out)), ctx,
              "hm_stage_finish")
        return out


class ShardedHeatmap:
    """One rank of the sharded hot path. ``stages`` provides local / merge / finish (LibStages on GPUs)."""

    def __init__(self, stages, device):
        self.stages = stages
        self.device = device
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        # the last batch's receive buffers: with out_memory=HM_MEM_DEVICE, out.latest_row points into winner_recv
        # (hm_stage_finish), so they stay alive until the next process_batch call
        self._recv = None

    def process_batch(self, epoch, batch, out_memory=HM_MEM_DEVICE, sync=None):
        sync = sync or (lambda: torch.cuda.current_stream(self.device).synchronize()
                        if self.device.type == "cuda" else None)
        tile_send, tcounts, cand_send, ccounts, local_max = self.stages.local(epoch, batch, self.world, self.rank)
        tile_recv, trc = exchange(tile_send, tcounts, HM_TILE_REC_BYTES, self.device)
        cand_recv, crc = exchange(cand_send, ccounts, HM_CAND_REC_BYTES, self.device)
        m = torch.tensor([local_max], dtype=torch.int64, device=self.device)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        global_max = int(m.item())
        sync()
        out, winner_send, wcounts = self.stages.merge(tile_recv, int(sum(trc)), cand_recv, int(sum(crc)), global_max,
                                                      out_memory)
        winner_recv, wrc = exchange(winner_send, wcounts, 8, self.device)
        sync()
        self._recv = (tile_recv, cand_recv, winner_recv)
        return self.stages.finish(winner_recv, int(sum(wrc)), out_memory, out)


def tile_hash(cell, wstart):
    """Python twin of kernels.h tile_hash (the key_hash field of a tile partial record)."""
    with np.errstate(over="ignore"):
        return _mix64(np.asarray(cell, np.uint64) ^ _mix64(np.asarray(wstart).astype(np.uint64) +
                                                           np.uint64(0x9E3779B97F4A7C15)))


def tile_owner(cell, wstart, world):
    """Python twin of the device routing (kernels.h owner_of(tile_hash(...)))."""
    return _owner(tile_hash(cell, wstart), world)


def vkey_owner(vkey, world):
    return _owner(_mix64(np.asarray(vkey, np.uint64) ^ np.uint64(0x2545F4914F6CDD1D)), world)


def _mix64(x):
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(33))
        x = x * np.uint64(0xFF51AFD7ED558CCD)
        x = x ^ (x >> np.uint64(33))
        x = x * np.uint64(0xC4CEB9FE1A85EC53)
        x = x ^ (x >> np.uint64(33))
    return x


def _owner(h, world):
    with np.errstate(over="ignore"):
        return (((h >> np.uint64(32)) * np.uint64(world)) >> np.uint64(32)).astype(np.int64)
