"""The multi-GPU hot path behind the reference's boundary: foreach_batch_func(df, epoch_id) with MOBHEAT_GPUS=N.

The reference hands each micro-batch to ``foreach_batch_func`` on the Spark driver, once per epoch, sequentially
(heatmap_stream.py:150,245), and writes the tiles and positions_latest documents from there (:159-235).  With N GPUs
the driver process runs rank 0 and N-1 persistent worker processes run ranks 1..N-1, one GPU each, joined by
torch.distributed (backend "nccl" = RCCL over xGMI; MOBHEAT_DIST_BACKEND=gloo rehearses several ranks on one GPU).
Workers are started with a fresh spawn (never an exec of a process that touched the GPU).  Per micro-batch:

  1. the driver extracts the batch's columns (stream.batch_columns; raw Kafka values are decoded on rank 0's GPU) and
     its string dictionaries into one POSIX shared-memory region, and tells every rank its contiguous share;
  2. every rank runs the sharded stages (distributed.ShardedHeatmap over the library's stage API, its share copied
     to its GPU by the library): snap, windows and latest-position maxima locally, the owner-keyed all-to-all, the
     owner merge into the state it owns;
  3. every rank encodes, on its GPU, the update statements of what it owns -- the tiles of its keys
     (hm_encode_tile_updates) and the positions of the latest rows it holds (hm_encode_position_updates) -- so no
     statement crosses the exchange; workers hand theirs back through shared memory;
  4. the driver writes them through the sink, tiles first, as the reference does (one connection per batch, unordered
     bulks of 1000);
  5. every rank checkpoints its own state (mobheat.checkpoint: per-rank chains; a restore into another GPU count
     re-partitions the keys by owner) while the driver writes the statements -- before the writes are known to have
     succeeded, which is safe: a restart re-runs the first uncommitted epoch E on the newest chain ending BEFORE E, and a
     replay of E in this process rewrites E's files.

A failure on any rank fails the batch (every rank leaves at the same collective, distributed.PeerFailed); a failure
after a merge began resets every rank's state, which the replayed epoch restores from the checkpoints.
"""
import atexit
import datetime
import os
import socket
import sys
import time
import traceback

import numpy as np

from . import _lib
from ._lib import HM_MEM_DEVICE, HM_MEM_HOST

COLS = ("lat", "lon", "ts_us", "speed", "speed_valid", "vkey", "row_valid")
# MOBHEAT_SHARDED_TRACE=1: every rank's protocol steps to stderr (a hung rank names its step)
_TRACE = os.environ.get("MOBHEAT_SHARDED_TRACE") == "1"
# seconds a rank waits for its peers at a rendezvous or a reply before the batch fails (a dead rank must not hang the
# stream: a worker that died shows up as a timeout here)
TIMEOUT_S = float(os.environ.get("MOBHEAT_SHARDED_TIMEOUT", "600"))


def _trace(rank, msg):
    if _TRACE:
        print(f"[mobheat r{rank} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)
_DT = {"lat": np.float64, "lon": np.float64, "ts_us": np.int64, "speed": np.float64, "speed_valid": np.uint8,
       "vkey": np.uint64, "row_valid": np.uint8}


# ------------------ shared memory ------------------
class ShmArena:
    """A growable POSIX shared-memory region holding named arrays (64-B aligned); put() returns the manifest a reader
    maps them with (shm_views).  A region replaced by a larger one is unlinked at once but stays mapped until
    close_retired(): numpy views of it (the last batch's statements, ShardedStream.last) do not pin the mapping, so
    closing it under them would leave them pointing at unmapped memory."""

    def __init__(self):
        self.shm = None
        self._retired = []   # replaced regions, unlinked, still mapped

    def put(self, arrays):
        layout, off = [], 0
        arrays = {k: np.ascontiguousarray(v) for k, v in arrays.items()}
        for name, a in arrays.items():
            layout.append((name, a.dtype.str, a.shape, off))
            off += (a.nbytes + 63) & ~63
        self._ensure(max(off, 64))
        for (name, dt, shp, o) in layout:
            a = arrays[name]
            if a.nbytes:
                np.ndarray(a.shape, a.dtype, buffer=self.shm.buf, offset=o)[...] = a
        return self.shm.name, layout

    def _ensure(self, nbytes):
        from multiprocessing import shared_memory
        if self.shm is not None and self.shm.size >= nbytes:
            return
        old = self.shm
        self.shm = shared_memory.SharedMemory(create=True, size=int(nbytes + nbytes // 4 + (1 << 20)))
        if old is not None:
            _unlink(old)
            self._retired.append(old)

    def close_retired(self):
        """Unmap the replaced regions (the caller holds no view of them any more: a new batch began)."""
        for r in self._retired:
            _close(r)
        self._retired = []

    def close(self):
        self.close_retired()
        if self.shm is not None:
            _unlink(self.shm)
            _close(self.shm)
            self.shm = None


def _unlink(shm):
    try:
        shm.unlink()
    except FileNotFoundError:
        pass


def _close(shm):
    try:
        shm.close()
    except BufferError:   # (a buffer export still alive: the mapping goes with the object)
        pass


_ATTACHED = {}
_DETACHED = []   # attachments to regions their writer replaced: still mapped until close_detached()


def shm_views(name, layout, slot="in"):
    """{name: array view} of a manifest in another process's region (attachments are cached).  (The spawned ranks share
    the driver's resource tracker, whose registry is a set: attaching adds nothing, and the region's creator
    unregisters it when it unlinks it.)"""
    from multiprocessing import shared_memory
    cur = _ATTACHED.get(slot)   # (slot: the writer -- its previous region is gone once it grew into a new one)
    if cur is None or cur.name != name:
        if cur is not None:   # (views of it may still be alive: unmapped by close_detached at the next batch)
            _DETACHED.append(cur)
        cur = _ATTACHED[slot] = shared_memory.SharedMemory(name=name)
    shm = cur
    return {n: np.ndarray(shp, np.dtype(dt), buffer=shm.buf, offset=o) for n, dt, shp, o in layout}


def close_detached():
    """Unmap the attachments to replaced regions (no view of them is left: a new batch began)."""
    global _DETACHED
    for r in _DETACHED:
        _close(r)
    _DETACHED = []


def dictionary_arrays(uniques):
    """A batch's string dictionary as (n, offsets, bytes) arrays (Arrow layout), whatever form it came in."""
    if isinstance(uniques, tuple):
        return uniques
    return _lib._dictionary(uniques)


# ------------------ one rank ------------------
class RankRunner:
    """One rank of the sharded writer: its engine (restored from the checkpoints when it starts), the stage pipeline,
    the statements of what it owns, its checkpoint chain."""

    def __init__(self, rank, world, device, cfg):
        import torch
        from .checkpoint import StateCheckpoints
        self.rank, self.world, self.cfg = rank, world, cfg
        self.device_index = device
        self.device = torch.device("cuda", device) if device is not None else torch.device("cpu")
        self.began = False
        self.engine = None
        self.sharded = None
        self.lineage = None
        self.store = StateCheckpoints(os.path.join(cfg["checkpoint_dir"], "mobheat-state"), rank, world)
        # the rank's statements, copied out of the engine's pinned buffers (each encode reuses them) into shared
        # memory the driver reads: tiles, positions
        self.out_t, self.out_p = ShmArena(), ShmArena()

    def reset(self):
        if self.engine is not None:
            self.engine.close()
        self.engine = self.sharded = None

    def _start(self, restore):
        from .distributed import LibStages, ShardedHeatmap, tile_owner
        from .engine import HeatmapEngine
        c = self.cfg
        eng = HeatmapEngine(h3_res=c["h3_res"], tile_minutes=c["tile_minutes"], watermark_delay_ms=c["delay_ms"],
                            device=self.device_index, shard=(self.rank, self.world))
        kind, val = restore
        if kind == "point":
            info, recs = self.store.load(val, owner=lambda cl, ws: tile_owner(cl, ws, self.world) == self.rank)
            eng.import_state(info, recs)
            self.lineage = val.lineage
        else:
            self.lineage = val
        self.engine = eng
        self.sharded = ShardedHeatmap(LibStages(eng), self.device)

    def run(self, epoch, views, lo, hi, restore):
        """Rank's share [lo, hi) of the batch in `views` (host arrays, the whole batch): the sharded stages, then the
        statements of the tiles it owns and of the latest rows it holds.  Returns (stats, tiles, positions), the
        statements as the manifests of the rank's shared-memory regions (positions None when it holds no latest row)."""
        if self.engine is None:
            self._start(restore)
        if self.rank:   # (a worker holds no view of its own replaced regions; rank 0's are dropped by the driver)
            self.out_t.close_retired()
            self.out_p.close_retired()
        eng = self.engine
        self.began = False
        v0 = eng.state_version()
        try:
            return self._run(eng, epoch, views, lo, hi)
        finally:
            self.began = eng.state_version() != v0

    def _run(self, eng, epoch, views, lo, hi):
        n = hi - lo
        batch = {"n": n, "memory": HM_MEM_HOST}
        for k in COLS:
            a = views[k]
            batch[k] = a.ctypes.data + lo * a.itemsize if a.size else None
        _trace(self.rank, f"batch {epoch}: {n} rows")
        out = self.sharded.process_batch(epoch, batch, out_memory=HM_MEM_DEVICE)
        return self._statements(eng, out, views)

    def run_device(self, epoch, views, bounds, restore, send=None):
        """The device-column form of run: the batch's columns were built on rank 0's GPU (hm_arrow_columns /
        hm_decode_json) and packed per rank (pack_columns); every rank takes its slice in the exchange's all_to_all
        (rank 0 sends, every rank receives -- device to device, no host copy of the columns) and runs the stages on it.
        views: the batch-wide string dictionaries (shared memory); send: rank 0's (buffer, bytes per rank)."""
        if self.engine is None:
            self._start(restore)
        if self.rank:
            self.out_t.close_retired()
            self.out_p.close_retired()
        eng = self.engine
        self.began = False
        v0 = eng.state_version()
        try:
            from .distributed import exchange_chunks
            buf, sb = send if send is not None else (None, [0] * self.world)
            recv, rb = exchange_chunks(buf, sb, self.device)
            # hm_stage_ingest reads the columns on the library's stream: it waits for the all_to_all that wrote them
            # (queued on torch's current stream) -- ADVICE r5: without this wait, ranks could ingest columns that had
            # only partly arrived
            self.sharded.after_collective()
            n = int(bounds[self.rank + 1] - bounds[self.rank])
            assert sum(rb) == packed_bytes(n), (sum(rb), n)
            self._cols = recv   # (alive until the next batch: the library reads it)
            batch = packed_batch(recv.data_ptr(), n)
            _trace(self.rank, f"batch {epoch}: {n} rows (device columns)")
            out = self.sharded.process_batch(epoch, batch, out_memory=HM_MEM_DEVICE)
            return self._statements(eng, out, views)
        finally:
            self.began = eng.state_version() != v0

    def _statements(self, eng, out, views):
        epoch_trace = f"{int(out.n_tiles)} tiles, {int(out.n_latest)} latest rows"
        _trace(self.rank, f"merged, {epoch_trace}")
        c = self.cfg
        tb, to = eng.encode_tile_updates(c["city"], c["ttl_min"])   # (views: copied before the next encode)
        tiles = self.out_t.put({"b": tb, "o": to})
        positions = None
        if out.n_latest:
            prov = (int(views["prov_n"][0]), views["prov_offs"], views["prov_bytes"])
            veh = (int(views["veh_n"][0]), views["veh_offs"], views["veh_bytes"])
            pb, po = eng.encode_position_updates(prov, veh)
            positions = self.out_p.put({"b": pb, "o": po})
        stats = dict(n_in=int(out.n_in), n_valid=int(out.n_valid), n_late=int(out.n_late), n_state=int(out.n_state),
                     n_tiles=int(out.n_tiles), n_latest=int(out.n_latest), watermark_ms=int(out.watermark_ms),
                     batch_max_event_ms=int(out.batch_max_event_ms), late_watermark_ms=int(out.late_watermark_ms),
                     n_partials=int(out.n_partials), counts=eng.last_counts())
        return stats, tiles, positions

    def commit(self, epoch):
        job = self.commit_prepare(epoch)
        if job is not None:
            self.commit_write(job)

    def commit_prepare(self, epoch):
        """The GPU half of the rank's checkpoint of `epoch` (mobheat.checkpoint prepare), or None when off."""
        if not (self.cfg["checkpoint"] and self.engine is not None):
            return None
        _trace(self.rank, f"checkpoint {epoch}")
        return self.store.prepare(epoch, self.engine, self.lineage, self.cfg["full_every"])

    def commit_write(self, job):
        kind = self.store.write(job)
        _trace(self.rank, f"checkpoint {job['epoch']}: {kind} written")
        return kind



# the device-column exchange: a rank's slice of n rows as one buffer -- lat, lon, ts_us, speed, vkey (8 B each), then
# speed_valid and row_valid (1 B each, each padded to 8 B)
_PACK = (("lat", 8), ("lon", 8), ("ts_us", 8), ("speed", 8), ("vkey", 8), ("speed_valid", 1), ("row_valid", 1))


def _pad8(b):
    return (b + 7) & ~7


def packed_bytes(n):
    return sum(_pad8(n * el) for _, el in _PACK)


def packed_batch(addr, n):
    """the stage API's batch over a packed slice at device address `addr`"""
    b, off = {"n": n, "memory": HM_MEM_DEVICE}, 0
    for k, el in _PACK:
        b[k] = addr + off if n else None
        off += _pad8(n * el)
    return b


def pack_columns(batch, bounds, device):
    """rank 0: the device columns of the whole batch (an HmBatchIn, device memory) packed per rank (rank r: rows
    [bounds[r], bounds[r+1])) into one device buffer by device-to-device copies -> (buffer, bytes per rank)"""
    import torch
    lib = _lib.load()
    world = len(bounds) - 1
    sizes = [packed_bytes(int(bounds[r + 1] - bounds[r])) for r in range(world)]
    buf = torch.empty(max(sum(sizes), 8), dtype=torch.uint8, device=device)
    base = buf.data_ptr()
    for r in range(world):
        lo, n = int(bounds[r]), int(bounds[r + 1] - bounds[r])
        for k, el in _PACK:
            src = getattr(batch, k)
            if n and src:
                _lib.check(lib.hm_memcpy(base, src + lo * el, n * el, 2), None, "hm_memcpy")
            base += _pad8(n * el)
    torch.cuda.synchronize(device)
    return buf, sizes


def _runner_class(cfg):
    """RankRunner, or the class cfg["runner"] names ("module:Class": the CPU tests' oracle-backed rank)."""
    name = cfg.get("runner")
    if not name:
        return RankRunner
    import importlib
    mod, cls = name.split(":")
    return getattr(importlib.import_module(mod), cls)


def _init_group(rank, world, port, backend, device):
    import torch
    import torch.distributed as dist
    if device is not None:
        torch.cuda.set_device(device)
    kw = {"device_id": torch.device("cuda", device)} if backend == "nccl" else {}
    _trace(rank, f"init_process_group {backend} port {port} device {device}")
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=TIMEOUT_S), **kw)
    _trace(rank, "process group up")


def _worker_main(rank, world, port, conn, cfg):
    """A worker rank's loop: ("batch", ...) -> ("ok", stats, out manifest) | ("err", repr, traceback);
    ("commit", epoch), ("reset",), ("close",)."""
    import torch.distributed as dist
    device = cfg["devices"][rank]
    if _TRACE:   # (a hung worker prints where it is)
        import faulthandler
        faulthandler.dump_traceback_later(100, repeat=True)
    try:
        _init_group(rank, world, port, cfg["backend"], device)
        runner = _runner_class(cfg)(rank, world, device, cfg)
    except Exception as e:   # (the driver's init_process_group times out; report why)
        conn.send(("err", repr(e), traceback.format_exc()))
        return
    conn.send(("ready",))
    while True:
        msg = conn.recv()
        op = msg[0]
        _trace(rank, f"op {op}")
        try:
            if op == "batch":
                _, epoch, name, layout, lo, hi, restore = msg
                stats, tiles, positions = runner.run(epoch, shm_views(name, layout), lo, hi, restore)
                conn.send(("ok", stats, tiles, positions))
            elif op == "batch_dev":
                _, epoch, name, layout, bounds, restore = msg
                stats, tiles, positions = runner.run_device(epoch, shm_views(name, layout), bounds, restore)
                conn.send(("ok", stats, tiles, positions))
            elif op == "commit":
                runner.commit(msg[1])
                conn.send(("ok",))
            elif op == "reset":
                runner.reset()
                conn.send(("ok",))
            elif op == "close":
                break
        except Exception as e:
            conn.send(("err", repr(e), traceback.format_exc(), type(e).__name__, getattr(runner, "began", False)))
    runner.reset()
    runner.out_t.close()
    runner.out_p.close()
    _trace(rank, "closing")
    conn.send(("closed",))
    try:
        dist.destroy_process_group()
    except Exception:
        pass
    _trace(rank, "closed")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class ShardedStream:
    """The driver's side: rank 0 in this process, ranks 1..world-1 in spawned workers."""

    def __init__(self, world, cfg):
        import torch
        import torch.distributed as dist
        import torch.multiprocessing as mp
        if dist.is_available() and dist.is_initialized():
            raise RuntimeError("MOBHEAT_GPUS > 1 starts its own process group: this process already has one")
        self.world = int(world)
        ndev = max(torch.cuda.device_count(), 1)
        cfg = dict(cfg)
        if cfg.get("cpu"):   # (the CPU tests: ranks without a GPU, gloo on host tensors)
            cfg["devices"] = [None] * self.world
        else:
            cfg["devices"] = [int(d) for d in cfg.get("devices") or [r % ndev for r in range(self.world)]]
        self.cfg = cfg
        port = _free_port()
        ctx = mp.get_context("spawn")
        self.conns, self.procs = [], []
        for r in range(1, self.world):
            parent, child = ctx.Pipe()
            p = ctx.Process(target=_worker_main, args=(r, self.world, port, child, cfg), daemon=True)
            p.start()
            self.conns.append(parent)
            self.procs.append(p)
        _init_group(0, self.world, port, cfg["backend"], cfg["devices"][0])
        for r, c in enumerate(self.conns, start=1):
            m = self._recv(c, r)
            if m[0] != "ready":
                raise RuntimeError(f"mobheat worker failed to start: {m[1]}\n{m[2]}")
        self.runner = _runner_class(cfg)(0, self.world, cfg["devices"][0], cfg)
        self.inputs = ShmArena()
        self.restore = None   # the restore point the ranks start from (set when they (re)start)
        self.last = None      # the last batch's per-rank statements (views) and stats
        self.closed = False
        atexit.register(self.close)

    # ---- one micro-batch ----
    def _restore_point(self, epoch):
        from .checkpoint import new_lineage
        pt = self.runner.store.restore_point(int(epoch)) if self.cfg["checkpoint"] and epoch is not None else None
        return ("point", pt) if pt is not None else ("fresh", new_lineage())

    def rank0_engine(self, epoch):
        """Rank 0's engine, started (restored) now if it is not yet (the Kafka decode runs on it before the batch)."""
        if self.restore is None:
            self.restore = self._restore_point(epoch)
        if self.runner.engine is None:
            self.runner._start(self.restore)
        return self.runner.engine

    def process(self, epoch, cols, dicts):
        """Run one micro-batch on every rank; returns the per-rank stats.  Raises (every rank's state reset when a merge
        may have begun) if any rank failed."""
        from .distributed import PeerFailed
        # the last batch's statement views are dropped: the regions replaced since can be unmapped now
        self.last = None
        self.inputs.close_retired()
        self.runner.out_t.close_retired()
        self.runner.out_p.close_retired()
        close_detached()
        n = int(cols["n"])
        arrays = {k: np.ascontiguousarray(cols[k] if cols.get(k) is not None else np.zeros(n), dtype=_DT[k]) for k in COLS}
        if cols.get("speed") is None:   # (no speed column: all null)
            arrays["speed_valid"] = np.zeros(n, np.uint8)
        pn, po, pb = dictionary_arrays(dicts[0])
        vn, vo, vb = dictionary_arrays(dicts[1])
        arrays.update(prov_n=np.array([pn], np.int64), prov_offs=po, prov_bytes=pb, veh_n=np.array([vn], np.int64),
                      veh_offs=vo, veh_bytes=vb)
        name, layout = self.inputs.put(arrays)
        views = {k: np.ndarray(shp, np.dtype(d), buffer=self.inputs.shm.buf, offset=o) for k, d, shp, o in layout}
        bounds = [r * n // self.world for r in range(self.world + 1)]
        if self.restore is None:   # (the ranks (re)start from the newest checkpoint before this epoch)
            self.restore = self._restore_point(epoch)
        for r, c in enumerate(self.conns, start=1):
            c.send(("batch", int(epoch), name, layout, bounds[r], bounds[r + 1], self.restore))
        err0 = res0 = None
        try:
            res0 = self.runner.run(int(epoch), views, bounds[0], bounds[1], self.restore)
        except Exception as e:
            err0 = e
        return self._collect(err0, res0, PeerFailed)

    def process_device(self, epoch, batch, dicts):
        """process() on device columns: `batch` (an HmBatchIn in rank 0's device memory: its engine's
        hm_arrow_columns / hm_decode_json) is packed per rank on rank 0's GPU and each rank takes its slice in one
        all_to_all -- no host copy of the columns; the string dictionaries (small) go through shared memory."""
        from .distributed import PeerFailed
        self.last = None
        self.inputs.close_retired()
        self.runner.out_t.close_retired()
        self.runner.out_p.close_retired()
        close_detached()
        n = int(batch.n)
        pn, po, pb = dictionary_arrays(dicts[0])
        vn, vo, vb = dictionary_arrays(dicts[1])
        name, layout = self.inputs.put(dict(prov_n=np.array([pn], np.int64), prov_offs=po, prov_bytes=pb,
                                            veh_n=np.array([vn], np.int64), veh_offs=vo, veh_bytes=vb))
        views = {k: np.ndarray(shp, np.dtype(d), buffer=self.inputs.shm.buf, offset=o) for k, d, shp, o in layout}
        bounds = [r * n // self.world for r in range(self.world + 1)]
        if self.restore is None:
            self.restore = self._restore_point(epoch)
        send = pack_columns(batch, bounds, self.runner.device)
        for c in self.conns:
            c.send(("batch_dev", int(epoch), name, layout, bounds, self.restore))
        err0 = res0 = None
        try:
            res0 = self.runner.run_device(int(epoch), views, bounds, self.restore, send=send)
        except Exception as e:
            err0 = e
        del send
        return self._collect(err0, res0, PeerFailed)

    def _collect(self, err0, res0, PeerFailed):
        replies = [self._recv(c, r) for r, c in enumerate(self.conns, start=1)]
        errs = [(0, err0)] if err0 is not None else []
        began = err0 is not None and getattr(self.runner, "began", False)
        for r, m in enumerate(replies, start=1):
            if m[0] != "ok":
                errs.append((r, RuntimeError(f"rank {r}: {m[1]}\n{m[2]}")))
                began = began or bool(m[4])
        if errs:
            if began:
                self.reset()
            first = next((e for _, e in errs if not isinstance(e, PeerFailed) and "PeerFailed" not in str(e)), errs[0][1])
            raise first
        try:
            per_rank = []
            for r, (stats, tiles, pos) in enumerate([res0] + [m[1:4] for m in replies]):
                per_rank.append((stats, self._views(r, tiles, "t"), self._views(r, pos, "p")))
        except BaseException:
            # every rank merged the batch but its statements cannot be handed over: drop every rank's state, so that
            # Spark's re-run of the epoch restores the state before it from the checkpoints instead of merging twice
            self.reset()
            raise
        self.last = per_rank
        return per_rank

    def _views(self, r, manifest, kind):
        if manifest is None:
            return None
        if r == 0:
            arena = self.runner.out_t if kind == "t" else self.runner.out_p
            v = {k: np.ndarray(shp, np.dtype(d), buffer=arena.shm.buf, offset=o) for k, d, shp, o in manifest[1]}
        else:
            v = shm_views(*manifest, slot=f"{kind}{r}")
        return v["b"], v["o"]

    def commit(self, epoch):
        """Checkpoint every rank's state after the epoch (commit_begin + commit_end)."""
        self.commit_begin(epoch)
        self.commit_end()

    def commit_begin(self, epoch):
        """Every rank checkpoints its state after the epoch: the workers in their processes, rank 0's file on a
        background thread -- concurrently with the driver's writes of the statements (stream._foreach_sharded)."""
        _trace(0, f"commit {epoch}")
        for c in self.conns:
            c.send(("commit", int(epoch)))
        self._commit = (None, None)
        try:
            job = self.runner.commit_prepare(epoch)
            if job is not None:
                from concurrent.futures import ThreadPoolExecutor
                if getattr(self, "_io", None) is None:
                    self._io = ThreadPoolExecutor(1, thread_name_prefix="mobheat-checkpoint")
                self._commit = (self._io.submit(self.runner.commit_write, job), None)
        except Exception as e:
            self._commit = (None, e)

    def commit_end(self):
        """Wait for every rank's checkpoint; then the files of an older world size are dropped once every rank of this
        one holds a snapshot."""
        fut, err = self._commit
        if fut is not None:
            e = fut.exception()
            err = err or e
        for r, c in enumerate(self.conns, start=1):
            m = self._recv(c, r)
            if m[0] != "ok" and err is None:
                err = RuntimeError(f"rank {r} checkpoint: {m[1]}")
        if err is not None:
            raise err
        if self.cfg["checkpoint"] and self.runner.lineage is not None:
            self.runner.store.prune_other_worlds(self.runner.lineage)

    def _recv(self, c, r):
        """A worker's reply, or RuntimeError when it died or did not answer within TIMEOUT_S."""
        p = self.procs[r - 1]
        t0 = time.monotonic()
        while not c.poll(1.0):
            if not p.is_alive():
                raise RuntimeError(f"mobheat worker rank {r} died (exit code {p.exitcode})")
            if time.monotonic() - t0 > TIMEOUT_S:
                raise RuntimeError(f"mobheat worker rank {r} did not answer within {TIMEOUT_S:.0f} s")
        return c.recv()

    def reset(self):
        """Drop every rank's state (the next batch restores from the checkpoints)."""
        for c in self.conns:
            c.send(("reset",))
        self.runner.reset()
        for r, c in enumerate(self.conns, start=1):
            self._recv(c, r)
        self.last = None
        self.restore = None

    def close(self):
        if self.closed:
            return
        self.closed = True
        _trace(0, "close")
        import torch.distributed as dist
        for c in self.conns:
            try:
                c.send(("close",))
            except Exception:
                pass
        self.runner.reset()
        for c, p in zip(self.conns, self.procs):
            try:
                if c.poll(60):
                    c.recv()
            except Exception:
                pass
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        _trace(0, "workers joined")
        try:
            dist.destroy_process_group()
        except Exception:
            pass
        self.inputs.close()
        self.runner.out_t.close()
        self.runner.out_p.close()
        _trace(0, "closed")
