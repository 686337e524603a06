"""Multi-GPU hot path: one process per GPU, torch.distributed (backend "nccl" = RCCL over xGMI).

Replaces Spark's shuffle of the two aggregations (spark.sql.shuffle.partitions = 4, reference
heatmap_stream.py:44).  Per micro-batch every rank snaps its own shard of the events (hm_stage_ingest: large shards
bin their records by region field inside k_ingest), then

  1. all_gather of the ranks' summaries (counts, max event time, window registry: ~64 KB per rank), from which
     every rank derives the same batch-wide decisions -- the watermark's input (:107), the aggregation path, the
     batch's global window registry;
  2. hm_stage_send writes ONE chunk per destination rank (include/mobheat.h): its tile records -- direct path, one 32-B
     record per aggregated row, grouped by region field with per-field counts and a per-window census; table mode,
     one 48-B partial per key -- and its latest-position candidates (32 B: vkey, ts, row, origin rank).  A tile key's
     owner holds a contiguous range of the key hash's region field (tile_owner), so the sender's bins are already
     grouped by destination and the owner merges each of its bins from the senders' segments;
  3. ONE all_to_all of the chunk sizes (with each rank's status), then ONE all_to_all of the chunks;
  4. hm_stage_merge on the owner, the winners' all_to_all back, hm_stage_finish.

Ownership is a pure function of the key, so the persistent state never moves between batches.  The exchange buffers
are torch tensors handed to RCCL directly; the library writes/reads them through plain device pointers.
"""
import ctypes
import os
from collections import namedtuple

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import HM_MEM_DEVICE, HM_STAGE_SUMMARY_WORDS, HmBatchIn, HmBatchOut, HmStageSizes, check

# one record stream of an exchange: buf (uint8 tensor), counts[r] records for rank r, rec_bytes per record
Stream = namedtuple("Stream", "name buf counts rec_bytes")

# summary word layout (csrc/api_stage.h SW_*); word 9 (SW_RESERVED in the library, which ignores it) carries the
# rank's status: nonzero when its stage failed, so that every rank leaves the batch at the same collective
SW_N_IN, SW_VALID, SW_LATE, SW_AGG, SW_MAX_MS, SW_SAMPLE_RUN, SW_PREV_AGG, SW_PREV_KEYS, SW_NWIN, SW_STATUS = range(10)
SW_WIN0 = 10
WREG_SLOTS = 4095
MAX_STREAMS = 1   # record streams of one exchange (exchange(): the winners)


class PeerFailed(RuntimeError):
    """Another rank's stage failed: this rank left the batch at the same collective (its own state is as a failed
    batch leaves it; the caller resets or replays)."""


# The batch's host metadata -- the summaries, the chunk sizes, the winner counts: host integers on every side -- moves
# over a gloo group of the same ranks when the payloads go over RCCL: a collective of host tensors
# needs no device round trip, where an RCCL one queued on torch's stream was followed by a .cpu() that waited for that
# stream (and for everything queued on it before) three times per batch.  MOBHEAT_META_BACKEND=same keeps them on the
# payloads' group; "gloo" forces a separate gloo group even under a gloo default (tests).
META_BACKEND = os.environ.get("MOBHEAT_META_BACKEND", "auto")
_META = {}


def meta_group():
    """(group, device) for the host metadata: a gloo group and the CPU when the default group is RCCL (or
    META_BACKEND is "gloo"), else (None, None) -- the default group on the caller's device.  Created at the first
    batch: every rank reaches it in the same order (ShardedHeatmap.process_batch, or the device-column scatter)."""
    want = META_BACKEND == "gloo" or (META_BACKEND == "auto" and dist.get_backend() != "gloo")
    if not want:
        return None, None
    if _META.get("world") is not dist.group.WORLD:   # (a new default group: a new metadata group with it)
        _META.update(world=dist.group.WORLD, group=dist.new_group(backend="gloo"))
    return _META["group"], torch.device("cpu")


def _meta_all_gather(t):
    """all_gather of a small int64 host-metadata tensor -> [world, ...] numpy (over meta_group when there is one)"""
    g, d = meta_group()
    x = t if g is None else t.to(d)
    out = [torch.empty_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(out, x, group=g)
    return torch.stack(out).cpu().numpy()


def all_gather_summaries(summary, device, status=0):
    """all_gather of every rank's int64[HM_STAGE_SUMMARY_WORDS] summary -> host array [world, words]; `status` != 0
    (this rank's ingest failed) makes every rank raise PeerFailed after the collective."""
    summary = np.array(summary, dtype=np.int64)
    summary[SW_STATUS] = status
    g, _ = meta_group()
    S = _meta_all_gather(torch.from_numpy(summary) if g is not None else torch.from_numpy(summary).to(device))
    if status == 0 and (S[:, SW_STATUS] != 0).any():
        raise PeerFailed(f"rank(s) {np.nonzero(S[:, SW_STATUS])[0].tolist()} failed the batch's ingest")
    return S


def exchange(streams, device, status=0):
    """all_to_all of several variable-size record streams: one all_to_all of all the per-destination counts (the
    batch's single host synchronization of the exchange; it also carries each rank's status: a rank whose stage failed
    sends status != 0 and no streams, and every rank raises PeerFailed before the payloads move -- and each rank's
    largest piece, so that every rank runs the same rounds), then each stream's payload (_exchange_words: rounds of at
    most round_bytes() per rank pair).  Payloads move as 8-byte words (record sizes are multiples of 8): a rank's share
    at 1e8 events per GPU is several GB, past 2^31 single-byte elements.  Returns [(recv uint8 tensor, recv_counts per
    source)] in stream order."""
    world = dist.get_world_size()
    k = len(streams)
    assert k <= MAX_STREAMS
    big = [max([int(c) * (s.rec_bytes // 8) for c in s.counts] + [0]) for s in streams] + [0] * (MAX_STREAMS - k)
    cnt = [[(streams[j].counts[r] if j < k else 0) for j in range(MAX_STREAMS)] + [status] + big for r in range(world)]
    g, md = meta_group()
    sc = torch.tensor(cnt, dtype=torch.int64, device=md if g is not None else device)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=g)
    rcounts = rc.cpu().tolist()
    bad = [r for r in range(world) if rcounts[r][MAX_STREAMS]]
    if bad and status == 0:
        raise PeerFailed(f"rank(s) {bad} failed the batch's stage before the exchange")
    if status:
        return []
    out = []
    for j, s in enumerate(streams):
        assert s.rec_bytes % 8 == 0 and len(s.counts) == world
        w = s.rec_bytes // 8
        recv_counts = [int(rcounts[r][j]) for r in range(world)]
        nrecv, nsend = sum(recv_counts), int(sum(s.counts))
        recv = torch.empty(max(nrecv * w, 2), dtype=torch.int64, device=device)
        biggest = max(int(rcounts[r][MAX_STREAMS + 1 + j]) for r in range(world))   # (every sender's largest piece)
        _exchange_words(recv, s.buf[: nsend * s.rec_bytes].view(torch.int64), [c * w for c in recv_counts],
                        [int(c) * w for c in s.counts], biggest)
        out.append((recv.view(torch.uint8), recv_counts))
    assert len(out) == k
    return out


# The largest piece of one (sender, receiver) pair that one all_to_all call moves -- a hard cap.  What was seen
# (round 5): the sharded bench's single all_to_all of a rank's ~3.2 GB of records (a world-1 RCCL group: the rank's
# whole share sent to itself in one call) was followed by hipErrorIllegalAddress, reported at hm_stage_merge's first
# error check after the collective (profiles/r5/r5e/fault_before_rounds.log; gpurun_out r5c2/r5d the same); the same
# exchange moved in rounds of <= 1 GiB per pair into the same receive buffer merged clean
# (profiles/r5/r5e/bench_sharded.log), and 4.5M-row batches (144 MB in one call) always passed.  So the fault follows
# one call that moves more than 2 GiB per peer (a 32-bit byte count or offset on the collective's path is the likely
# limit; which kernel took the illegal access was not isolated -- the library's debug build, MOBHEAT_BOUNDS_CHECK, now
# checks every segment read of the owner's merge).  The exchange never issues such a call: whatever
# MOBHEAT_EXCHANGE_ROUND_BYTES says, a round moves at most this much per pair
# (tests/test_distributed_gloo.py::test_exchange_round_cap records every call's per-pair sizes).
EXCHANGE_ROUND_CAP = 1 << 30
# the round size asked for (bytes per rank pair); values <= 0 or above the cap mean the cap
EXCHANGE_ROUND_BYTES = int(os.environ.get("MOBHEAT_EXCHANGE_ROUND_BYTES", str(EXCHANGE_ROUND_CAP)))


def round_bytes():
    """bytes per rank pair and all_to_all call: EXCHANGE_ROUND_BYTES clamped to (0, EXCHANGE_ROUND_CAP], whole words"""
    b = EXCHANGE_ROUND_BYTES
    if b <= 0 or b > EXCHANGE_ROUND_CAP:
        b = EXCHANGE_ROUND_CAP
    return max(8, b & ~7)


def _exchange_words(recv, words, recv_words, send_words, biggest):
    """all_to_all of int64 words: send_words[r] of `words` (concatenated by destination) to rank r, recv_words[s] from
    rank s into `recv` (concatenated by source).  `biggest`: the largest piece any pair moves, in words, the same on
    every rank (it sets the round count); rounds of at most round_bytes() per pair, every piece received in place."""
    world = len(send_words)
    step = round_bytes() // 8
    rounds = max(1, -(-int(biggest) // step))
    if rounds == 1:
        dist.all_to_all_single(recv[: sum(recv_words)], words, list(recv_words), list(send_words))
        return
    s_off = [sum(send_words[:r]) for r in range(world)]
    r_off = [sum(recv_words[:s]) for s in range(world)]
    for k in range(rounds):
        a = k * step
        ins = [words[s_off[r] + a: s_off[r] + a + max(0, min(step, send_words[r] - a))] for r in range(world)]
        outs = [recv[r_off[s] + a: r_off[s] + a + max(0, min(step, recv_words[s] - a))] for s in range(world)]
        _all_to_all_views(outs, ins)


def exchange_chunks(buf, send_bytes, device, status=0):
    """The batch's record exchange: one all_gather of every rank's per-destination chunk sizes in bytes (with its
    status: a rank whose stage failed sends status != 0 and no chunks, and every rank raises PeerFailed before the
    payloads move), then the chunks in rounds of at most round_bytes() per rank pair (one all_to_all when every pair
    fits), every piece received at its place -- as 8-byte words (chunk sizes are multiples of 32).  Returns (recv
    uint8 tensor, recv_bytes per source rank)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    g, _ = meta_group()
    row = torch.tensor([int(send_bytes[r]) if send_bytes else 0 for r in range(world)] + [status], dtype=torch.int64,
                       device="cpu" if g is not None else device)
    M = _meta_all_gather(row).tolist()   # M[s][r]: bytes s sends r; M[s][world]: s's status
    bad = [r for r in range(world) if M[r][world]]
    if bad and status == 0:
        raise PeerFailed(f"rank(s) {bad} failed the batch's stage before the exchange")
    if status:
        return None, []
    recv_bytes = [int(M[s][rank]) for s in range(world)]
    assert all(b % 8 == 0 for b in recv_bytes) and all(int(b) % 8 == 0 for b in send_bytes)
    nrecv, nsend = sum(recv_bytes), int(sum(send_bytes))
    recv = torch.empty(max(nrecv // 8, 2), dtype=torch.int64, device=device)
    words = buf[:nsend].view(torch.int64) if nsend else torch.empty(0, dtype=torch.int64, device=device)
    biggest = max(max(r[:world]) for r in M) // 8
    _exchange_words(recv, words, [b // 8 for b in recv_bytes], [int(b) // 8 for b in send_bytes], biggest)
    return recv.view(torch.uint8), recv_bytes


def _all_to_all_views(outs, ins):
    """all_to_all of tensor views: RCCL takes the lists as they are (grouped send/recv); gloo has only the single-tensor
    form, so the pieces go through one contiguous send and receive buffer there."""
    if dist.get_backend() == "nccl":
        dist.all_to_all(outs, ins)
        return
    send = torch.cat(ins) if ins else None
    recv = torch.empty(sum(o.numel() for o in outs), dtype=outs[0].dtype, device=outs[0].device)
    dist.all_to_all_single(recv, send, [o.numel() for o in outs], [i.numel() for i in ins])
    k = 0
    for o in outs:
        o.copy_(recv[k: k + o.numel()])
        k += o.numel()


def global_window_registry(summaries, tile_us):
    """Python twin of the library's stage_decide registry: the union of the ranks' windows in ascending order,
    hashed like k_ingest's registry (slot = window quotient mod WREG_SLOTS, linear probing).  Returns wenc per slot."""
    wins = set()
    for S in summaries:
        n = int(S[SW_NWIN])
        wins.update(int(x) & (2 ** 64 - 1) for x in S[SW_WIN0 + 1: SW_WIN0 + 2 * n: 2])
    reg = [0] * WREG_SLOTS
    for we in sorted(wins):
        u = we ^ (1 << 63)
        start = u - (1 << 64) if u >= (1 << 63) else u
        h = ((start // tile_us) % (1 << 64)) % WREG_SLOTS   # (C: (uint64_t)wq % WREG_SLOTS)
        for _ in range(WREG_SLOTS):
            if not reg[h]:
                break
            h = (h + 1) % WREG_SLOTS
        else:
            raise OverflowError("more than 4095 windows in one micro-batch")
        reg[h] = we
    return reg


class LibStages:
    """The library's stage API (hm_stage_ingest / send / merge / finish) on torch device buffers."""

    def __init__(self, engine):
        self.engine = engine
        self.lib = _lib.load()
        self.dev = torch.device("cuda", engine.device)
        self._bufs = {}
        self._summary = np.zeros(HM_STAGE_SUMMARY_WORDS, np.int64)

    def _buf(self, name, nbytes):
        b = self._bufs.get(name)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=self.dev)
            self._bufs[name] = b
        return b

    def ingest(self, epoch, batch, world, rank):
        """batch: n and the column pointers (device memory, or host memory with batch["memory"] = HM_MEM_HOST: the
        library copies them, sharded.py's per-rank slices of the micro-batch)."""
        self.world = world
        self._n = n = int(batch["n"])
        b = HmBatchIn(n=n, memory=int(batch.get("memory", HM_MEM_DEVICE)), lat=batch["lat"], lon=batch["lon"], ts_us=batch["ts_us"],
                      speed=batch.get("speed"), speed_valid=batch.get("speed_valid"), vkey=batch["vkey"],
                      row_valid=batch.get("row_valid"))
        ctx = self.engine._ctx
        check(self.lib.hm_stage_ingest(ctx, int(epoch), ctypes.byref(b), world, rank, self._summary.ctypes.data), ctx,
              "hm_stage_ingest")
        return self._summary

    def send(self, summaries):
        """-> (send buffer, bytes of each destination's chunk)"""
        world, n = self.world, self._n
        summaries = np.ascontiguousarray(summaries, dtype=np.int64)
        cap = int(self.lib.hm_stage_send_capacity(n, world))
        buf = self._buf("send", cap)
        sb = (ctypes.c_int64 * world)()
        sizes = HmStageSizes()
        ctx = self.engine._ctx
        check(self.lib.hm_stage_send(ctx, summaries.ctypes.data, buf.data_ptr(), cap, sb, ctypes.byref(sizes)), ctx,
              "hm_stage_send")
        self.table_mode = bool(sizes.table_mode)
        self.sizes = sizes
        return buf, list(sb)

    def merge(self, recv, recv_bytes, out_memory):
        world = self.world
        cap = max(sum(recv_bytes) // 32, 1)   # (candidates are 32 B each: at most one winner per received 32 B)
        winner_send = self._buf("winner", cap * 8)
        rb = (ctypes.c_int64 * world)(*recv_bytes)
        wc = (ctypes.c_int64 * world)()
        out = HmBatchOut()
        ctx = self.engine._ctx
        check(self.lib.hm_stage_merge(ctx, recv.data_ptr(), rb, out_memory, ctypes.byref(out), winner_send.data_ptr(),
                                      cap, wc), ctx, "hm_stage_merge")
        return out, Stream("winner", winner_send, list(wc), 8)

    def wait_stream(self, stream):
        """The library's stream waits for the work queued on `stream` (torch's current stream, where the collective
        ran): hm_stream_wait, no host synchronization."""
        ctx = self.engine._ctx
        check(self.lib.hm_stream_wait(ctx, stream.cuda_stream), ctx, "hm_stream_wait")

    def finish(self, winner_recv, n_winner, out_memory, out):
        ctx = self.engine._ctx
        check(self.lib.hm_stage_finish(ctx, winner_recv.data_ptr(), n_winner, out_memory, ctypes.byref(out)), ctx,
              "hm_stage_finish")
        return out


class _PhaseClock:
    """host wall time of each phase of a sharded batch (ms; a phase ends where the host next waits for the device or a
    collective: the stages' own synchronizations, .cpu() of the collectives' sizes)"""

    def __init__(self):
        import time
        self._t = time.perf_counter
        self._last = self._t()
        self.ms = {}

    def __call__(self, name):
        t = self._t()
        self.ms[name] = round(1e3 * (t - self._last), 3)
        self._last = t


class ShardedHeatmap:
    """One rank of the sharded hot path. ``stages`` provides ingest / send / merge / finish (LibStages on GPUs)."""

    def __init__(self, stages, device):
        self.stages = stages
        self.device = device
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        # the last batch's receive buffers: with out_memory=HM_MEM_DEVICE, out.latest_row points into the winners'
        # receive buffer (hm_stage_finish), so they stay alive until the next process_batch call
        self._recv = None

    def after_collective(self):
        """Order the library's next reads after the collectives queued so far: the library reads received buffers on
        its own stream, after RCCL's (torch's current stream) -- an event wait between the two streams (the stages'
        wait_stream, hm_stream_wait), not a host synchronization; without wait_stream, the current stream is
        synchronized; on the CPU (gloo) nothing is asynchronous."""
        if self.device.type != "cuda":
            return
        wait = getattr(self.stages, "wait_stream", None)
        if wait is not None:
            wait(torch.cuda.current_stream(self.device))
        else:
            torch.cuda.current_stream(self.device).synchronize()

    def process_batch(self, epoch, batch, out_memory=HM_MEM_DEVICE, sync=None):
        """One micro-batch on this rank.  A stage that raises on one rank makes every rank leave at the next
        collective (the failed rank re-raises its error, the others PeerFailed), so no rank waits on a collective its
        peers never reach."""
        if sync is None:
            sync = self.after_collective
        err = None
        clock = _PhaseClock()
        try:
            summary = self.stages.ingest(epoch, batch, self.world, self.rank)
        except Exception as e:
            err, summary = e, np.zeros(HM_STAGE_SUMMARY_WORDS, np.int64)
        clock("ingest")
        summaries = all_gather_summaries(summary, self.device, status=1 if err else 0)
        clock("summaries")
        if err:
            raise err
        try:
            buf, send_bytes = self.stages.send(summaries)
        except Exception as e:
            exchange_chunks(None, None, self.device, status=1)
            raise e
        clock("send")
        recv, recv_bytes = exchange_chunks(buf, send_bytes, self.device)
        sync()
        clock("exchange")
        try:
            out, winners = self.stages.merge(recv, recv_bytes, out_memory)
        except Exception as e:
            exchange([], self.device, status=1)
            raise e
        clock("merge")
        [(winner_recv, wrc)] = exchange([winners], self.device)
        sync()
        clock("winners")
        self._recv = (recv, winner_recv)
        res = self.stages.finish(winner_recv, int(sum(wrc)), out_memory, out)
        clock("finish")
        self.last_phase_ms = clock.ms
        return res


def tile_hash(cell, wstart):
    """Python twin of kernels.h tile_hash (the key_hash field of a tile partial record)."""
    with np.errstate(over="ignore"):
        return _mix64(np.asarray(cell, np.uint64) ^ _mix64(np.asarray(wstart).astype(np.uint64) +
                                                           np.uint64(0x9E3779B97F4A7C15)))


REGION_BITS = 13


def region_field(h):
    """Python twin of kernels.h region_field: hash bits [32 - REGION_BITS, 32)."""
    return ((np.asarray(h, np.uint64) >> np.uint64(32 - REGION_BITS)) & np.uint64((1 << REGION_BITS) - 1)).astype(np.int64)


def shard_lo(r, world):
    """The first region field rank r of `world` owns (kernels.h shard_lo)."""
    return ((r << REGION_BITS) + world - 1) // world


def tile_owner(cell, wstart, world):
    """Python twin of the device routing (kernels.h tile_owner_of(tile_hash(...))): contiguous region-field ranges."""
    return (region_field(tile_hash(cell, wstart)) * world) >> REGION_BITS


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
