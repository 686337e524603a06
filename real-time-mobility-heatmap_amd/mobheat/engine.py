"""HeatmapEngine: one device context running the per-micro-batch hot path on one GPU.

Wraps hm_create / hm_process_batch / hm_destroy (include/mobheat.h).  The engine owns the persistent
tile state (Spark's state store for the window aggregation, reference heatmap_stream.py:111-133 in
update mode, :243) and the watermark bookkeeping (withWatermark 10 minutes, :107).
"""
import ctypes
import json
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import (HM_JSON_SPLICE, HM_MEM_DEVICE, HM_MEM_HOST, HM_MEM_HOST_STREAM, STATE_REC_DTYPE, HmArrowIn, HmBatchIn, HmBatchOut, HmConfig,
                   HmJsonIn, HmJsonOut, HmStateInfo, check, ptr)

_INFO_FIELDS = [f for f, _ in HmStateInfo._fields_ if f != "reserved"]


@dataclass
class TileRows:
    """Update-mode output of the tiles aggregation (reference heatmap_stream.py:124-132)."""
    cell: np.ndarray            # uint64 H3 index (cellId = format(cell, 'x'))
    window_start_us: np.ndarray  # int64
    window_end_us: np.ndarray    # int64
    count: np.ndarray            # int64
    avg_speed: np.ndarray        # float64 (0.0 where speed_null)
    speed_null: np.ndarray       # bool: avg(speedKmh) is null (no non-null speed in the group)
    avg_lon: np.ndarray          # float64
    avg_lat: np.ndarray          # float64

    def __len__(self):
        return int(self.cell.size)


@dataclass
class KafkaBatch:
    """hm_decode_json's result: device columns (batch, valid until the next decode on the engine) and copies of the
    batch's string dictionaries (vkey = provider_code * n_vehicles + vehicle_code)."""
    batch: HmBatchIn
    providers: tuple            # (n, offsets int64[n+1], bytes uint8): Arrow layout, as _lib._dictionary builds
    vehicles: tuple
    n_malformed: int
    n_spliced: int = 0          # records decoded on the host (kafka_host) and written in with hm_json_patch


@dataclass
class BatchResult:
    tiles: TileRows             # None when the rows stayed on the device (rows_on_device=True)
    latest_rows: np.ndarray     # int64 row indices of the in-batch latest positions (ties included); None likewise
    n_in: int
    n_valid: int
    n_late: int
    n_state: int
    batch_max_event_ms: int
    watermark_ms: int
    late_watermark_ms: int
    n_partials: int = 0         # partial records merged (direct path: aggregated rows; table mode: ~ distinct keys)
    n_tiles: int = 0
    n_latest: int = 0


def _extend_dictionary(d, strings):
    """Arrow-layout dictionary (n, offsets, bytes) + strings (str or None) -> (the dictionary with the new strings
    appended, int64 codes: -1 for None)."""
    n, offs, raw = d
    have = {raw[offs[i]:offs[i + 1]].tobytes(): i for i in range(n)} if any(s is not None for s in strings) else {}
    new, codes = [], np.full(len(strings), -1, np.int64)
    for k, s in enumerate(strings):
        if s is None:
            continue
        b = s.encode("utf-8")
        code = have.get(b)
        if code is None:
            code = have[b] = n + len(new)
            new.append(b)
        codes[k] = code
    if not new:
        return d, codes
    tail = np.cumsum([len(b) for b in new], dtype=np.int64) + offs[n]
    blob = np.frombuffer(b"".join(new), np.uint8) if any(new) else np.zeros(0, np.uint8)
    raw2 = np.concatenate([raw[:offs[n]], blob]) if int(tail[-1]) else np.zeros(1, np.uint8)
    return (n + len(new), np.concatenate([offs[:n + 1], tail]), raw2), codes


def _u8(a, n):
    if a is None:
        return None
    a = np.ascontiguousarray(a)
    if a.dtype == np.bool_:
        a = a.view(np.uint8)
    assert a.dtype == np.uint8 and a.size == n
    return a


class HeatmapEngine:
    def __init__(self, h3_res=8, tile_minutes=5, watermark_delay_ms=600_000, device=0,
                 late_uses_prev_watermark=True, state_capacity_hint=0, batch_capacity_hint=0, state_arena_bytes=0,
                 shard=None):
        """shard: (rank, world) of a multi-GPU stage context (its state holds only the keys that rank owns); None =
        fixed by the first hm_stage_ingest, or a single GPU."""
        self._lib = _lib.load()
        self.h3_res = int(h3_res)
        self.tile_us = int(tile_minutes) * 60 * 1_000_000
        self.device = int(device)
        cfg = HmConfig(abi_version=_lib.HM_ABI_VERSION, h3_res=self.h3_res, device=self.device,
                       late_uses_prev_watermark=1 if late_uses_prev_watermark else 0, tile_us=self.tile_us,
                       watermark_delay_ms=int(watermark_delay_ms), state_capacity_hint=int(state_capacity_hint),
                       batch_capacity_hint=int(batch_capacity_hint), state_arena_bytes=int(state_arena_bytes),
                       shard_rank=int(shard[0]) if shard else 0, shard_count=int(shard[1]) if shard else 0)
        h = ctypes.c_void_p()
        check(self._lib.hm_create(ctypes.byref(cfg), ctypes.byref(h)), None, "hm_create")
        self._ctx = h

    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.hm_destroy(self._ctx)
            self._ctx = None
        self._free_pinned()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- host-memory batch (the foreach_batch_func path) ----
    def process_batch(self, epoch_id, lat, lon, ts_us, speed=None, speed_valid=None, vkey=None, row_valid=None,
                      copy=True, rows_on_device=False):
        """One micro-batch from host columns (the foreach_batch_func path).  copy=False returns views of the
        library's pinned output buffers, valid until the next call on this engine (a 1e8-tile batch's outputs are
        ~5 GB: copying them costs about as much as the whole GPU pipeline and both PCIe transfers).
        rows_on_device=True leaves the tile rows and latest rows on the device (tiles / latest_rows None, the counts
        in n_tiles / n_latest): what the writer needs, since it encodes the statements from the device rows."""
        n = int(np.asarray(lat).size)
        lat = np.ascontiguousarray(lat, dtype=np.float64)
        lon = np.ascontiguousarray(lon, dtype=np.float64)
        ts_us = np.ascontiguousarray(ts_us, dtype=np.int64)
        assert lon.size == n and ts_us.size == n
        speed = None if speed is None else np.ascontiguousarray(speed, dtype=np.float64)
        vkey = np.zeros(n, np.uint64) if vkey is None else np.ascontiguousarray(vkey, dtype=np.uint64)
        b = HmBatchIn(n=n, memory=HM_MEM_HOST, lat=ptr(lat), lon=ptr(lon), ts_us=ptr(ts_us), speed=ptr(speed),
                      speed_valid=ptr(_u8(speed_valid, n)), vkey=ptr(vkey), row_valid=ptr(_u8(row_valid, n)))
        out = HmBatchOut()
        mem = HM_MEM_DEVICE if rows_on_device else HM_MEM_HOST
        check(self._lib.hm_process_batch(self._ctx, int(epoch_id), ctypes.byref(b), mem, ctypes.byref(out)),
              self._ctx, "hm_process_batch")
        return self._result_counts(out) if rows_on_device else self._result_from_host(out, copy)

    # ---- Kafka values (row f1): JSON decoded on the GPU, then the batch ----
    def decode_json(self, values, offsets):
        """The micro-batch's Kafka values (bytes uint8 back to back + offsets int64[n+1], Arrow's binary layout) ->
        KafkaBatch: from_json(value, schema) + to_timestamp(ts) on the device (reference heatmap_stream.py:88-93).
        The records outside the device decoder (HM_JSON_SPLICE lists them) are decoded on the host and spliced in."""
        buf = np.ascontiguousarray(values, dtype=np.uint8)
        offs = np.ascontiguousarray(offsets, dtype=np.int64)
        jin = HmJsonIn(n=offs.size - 1, memory=HM_MEM_HOST, flags=HM_JSON_SPLICE, bytes=ptr(buf) if buf.size else None,
                       offsets=ptr(offs))
        jout = HmJsonOut()
        check(self._lib.hm_decode_json(self._ctx, ctypes.byref(jin), ctypes.byref(jout)), self._ctx, "hm_decode_json")
        kb = _device_batch(jout)
        m = int(jout.n_unsupported)
        if m:
            rows = np.ctypeslib.as_array(ctypes.cast(jout.unsupported_rows, ctypes.POINTER(ctypes.c_int64)),
                                         shape=(m,)).copy()
            self._splice(kb, buf, offs, rows)
        return kb

    def _splice(self, kb, buf, offs, rows):
        """Decode records `rows` on the host (kafka_host: the device decoder's rules plus the cases it leaves out),
        extend the string dictionaries with their new strings and write them into the device batch (hm_json_patch)."""
        from . import kafka_host
        c = kafka_host.decode_columns(buf, offs, rows)
        kb.providers, pcode = _extend_dictionary(kb.providers, c["provider"])
        kb.vehicles, vcode = _extend_dictionary(kb.vehicles, c["vehicleId"])
        m = rows.size
        f64 = lambda v: np.array([np.nan if x is None else x for x in v], np.float64)   # noqa: E731
        lat, lon = f64(c["lat"]), f64(c["lon"])
        sv = np.array([x is not None for x in c["speedKmh"]], np.uint8)
        speed = np.where(sv.astype(bool), f64(c["speedKmh"]), 0.0)
        ts_ok = np.asarray(c["ts_ok"], bool)
        rv = ((pcode >= 0) & (vcode >= 0) & ts_ok).astype(np.uint8)
        ts = np.where(ts_ok, np.asarray(c["ts_us"], np.int64), 0)
        pcode, vcode = np.maximum(pcode, 0), np.maximum(vcode, 0)
        check(self._lib.hm_json_patch(self._ctx, m, ptr(rows), ptr(lat), ptr(lon), ptr(ts), ptr(speed), ptr(sv),
                                      ptr(rv), ptr(pcode), ptr(vcode), kb.providers[0], kb.vehicles[0]),
              self._ctx, "hm_json_patch")
        kb.n_malformed += int(sum(c["malformed"]))
        kb.n_spliced = int(m)

    def arrow_columns(self, arrow_in):
        """hm_arrow_columns: the micro-batch's Arrow columns (an HmArrowIn over host buffers the caller keeps alive,
        stream.ArrowColumns) -> KafkaBatch: the batch columns on the device and the string dictionaries."""
        jout = HmJsonOut()
        check(self._lib.hm_arrow_columns(self._ctx, ctypes.byref(arrow_in), ctypes.byref(jout)), self._ctx,
              "hm_arrow_columns")
        return _device_batch(jout)

    def process_arrow(self, epoch_id, arrow_in, copy=True, rows_on_device=False):
        """arrow_columns + hm_process_batch on the device columns; (BatchResult, KafkaBatch)."""
        kb = self.arrow_columns(arrow_in)
        out = HmBatchOut()
        mem = HM_MEM_DEVICE if rows_on_device else HM_MEM_HOST
        check(self._lib.hm_process_batch(self._ctx, int(epoch_id), ctypes.byref(kb.batch), mem, ctypes.byref(out)),
              self._ctx, "hm_process_batch")
        return (self._result_counts(out) if rows_on_device else self._result_from_host(out, copy)), kb

    def process_kafka(self, epoch_id, values, offsets, copy=True, rows_on_device=False):
        """decode_json + hm_process_batch on the decoded device columns; (BatchResult, KafkaBatch)."""
        kb = self.decode_json(values, offsets)
        out = HmBatchOut()
        mem = HM_MEM_DEVICE if rows_on_device else HM_MEM_HOST
        check(self._lib.hm_process_batch(self._ctx, int(epoch_id), ctypes.byref(kb.batch), mem, ctypes.byref(out)),
              self._ctx, "hm_process_batch")
        return (self._result_counts(out) if rows_on_device else self._result_from_host(out, copy)), kb

    def latest_buckets(self):
        """The distinct 900-s buckets of the last batch's latest rows' eventTs (computed on the device)."""
        n = ctypes.c_int64()
        check(self._lib.hm_last_latest_buckets(self._ctx, None, 0, ctypes.byref(n)), self._ctx, "hm_last_latest_buckets")
        ids = np.zeros(max(n.value, 1), np.int64)
        if n.value:
            check(self._lib.hm_last_latest_buckets(self._ctx, ptr(ids), ids.size, ctypes.byref(n)), self._ctx,
                  "hm_last_latest_buckets")
        return ids[:n.value]

    # ---- device-resident batch (bench / multi-GPU): raw device pointers, results stay on the device ----
    def process_batch_device(self, epoch_id, n, lat, lon, ts_us, speed, speed_valid, vkey, row_valid):
        b = HmBatchIn(n=int(n), memory=HM_MEM_DEVICE, lat=lat, lon=lon, ts_us=ts_us, speed=speed,
                      speed_valid=speed_valid, vkey=vkey, row_valid=row_valid)
        out = HmBatchOut()
        check(self._lib.hm_process_batch(self._ctx, int(epoch_id), ctypes.byref(b), HM_MEM_DEVICE,
                                         ctypes.byref(out)), self._ctx, "hm_process_batch")
        return out

    # ---- tile-state checkpoint (Spark's state store under checkpointLocation, heatmap_stream.py:37,244) ----
    def export_state(self, reuse=False):
        """(info dict, records) of the persistent tile state after the last batch: one STATE_REC_DTYPE record per
        live (cell, windowStart) key with its cumulative count / non-null speed count / sums, plus the epoch and
        watermarks the next batch continues from.  reuse: as export_state_delta."""
        info = HmStateInfo()
        check(self._lib.hm_state_export(self._ctx, ctypes.byref(info), None, 0), self._ctx, "hm_state_export")
        recs = self._export_buffer(int(info.n_keys), reuse)
        if recs.size:
            check(self._lib.hm_state_export(self._ctx, ctypes.byref(info), ptr(recs), recs.size), self._ctx,
                  "hm_state_export")
        return {f: int(getattr(info, f)) for f in _INFO_FIELDS}, recs

    def state_version(self):
        """Bumped whenever a batch starts merging into the persistent state (a failed call that left it unchanged did
        not touch the state)."""
        return int(self._lib.hm_state_version(self._ctx))

    def _export_buffer(self, n, reuse, raw_out=None):
        """n state records of host memory: a fresh array, or (reuse) a view of the engine's page-locked export buffer --
        valid until the next reuse export (a device-to-host copy into pageable memory ran at ~10 GB/s: 66 ms of a
        1e7-key delta, profiles/r5).  The buffer is page-aligned and holds the records rounded up to 4 KiB (the
        checkpoint writer's O_DIRECT writes); raw_out (a list) receives the whole buffer as uint8."""
        if not reuse:
            return np.zeros(n, STATE_REC_DTYPE)
        nbytes = max(n, 1) * STATE_REC_DTYPE.itemsize
        need = -(-nbytes // 4096) * 4096
        buf = getattr(self, "_pinned", None)
        if buf is None or buf[1] < need:
            self._free_pinned()
            p = ctypes.c_void_p()
            cap = max(need, -(-(nbytes + nbytes // 4) // 4096) * 4096)
            check(self._lib.hm_host_alloc(cap, ctypes.byref(p)), None, "hm_host_alloc")
            buf = self._pinned = (p.value, cap)
        raw = np.ctypeslib.as_array(ctypes.cast(buf[0], ctypes.POINTER(ctypes.c_uint8)), shape=(buf[1],))
        if raw_out is not None:
            raw_out.append(raw)
        return raw[: n * STATE_REC_DTYPE.itemsize].view(STATE_REC_DTYPE)

    def export_begin(self, touched_only, slice_records=1 << 19):
        """hm_state_export_begin: the state (or the last batch's touched keys) dumped on the device, and its copy into
        the page-locked export buffer enqueued in slices (hm_state_export_copy_async, at most 64; call this before the
        statements' encode, whose copies then queue behind these) -> (info dict, n, recs, raw, fill): recs a view of
        the buffer (raw: all of it, uint8); fill(first, count) returns once records [first, first + count) have landed
        (hm_state_export_copy_wait) -- from any thread, while this engine encodes the batch's statements (the
        checkpoint writer: mobheat.checkpoint)."""
        info = HmStateInfo()
        n = ctypes.c_int64()
        check(self._lib.hm_state_export_begin(self._ctx, ctypes.byref(info), int(bool(touched_only)), ctypes.byref(n)),
              self._ctx, "hm_state_export_begin")
        n = int(n.value)
        raw = []
        recs = self._export_buffer(n, True, raw)
        base = raw[0].ctypes.data
        size = STATE_REC_DTYPE.itemsize
        s = max(int(slice_records), -(-n // 64), 1)
        for k in range(-(-n // s)):
            lo = k * s
            check(self._lib.hm_state_export_copy_async(self._ctx, base + lo * size, lo, min(s, n - lo), k), self._ctx,
                  "hm_state_export_copy_async")

        def fill(first, count):
            if first < 0 or count < 0 or first + count > n:
                raise RuntimeError(f"hm_state_export_copy: records [{first}, {first + count}) outside the dump of {n}")
            for k in range(first // s, -(-(first + count) // s)):
                check(self._lib.hm_state_export_copy_wait(self._ctx, k), self._ctx, "hm_state_export_copy_wait")
        return {f: int(getattr(info, f)) for f in _INFO_FIELDS}, n, recs, raw[0], fill

    def _free_pinned(self):
        buf = getattr(self, "_pinned", None)
        if buf is not None:
            self._pinned = None
            self._lib.hm_host_free(buf[0])

    def export_state_delta(self, reuse=False):
        """(info dict, records) of the keys the last batch touched: an incremental checkpoint (see merge_state).
        reuse: the records are a view of the engine's page-locked export buffer (valid until the next reuse export)."""
        info = HmStateInfo()
        n = ctypes.c_int64()
        check(self._lib.hm_state_export_touched(self._ctx, ctypes.byref(info), None, 0, ctypes.byref(n)), self._ctx,
              "hm_state_export_touched")
        recs = self._export_buffer(int(n.value), reuse)
        if recs.size:
            check(self._lib.hm_state_export_touched(self._ctx, ctypes.byref(info), ptr(recs), recs.size, ctypes.byref(n)),
                  self._ctx, "hm_state_export_touched")
            recs = recs[: int(n.value)]
        return {f: int(getattr(info, f)) for f in _INFO_FIELDS}, recs

    def import_state(self, info, recs):
        """Restore an exported state into this engine (which must not have processed a batch yet)."""
        recs = np.ascontiguousarray(recs, dtype=STATE_REC_DTYPE)
        hi = HmStateInfo(**{f: int(info[f]) for f in _INFO_FIELDS})
        hi.n_keys = recs.size
        check(self._lib.hm_state_import(self._ctx, ctypes.byref(hi), ptr(recs) if recs.size else None), self._ctx,
              "hm_state_import")

    def save_state(self, path):
        """export_state() written atomically to `path` (save_state_file: a JSON header and the raw records)."""
        info, recs = self.export_state()
        save_state_file(path, info, recs)
        return info

    def load_state(self, path):
        info, recs = load_state_file(path)
        self.import_state(info, recs)
        return info

    # ---- tiles as MongoDB update statements, BSON-encoded on the GPU (reference heatmap_stream.py:164-196) ----
    def encode_tile_updates_streamed(self, city, ttl_minutes):
        """encode_tile_updates with HM_MEM_HOST_STREAM: (bytes, offsets, landed) -- the offsets are there, the bytes
        land in pieces after the call; landed(upto) blocks until bytes[:upto] have (hm_statements_wait).  The sink
        sends each command once its statements have landed (mobheat.stream._flush_statements)."""
        return self._encode_tiles(city, ttl_minutes, HM_MEM_HOST_STREAM)

    def encode_position_updates_streamed(self, provider_uniques, vehicle_uniques):
        """encode_position_updates with HM_MEM_HOST_STREAM: (bytes, offsets, landed), as encode_tile_updates_streamed."""
        bucket_ids = self.latest_buckets()
        cfg, keep = _lib.position_doc_cfg(provider_uniques, vehicle_uniques, None, bucket_ids=bucket_ids)
        pb, po, nd = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
        check(self._lib.hm_encode_position_updates(self._ctx, ctypes.byref(cfg), HM_MEM_HOST_STREAM, ctypes.byref(pb),
                                                   ctypes.byref(po), ctypes.byref(nd)), self._ctx,
              "hm_encode_position_updates")
        return _host_statements(pb, po, nd, False) + (self._landed,)

    def _landed(self, upto):
        check(self._lib.hm_statements_wait(self._ctx, int(upto)), self._ctx, "hm_statements_wait")

    def _encode_tiles(self, city, ttl_minutes, memory):
        n = ctypes.c_int64()
        check(self._lib.hm_last_windows(self._ctx, None, 0, ctypes.byref(n)), self._ctx, "hm_last_windows")
        wins = np.zeros(n.value, np.int64)
        if wins.size:
            check(self._lib.hm_last_windows(self._ctx, ptr(wins), wins.size, ctypes.byref(n)), self._ctx, "hm_last_windows")
        cfg, keep = _lib.tile_doc_cfg(city, ttl_minutes, wins, self.tile_us)
        pb, po, nd = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
        check(self._lib.hm_encode_tile_updates(self._ctx, ctypes.byref(cfg), memory, ctypes.byref(pb),
                                               ctypes.byref(po), ctypes.byref(nd)), self._ctx, "hm_encode_tile_updates")
        return _host_statements(pb, po, nd, False) + (self._landed,)

    def encode_tile_updates(self, city, ttl_minutes, copy=False):
        """The last batch's tiles as the `update` statements pymongo would send for the reference's UpdateOne ops:
        (bytes uint8, offsets int64[n+1]); statement i = bytes[offsets[i]:offsets[i+1]].  Views of the library's
        pinned buffers, valid until the next call on this engine (copy=True to keep them)."""
        n = ctypes.c_int64()
        check(self._lib.hm_last_windows(self._ctx, None, 0, ctypes.byref(n)), self._ctx, "hm_last_windows")
        wins = np.zeros(n.value, np.int64)
        if wins.size:
            check(self._lib.hm_last_windows(self._ctx, ptr(wins), wins.size, ctypes.byref(n)), self._ctx, "hm_last_windows")
        cfg, keep = _lib.tile_doc_cfg(city, ttl_minutes, wins, self.tile_us)
        pb, po, nd = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
        check(self._lib.hm_encode_tile_updates(self._ctx, ctypes.byref(cfg), HM_MEM_HOST, ctypes.byref(pb),
                                               ctypes.byref(po), ctypes.byref(nd)), self._ctx, "hm_encode_tile_updates")
        return _host_statements(pb, po, nd, copy)

    def encode_position_updates(self, provider_uniques, vehicle_uniques, latest_ts_us=None, copy=False):
        """The last batch's latest rows as positions_latest update statements (reference heatmap_stream.py:211-235):
        (bytes uint8, offsets int64[n+1]).  The dictionaries are the batch's factorization its vkeys were built
        from (vkey = provider_code * n_vehicles + vehicle_code): lists of strings, or (n, offsets, bytes) as
        decode_json returns them.  The local offsets are looked up for the 900-s buckets of latest_ts_us (the
        latest rows' eventTs), or, when it is None, of the buckets the device finds among the latest rows."""
        bucket_ids = self.latest_buckets() if latest_ts_us is None else None
        cfg, keep = _lib.position_doc_cfg(provider_uniques, vehicle_uniques, latest_ts_us, bucket_ids=bucket_ids)
        pb, po, nd = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
        check(self._lib.hm_encode_position_updates(self._ctx, ctypes.byref(cfg), HM_MEM_HOST, ctypes.byref(pb),
                                                   ctypes.byref(po), ctypes.byref(nd)), self._ctx,
              "hm_encode_position_updates")
        return _host_statements(pb, po, nd, copy)

    def encode_tile_updates_device(self, city, ttl_minutes):
        """The same, left on the device: (device pointer of the bytes, of the offsets, n statements)."""
        n = ctypes.c_int64()
        check(self._lib.hm_last_windows(self._ctx, None, 0, ctypes.byref(n)), self._ctx, "hm_last_windows")
        wins = np.zeros(n.value, np.int64)
        if wins.size:
            check(self._lib.hm_last_windows(self._ctx, ptr(wins), wins.size, ctypes.byref(n)), self._ctx, "hm_last_windows")
        cfg, keep = _lib.tile_doc_cfg(city, ttl_minutes, wins, self.tile_us)
        pb, po, nd = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
        check(self._lib.hm_encode_tile_updates(self._ctx, ctypes.byref(cfg), HM_MEM_DEVICE, ctypes.byref(pb),
                                               ctypes.byref(po), ctypes.byref(nd)), self._ctx, "hm_encode_tile_updates")
        return pb.value, po.value, nd.value

    def last_timings(self):
        ms = (ctypes.c_double * 8)()
        check(self._lib.hm_last_timings(self._ctx, ms, 8), self._ctx)
        return {"ingest": ms[0], "aggregate": ms[1], "merge": ms[2], "emit": ms[3], "dedup": ms[4], "total": ms[5],
                "partition": ms[6], "send": ms[7]}

    def last_host_timings(self):
        """Host side of the last process_batch (ms): the call, stream synchronizations, allocations + frees, the
        longest synchronization and its library source line, allocations + frees made."""
        ms = (ctypes.c_double * 14)()
        check(self._lib.hm_last_timings(self._ctx, ms, 14), self._ctx)
        return {"call": ms[8], "sync": ms[9], "alloc": ms[10], "max_sync": ms[11], "max_sync_line": int(ms[12]),
                "allocs_frees": int(ms[13])}

    def last_counts(self):
        c = (ctypes.c_int64 * 11)()
        check(self._lib.hm_last_counts(self._ctx, c, 11), self._ctx)
        return {"state_new": c[0], "partials": c[1], "tiles": c[2], "table_mode": bool(c[3]), "evicted": c[4],
                "sent": c[5], "allocs": c[6], "frees": c[7], "binned": bool(c[8]), "self_held": c[9],
                "pipe_chunks": c[10]}

    def _result_from_host(self, out, copy=True):
        def arr(p, n, dt):
            if n == 0 or not p:
                return np.zeros(0, dt)
            a = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(n,))
            return a.copy() if copy else a
        nt = int(out.n_tiles)
        ws = arr(out.window_start_us, nt, np.int64)
        tiles = TileRows(cell=arr(out.cell, nt, np.uint64), window_start_us=ws, window_end_us=ws + self.tile_us,
                         count=arr(out.count, nt, np.int64), avg_speed=arr(out.avg_speed, nt, np.float64),
                         speed_null=arr(out.speed_null, nt, np.uint8).view(np.bool_),
                         avg_lon=arr(out.avg_lon, nt, np.float64), avg_lat=arr(out.avg_lat, nt, np.float64))
        return BatchResult(tiles=tiles, latest_rows=arr(out.latest_row, int(out.n_latest), np.int64),
                           n_in=int(out.n_in), n_valid=int(out.n_valid), n_late=int(out.n_late),
                           n_state=int(out.n_state), batch_max_event_ms=int(out.batch_max_event_ms),
                           watermark_ms=int(out.watermark_ms), late_watermark_ms=int(out.late_watermark_ms),
                           n_partials=int(out.n_partials), n_tiles=nt, n_latest=int(out.n_latest))

    @staticmethod
    def _result_counts(out):
        """The statistics of a batch whose rows stayed on the device (HM_MEM_DEVICE outputs)."""
        return BatchResult(tiles=None, latest_rows=None, n_in=int(out.n_in), n_valid=int(out.n_valid),
                           n_late=int(out.n_late), n_state=int(out.n_state),
                           batch_max_event_ms=int(out.batch_max_event_ms), watermark_ms=int(out.watermark_ms),
                           late_watermark_ms=int(out.late_watermark_ms), n_partials=int(out.n_partials),
                           n_tiles=int(out.n_tiles), n_latest=int(out.n_latest))


def _device_batch(jout):
    """KafkaBatch of an HmJsonOut (hm_decode_json / hm_arrow_columns): the device columns and copies of the dictionaries
    (the library's pinned buffers are reused by the next call)."""
    def dictionary(n, po, pb):
        offs_ = np.ctypeslib.as_array(ctypes.cast(po, ctypes.POINTER(ctypes.c_int64)), shape=(n + 1,)).copy()
        total = int(offs_[-1])
        raw = (np.ctypeslib.as_array(ctypes.cast(pb, ctypes.POINTER(ctypes.c_uint8)), shape=(total,)).copy()
               if total else np.zeros(1, np.uint8))
        return n, offs_, raw
    return KafkaBatch(batch=jout.batch, providers=dictionary(int(jout.n_providers), jout.provider_offsets, jout.provider_bytes),
                      vehicles=dictionary(int(jout.n_vehicles), jout.vehicle_offsets, jout.vehicle_bytes),
                      n_malformed=int(jout.n_malformed))


def _host_statements(pb, po, nd, copy):
    """(bytes, offsets) of statements in the library's pinned host buffers: views valid until the next call on the
    engine unless copy=True (a 1e8-tile batch is ~37 GB: a copy costs seconds)."""
    offs = np.ctypeslib.as_array(ctypes.cast(po, ctypes.POINTER(ctypes.c_int64)), shape=(nd.value + 1,))
    total = int(offs[-1])
    buf = (np.ctypeslib.as_array(ctypes.cast(pb, ctypes.POINTER(ctypes.c_uint8)), shape=(total,))
           if total else np.zeros(0, np.uint8))
    return (buf.copy(), offs.copy()) if copy else (buf, offs)


def merge_state(base, deltas):
    """The state after the last of `deltas` from a full export `base` and the incremental exports of the batches since,
    in order (each an (info, recs) pair): the last-written record of every (cell, windowStart) key, keeping the keys
    whose window outlives the last batch's eviction watermark (hm_state_export_touched).  Returns (info, recs)."""
    info, recs = base
    parts = [recs] + [d[1] for d in deltas]
    if deltas:
        info = deltas[-1][0]
    allr = np.concatenate(parts) if len(parts) > 1 else recs
    if allr.size:
        # last occurrence of each key wins: reverse, stable unique on (cell, window_start), map back
        rev = allr[::-1]
        key = np.empty(rev.size, dtype=[("c", "<u8"), ("w", "<i8")])
        key["c"], key["w"] = rev["cell"], rev["window_start_us"]
        _, first = np.unique(key, return_index=True)
        allr = rev[np.sort(first)]
        tile_us = int(info["tile_us"])
        allr = allr[allr["window_start_us"] + tile_us > int(info["prev_watermark_ms"]) * 1000]
    info = dict(info, n_keys=int(allr.size))
    return info, np.ascontiguousarray(allr)


STATE_FILE_MAGIC = b"MHSTATE1"   # raw state file: magic, u64 header bytes, JSON header, padding to 64 B, the records


def save_state_file(path, info, recs, meta=None, fill=None, raw=None):
    """info + records written atomically to `path` (tmp file, fsync, rename): a JSON header (the hm_state_info fields,
    the record count and layout, `meta` -- a str: the checkpoint chain record, mobheat.checkpoint) and the 64-B records
    as raw bytes.  (np.savez's zip container CRC-checked and copied every byte under the GIL: the checkpoint thread then
    slowed the next batch's host work and waited ~0.4 s per 10M-key delta, profiles/r4.)

    fill / raw (Engine.export_begin): the records are still on the device -- fill(first, count) copies them into recs,
    slice by slice on a copier thread while this thread writes the slices that have landed; raw is recs' page-aligned
    buffer, and the file then goes to the disk with O_DIRECT writes straight from it (the header padded to 4 KiB), so
    that neither a page-cache copy nor an fsync of the data follows the write (on the GPU box: 635 MB in ~85 ms vs
    ~62 ms write + ~63 ms fsync buffered, profiles/r6/r6d/file_probe.log).  MOBHEAT_CKPT_DIRECT=0, or a file system
    that refuses O_DIRECT, writes buffered + fsync."""
    import os
    recs = recs if fill is not None else np.ascontiguousarray(recs, dtype=STATE_REC_DTYPE)
    n = int(recs.size)
    size = STATE_REC_DTYPE.itemsize
    direct = raw is not None and hasattr(os, "O_DIRECT") and os.getenv("MOBHEAT_CKPT_DIRECT", "1") != "0"
    head = json.dumps({"info": {k: int(info[k]) for k in _INFO_FIELDS}, "n": n,
                       "fields": list(STATE_REC_DTYPE.names), "itemsize": STATE_REC_DTYPE.itemsize,
                       "meta": meta}).encode()
    head += b" " * (-(len(head) + 16) % (4096 if direct else 64))
    header = STATE_FILE_MAGIC + len(head).to_bytes(8, "little") + head
    tmp = f"{path}.tmp{os.getpid()}"
    slices = _Slices(n, fill)
    try:
        if direct:
            try:
                _write_direct(tmp, header, raw, n * size, slices)
            except OSError as e:
                import errno
                if e.errno != errno.EINVAL:
                    raise
                direct = False   # (a file system without O_DIRECT: buffered below, the same bytes)
                head = head.rstrip(b" ")
                head += b" " * (-(len(head) + 16) % 64)
                header = STATE_FILE_MAGIC + len(head).to_bytes(8, "little") + head
        if not direct:
            with open(tmp, "wb") as f:
                f.write(header)
                body = memoryview(recs.view(np.uint8)) if n else None
                for lo, hi in slices:
                    f.write(body[lo * size:hi * size])
                f.flush()
                os.fsync(f.fileno())
    except BaseException:
        slices.close()
        try:
            os.remove(tmp)
        except OSError:
            pass
        raise
    slices.close()
    os.replace(tmp, path)
    return {"ckpt_copy_wait": slices.waited_ms, "ckpt_direct": float(direct)}


class _Slices:
    """The records in slices of SLICE records, in order: each yielded (lo, hi) once fill(lo, hi - lo) has landed it --
    a copier thread runs the fills ahead of the consumer (fill None: the records are in memory already)."""
    SLICE = 1 << 19   # (32 MiB of records: a multiple of 4 KiB)

    def __init__(self, n, fill):
        import threading
        self.bounds = [(lo, min(lo + self.SLICE, n)) for lo in range(0, n, self.SLICE)]
        self.fill = fill
        self.done = [threading.Event() for _ in self.bounds]
        self.err = None
        self.waited_ms = 0.0   # (the consumer's time blocked on slices not yet copied)
        self.stop = False
        self.thread = None
        if fill is not None and self.bounds:
            self.thread = threading.Thread(target=self._run, name="mobheat-export-copy", daemon=True)
            self.thread.start()

    def _run(self):
        try:
            for (lo, hi), ev in zip(self.bounds, self.done):
                if self.stop:
                    return
                self.fill(lo, hi - lo)
                ev.set()
        except BaseException as e:   # (handed to the consumer)
            self.err = e
        finally:
            for ev in self.done:
                ev.set()

    def __iter__(self):
        for (lo, hi), ev in zip(self.bounds, self.done):
            if self.thread is not None:
                if not ev.is_set():
                    import time
                    t = time.perf_counter()
                    ev.wait()
                    self.waited_ms += 1e3 * (time.perf_counter() - t)
                if self.err is not None:
                    raise self.err
            yield lo, hi

    def close(self):
        self.stop = True
        if self.thread is not None:
            self.thread.join()
            self.thread = None


def _write_direct(tmp, header, raw, nbytes, slices):
    """header + raw[:nbytes] to tmp with O_DIRECT writes (4-KiB aligned offsets, lengths and buffers: the last block
    zero-padded in raw, then the file truncated to its size) and one fsync (metadata only: the data went to the disk)."""
    import mmap
    import os
    fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC | os.O_DIRECT, 0o644)
    try:
        hb = mmap.mmap(-1, len(header))   # (page-aligned)
        hb.write(header)
        _pwrite_all(fd, memoryview(hb), 0)
        hb.close()
        off = len(header)
        mv = memoryview(raw)
        rec = STATE_REC_DTYPE.itemsize
        for lo, hi in slices:
            b0, b1 = lo * rec, hi * rec
            if b1 == nbytes and b1 % 4096:
                pad = -b1 % 4096
                raw[b1:b1 + pad] = 0
                b1 += pad
            _pwrite_all(fd, mv[b0:b1], off + b0)
        os.ftruncate(fd, off + nbytes)
        os.fsync(fd)
    finally:
        os.close(fd)


def _pwrite_all(fd, mv, off):
    import os
    done = 0
    while done < len(mv):
        k = os.pwrite(fd, mv[done:], off + done)
        if k <= 0:
            raise OSError("short O_DIRECT write")
        done += k


def _state_header(f, path):
    """The JSON header of a raw state file (f positioned at its start), or None for a legacy .npz file."""
    if f.read(8) != STATE_FILE_MAGIC:
        return None
    n = int.from_bytes(f.read(8), "little")
    h = json.loads(f.read(n))
    if h.get("itemsize") != STATE_REC_DTYPE.itemsize or h.get("fields") != list(STATE_REC_DTYPE.names):
        raise RuntimeError(f"{path}: state records of another layout")
    return h


def load_state_file(path):
    """(info, records) of a state file: the raw format, or the .npz files written before round 4."""
    with open(path, "rb") as f:
        h = _state_header(f, path)
        if h is not None:
            recs = np.fromfile(f, dtype=STATE_REC_DTYPE, count=h["n"])
            if recs.size != h["n"]:
                raise RuntimeError(f"{path}: truncated ({recs.size} of {h['n']} records)")
            return {k: int(h["info"][k]) for k in _INFO_FIELDS}, recs
    with np.load(path, allow_pickle=False) as z:
        vals = z["info"]
        recs = z["recs"]
    if vals.size != len(_INFO_FIELDS) or recs.dtype != STATE_REC_DTYPE:
        raise RuntimeError(f"{path}: not a mobheat state checkpoint")
    return {k: int(v) for k, v in zip(_INFO_FIELDS, vals)}, recs


def read_state_meta(path):
    """The `meta` string stored with a state file (None when it has none)."""
    with open(path, "rb") as f:
        h = _state_header(f, path)
        if h is not None:
            return h.get("meta")
    with np.load(path, allow_pickle=False) as z:
        return str(z["meta"]) if "meta" in z.files else None


def latlng_to_cell(lat, lon, res, device=0):
    """The reference UDF's arithmetic (h3.latlng_to_cell) for arrays, on the GPU. 0 = None."""
    lib = _lib.load()
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    lon = np.ascontiguousarray(lon, dtype=np.float64)
    out = np.empty(lat.size, dtype=np.uint64)
    check(lib.hm_latlng_to_cell(ptr(lat), ptr(lon), lat.size, int(res), HM_MEM_HOST, int(device), ptr(out)),
          None, "hm_latlng_to_cell")
    return out
