"""ctypes binding of libmobheat.so (C ABI declared in include/mobheat.h).

The library is built in-tree (``real-time-mobility-heatmap_amd/csrc/libmobheat.so``); there is no CPU fallback:
if it cannot be loaded, every entry point raises.  Negative return codes raise ``RuntimeError`` with the
library's message, which keeps the reference's fail-the-batch behaviour (reference heatmap_stream.py:192-235
has no try/except around the writes; any exception kills the streaming query at :249).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MOBHEAT_LIB: load another build of the same ABI (kernel variants under csrc/variants/ for tuning runs)
LIB_PATH = os.environ.get("MOBHEAT_LIB") or os.path.normpath(os.path.join(_HERE, "..", "csrc", "libmobheat.so"))

HM_ABI_VERSION = 11
HM_MEM_HOST = 0
HM_MEM_DEVICE = 1
HM_MEM_HOST_STREAM = 2
HM_JSON_SPLICE = 1
HM_E_INVALID, HM_E_HIP, HM_E_NOMEM, HM_E_OVERFLOW, HM_E_STATE, HM_E_UNSUPPORTED = -1, -2, -3, -4, -5, -6
HM_STAGE_SUMMARY_WORDS = 8200
HM_TILE_REC_BYTES = 48       # table mode's tile partial
HM_EVENT_REC_BYTES = 32      # direct path: one record per aggregated row
HM_CAND_REC_BYTES = 32

c_i32, c_i64, c_u64, c_dbl, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double, ctypes.c_void_p


class HmConfig(ctypes.Structure):
    _fields_ = [
        ("abi_version", c_i32), ("h3_res", c_i32), ("device", c_i32), ("late_uses_prev_watermark", c_i32),
        ("tile_us", c_i64), ("watermark_delay_ms", c_i64), ("state_capacity_hint", c_i64),
        ("batch_capacity_hint", c_i64), ("state_arena_bytes", c_i64), ("shard_rank", c_i32), ("shard_count", c_i32),
    ]


class HmBatchIn(ctypes.Structure):
    _fields_ = [
        ("n", c_i64), ("memory", c_i32), ("reserved", c_i32),
        ("lat", c_vp), ("lon", c_vp), ("ts_us", c_vp), ("speed", c_vp), ("speed_valid", c_vp),
        ("vkey", c_vp), ("row_valid", c_vp),
    ]


class HmBatchOut(ctypes.Structure):
    _fields_ = [
        ("n_tiles", c_i64), ("cell", c_vp), ("window_start_us", c_vp), ("count", c_vp), ("avg_speed", c_vp),
        ("speed_null", c_vp), ("avg_lon", c_vp), ("avg_lat", c_vp),
        ("n_latest", c_i64), ("latest_row", c_vp),
        ("n_in", c_i64), ("n_valid", c_i64), ("n_late", c_i64), ("n_state", c_i64),
        ("batch_max_event_ms", c_i64), ("watermark_ms", c_i64), ("late_watermark_ms", c_i64), ("n_partials", c_i64),
    ]


class HmJsonIn(ctypes.Structure):
    _fields_ = [("n", c_i64), ("memory", c_i32), ("flags", c_i32), ("bytes", c_vp), ("offsets", c_vp)]


class HmJsonOut(ctypes.Structure):
    _fields_ = [("batch", HmBatchIn), ("n_providers", c_i64), ("provider_offsets", c_vp), ("provider_bytes", c_vp),
                ("n_vehicles", c_i64), ("vehicle_offsets", c_vp), ("vehicle_bytes", c_vp), ("n_malformed", c_i64),
                ("n_unsupported", c_i64), ("unsupported_rows", c_vp)]


class HmArrowCol(ctypes.Structure):
    _fields_ = [("values", c_vp), ("data", c_vp), ("validity", c_vp), ("validity_offset", c_i64), ("offset_bytes", c_i32),
                ("unit", c_i32)]


class HmArrowIn(ctypes.Structure):
    _fields_ = [("n", c_i64), ("lat", HmArrowCol), ("lon", HmArrowCol), ("speed", HmArrowCol), ("ts_us", HmArrowCol),
                ("provider", HmArrowCol), ("vehicle", HmArrowCol)]


class HmStageSizes(ctypes.Structure):
    _fields_ = [("table_mode", c_i64), ("n_tile_records", c_i64), ("n_cands", c_i64), ("global_batch_max_event_ms", c_i64),
                ("n_valid", c_i64), ("n_late", c_i64), ("n_self_records", c_i64)]


class HmStateInfo(ctypes.Structure):
    _fields_ = [("epoch_id", c_i64), ("n_keys", c_i64), ("watermark_ms", c_i64), ("prev_watermark_ms", c_i64),
                ("tile_us", c_i64), ("watermark_delay_ms", c_i64), ("h3_res", c_i32), ("reserved", c_i32)]


class HmTileDocCfg(ctypes.Structure):
    _fields_ = [("city", ctypes.c_char_p), ("city_len", c_i32), ("reserved", c_i32), ("ttl_ms", c_i64),
                ("n_windows", c_i64), ("window_start_us", c_vp), ("start_offset_s", c_vp), ("end_offset_s", c_vp)]


class HmPositionDocCfg(ctypes.Structure):
    _fields_ = [("n_providers", c_i64), ("provider_offsets", c_vp), ("provider_bytes", c_vp),
                ("n_vehicles", c_i64), ("vehicle_offsets", c_vp), ("vehicle_bytes", c_vp),
                ("n_buckets", c_i64), ("bucket_ids", c_vp), ("bucket_offset_s", c_vp)]


# hm_state_rec (64 B): one live (cellId, windowStart) key of the tile state
STATE_REC_DTYPE = np.dtype([("cell", "<u8"), ("window_start_us", "<i8"), ("count", "<i8"), ("n_speed", "<i8"),
                            ("sum_speed", "<f8"), ("sum_lat", "<f8"), ("sum_lon", "<f8"), ("reserved", "<i8")])
assert STATE_REC_DTYPE.itemsize == 64

_P = ctypes.POINTER
# name -> (restype, argtypes); must match include/mobheat.h (tests/test_abi.py checks the symbol set)
SIGNATURES = {
    "hm_create": (c_i32, [_P(HmConfig), _P(c_vp)]),
    "hm_destroy": (None, [c_vp]),
    "hm_last_error": (ctypes.c_char_p, [c_vp]),
    "hm_process_batch": (c_i32, [c_vp, c_i64, _P(HmBatchIn), c_i32, _P(HmBatchOut)]),
    "hm_latlng_to_cell": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp]),
    "hm_stage_ingest": (c_i32, [c_vp, c_i64, _P(HmBatchIn), c_i32, c_i32, c_vp]),
    "hm_stage_send_capacity": (c_i64, [c_i64, c_i32]),
    "hm_stage_send": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_vp, _P(HmStageSizes)]),
    "hm_stage_merge": (c_i32, [c_vp, c_vp, c_vp, c_i32, _P(HmBatchOut), c_vp, c_i64, c_vp]),
    "hm_stage_finish": (c_i32, [c_vp, c_vp, c_i64, c_i32, _P(HmBatchOut)]),
    "hm_stream_wait": (c_i32, [c_vp, c_vp]),
    "hm_device_memory": (c_i32, [c_i32, _P(c_i64), _P(c_i64)]),
    "hm_device_alloc": (c_i32, [c_i32, c_i64, _P(c_vp)]),
    "hm_device_free": (c_i32, [c_i32, c_vp]),
    "hm_host_alloc": (c_i32, [c_i64, _P(c_vp)]),
    "hm_host_free": (c_i32, [c_vp]),
    "hm_memcpy": (c_i32, [c_vp, c_vp, c_i64, c_i32]),
    "hm_selftest_ld_ops": (c_i32, [c_vp, c_i64, c_i32, c_vp]),
    "hm_selftest_floor_div": (c_i32, [c_vp, c_i64, c_i64, c_vp]),
    "hm_selftest_latlng_to_cell_host": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_vp]),
    "hm_selftest_latlng_to_cell_fast_host": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp]),
    "hm_selftest_glibc_libm_host": (c_i32, [c_i32, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "hm_selftest_glibc_libm_device": (c_i32, [c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_i32]),
    "hm_state_export": (c_i32, [c_vp, _P(HmStateInfo), c_vp, c_i64]),
    "hm_state_export_touched": (c_i32, [c_vp, _P(HmStateInfo), c_vp, c_i64, c_vp]),
    "hm_state_export_begin": (c_i32, [c_vp, _P(HmStateInfo), c_i32, c_vp]),
    "hm_state_export_copy": (c_i32, [c_vp, c_vp, c_i64, c_i64]),
    "hm_state_export_copy_async": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i32]),
    "hm_state_export_copy_wait": (c_i32, [c_vp, c_i32]),
    "hm_state_version": (c_i64, [c_vp]),
    "hm_state_import": (c_i32, [c_vp, _P(HmStateInfo), c_vp]),
    "hm_last_windows": (c_i32, [c_vp, c_vp, c_i64, _P(c_i64)]),
    "hm_encode_tile_updates": (c_i32, [c_vp, _P(HmTileDocCfg), c_i32, _P(c_vp), _P(c_vp), _P(c_i64)]),
    "hm_selftest_tile_statements": (c_i32, [_P(HmTileDocCfg), c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                            c_i64, c_vp, c_i64, c_vp]),
    "hm_encode_position_updates": (c_i32, [c_vp, _P(HmPositionDocCfg), c_i32, _P(c_vp), _P(c_vp), _P(c_i64)]),
    "hm_statements_wait": (c_i32, [c_vp, c_i64]),
    "hm_selftest_position_statements": (c_i32, [_P(HmPositionDocCfg), c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64,
                                                c_vp]),
    "hm_last_timings": (c_i32, [c_vp, c_vp, c_i32]),
    "hm_last_counts": (c_i32, [c_vp, c_vp, c_i32]),
    "hm_decode_json": (c_i32, [c_vp, _P(HmJsonIn), _P(HmJsonOut)]),
    "hm_arrow_columns": (c_i32, [c_vp, _P(HmArrowIn), _P(HmJsonOut)]),
    "hm_json_patch": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64]),
    "hm_latlng_to_cell_last_exact": (c_i64, [c_i32]),
    "hm_cells_to_boundary": (c_i32, [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp]),
    "hm_selftest_cells_to_boundary_host": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_vp]),
    "hm_last_latest_buckets": (c_i32, [c_vp, c_vp, c_i64, _P(c_i64)]),
    "hm_selftest_json_records": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                         c_vp, c_vp]),
    "hm_selftest_decimal_to_double": (c_i32, [c_vp, c_vp, c_i64, c_vp]),
    "hm_abi_version": (c_i32, []),
}

_lib = None


def load():
    """Load libmobheat.so (raises if it is missing: the product path never falls back to the CPU)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libmobheat.so not built at {LIB_PATH}; run __graft_entry__.build() (or make -C csrc)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.hm_abi_version() != HM_ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH} was built for ABI {lib.hm_abi_version()}, this binding is ABI {HM_ABI_VERSION}: "
                           "rebuild it (__graft_entry__.build())")
    _lib = lib
    return lib


class MobheatError(RuntimeError):
    """A failed library call: `code` is the C-ABI error code (HM_E_*)."""

    def __init__(self, msg, code):
        super().__init__(msg)
        self.code = code


def check(rc, ctx=None, what="mobheat"):
    if rc < 0:
        lib = load()
        msg = lib.hm_last_error(ctx)
        raise MobheatError(f"{what} failed ({rc}): {msg.decode() if msg else ''}", rc)
    return rc


def ptr(a):
    """Address of a contiguous numpy array (or None)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays must be contiguous"
    return a.ctypes.data


def ld_ops_selftest(a, op):
    """Host execution of the kernels' x87 emulation (see hm_selftest_ld_ops)."""
    lib = load()
    a = np.ascontiguousarray(a, dtype=np.float64)
    out = np.empty_like(a)
    check(lib.hm_selftest_ld_ops(ptr(a), a.size, op, ptr(out)))
    return out


def floor_div_selftest(t, d):
    """Host execution of k_ingest's window division floor(t / d) (kernels.h FloorDiv)."""
    lib = load()
    t = np.ascontiguousarray(t, dtype=np.int64)
    out = np.empty_like(t)
    check(lib.hm_selftest_floor_div(ptr(t), t.size, int(d), ptr(out)))
    return out


def latlng_to_cell_host_selftest(lat, lon, res):
    """Host execution of the device exact latLngToCell path (glibc's routines as restated in glibc_libm.h)."""
    lib = load()
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    lon = np.ascontiguousarray(lon, dtype=np.float64)
    out = np.empty(lat.size, dtype=np.uint64)
    check(lib.hm_selftest_latlng_to_cell_host(ptr(lat), ptr(lon), lat.size, res, ptr(out)))
    return out


GLIBC_FNS = {"sincos": 0, "acos": 1, "atan2": 2, "tan": 3, "asin": 4, "atan": 5}


def glibc_libm_selftest(fn, a, b=None, device=None):
    """glibc's sincos (-> (sin, cos)) / acos / atan2(a, b) / tan / asin / atan as csrc/glibc_libm.h restates them, executed on the
    host (device=None) or on GPU `device`."""
    lib = load()
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
    out = np.empty(a.size)
    out2 = np.empty(a.size) if fn == "sincos" else None
    args = (GLIBC_FNS[fn], ptr(a), None if b is None else ptr(b), a.size, ptr(out), None if out2 is None else ptr(out2))
    if device is None:
        check(lib.hm_selftest_glibc_libm_host(*args))
    else:
        check(lib.hm_selftest_glibc_libm_device(*args, int(device)))
    return (out, out2) if fn == "sincos" else out


def latlng_to_cell_fast_host_selftest(lat, lon, res):
    """Host execution of the kernels' fast path + exact fallback; returns (cells, fell_back mask)."""
    lib = load()
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    lon = np.ascontiguousarray(lon, dtype=np.float64)
    out = np.empty(lat.size, dtype=np.uint64)
    fb = np.empty(lat.size, dtype=np.uint8)
    check(lib.hm_selftest_latlng_to_cell_fast_host(ptr(lat), ptr(lon), lat.size, res, ptr(out), ptr(fb)))
    return out, fb.astype(bool)


def local_offsets_s(window_start_us, tile_us):
    """Local-time offsets (s) at each window's start and end, as the reference's datetimes carry them: pyspark's
    TimestampType.fromInternal gives naive local wall times (datetime.fromtimestamp), which bson then encodes as
    if they were UTC (reference heatmap_stream.py:166-177 via stream._spark_datetime)."""
    import calendar
    import datetime as _dt

    def off(us):
        s = int(us) // 1_000_000
        return calendar.timegm(_dt.datetime.fromtimestamp(s).timetuple()) - s
    ws = np.ascontiguousarray(window_start_us, dtype=np.int64)
    return (np.array([off(w) for w in ws], np.int64), np.array([off(w + tile_us) for w in ws], np.int64))


def tile_doc_cfg(city, ttl_minutes, window_start_us, tile_us):
    """hm_tile_doc_cfg for the given windows; the returned tuple keeps the arrays alive."""
    cb = city.encode("utf-8")
    ws = np.ascontiguousarray(window_start_us, dtype=np.int64)
    so, eo = local_offsets_s(ws, tile_us)
    cfg = HmTileDocCfg(city=cb, city_len=len(cb), ttl_ms=int(ttl_minutes) * 60_000, n_windows=ws.size,
                       window_start_us=ptr(ws), start_offset_s=ptr(so), end_offset_s=ptr(eo))
    return cfg, (cb, ws, so, eo)


def tile_statements_selftest(tiles, city, h3_res, ttl_minutes, tile_us):
    """Host execution of the GPU statement encoder on a TileRows (no GPU): (bytes uint8, offsets int64)."""
    lib = load()
    n = len(tiles)
    wins = np.unique(tiles.window_start_us) if n else np.zeros(1, np.int64)
    cfg, keep = tile_doc_cfg(city, ttl_minutes, wins, tile_us)
    cap = (600 + 3 * len(city.encode("utf-8"))) * max(n, 1)   # (the city is in q._id, $set._id and $set.city)
    buf = np.zeros(cap, np.uint8)
    offs = np.zeros(n + 1, np.int64)
    a = [np.ascontiguousarray(x) for x in (tiles.cell.astype(np.uint64), tiles.window_start_us.astype(np.int64),
                                           tiles.count.astype(np.int64), tiles.avg_speed.astype(np.float64),
                                           tiles.speed_null.astype(np.uint8), tiles.avg_lon.astype(np.float64),
                                           tiles.avg_lat.astype(np.float64))]
    check(lib.hm_selftest_tile_statements(ctypes.byref(cfg), int(h3_res), int(tile_us), *[ptr(x) for x in a], n,
                                          ptr(buf), cap, ptr(offs)), None, "hm_selftest_tile_statements")
    return buf[:offs[-1]].copy(), offs


def _dictionary(strings):
    """(n, offsets int64[n+1], bytes) of a list of str or an Arrow string array, UTF-8 (Arrow's string layout)."""
    import pyarrow as pa
    if isinstance(strings, pa.ChunkedArray):
        strings = strings.combine_chunks()
    arr = strings.cast(pa.large_string()) if isinstance(strings, pa.Array) else pa.array(list(strings), type=pa.large_string())
    n = len(arr)
    offs = np.frombuffer(arr.buffers()[1], dtype=np.int64, count=n + 1, offset=arr.offset * 8).copy() if n else np.zeros(1, np.int64)
    offs -= offs[0]
    data = arr.buffers()[2]
    raw = np.frombuffer(data, dtype=np.uint8).copy() if data is not None and offs[-1] else np.zeros(1, np.uint8)
    return n, offs, raw


def time_buckets(ts_us, bucket_ids=None):
    """The distinct 900-s buckets floor(ts_s / 900) of the rows' eventTs (ascending; or the given bucket_ids) and the
    local-time offset of each (pyspark's naive local datetimes, stream._spark_datetime).  Only the buckets the rows
    use are looked up, so a batch mixing a 1970 GPS time with current traffic costs two lookups, not 55 years of
    buckets."""
    import calendar
    import datetime as _dt
    if bucket_ids is not None:
        ids = np.unique(np.asarray(bucket_ids, dtype=np.int64))
    else:
        ts_us = np.asarray(ts_us, dtype=np.int64)
        ids = np.unique(np.floor_divide(np.floor_divide(ts_us, 1_000_000), 900)) if ts_us.size else np.zeros(0, np.int64)

    def off(s):
        return calendar.timegm(_dt.datetime.fromtimestamp(s).timetuple()) - s
    offs = np.array([off(int(b) * 900) for b in ids], np.int64)
    if any(off(int(b) * 900 + 899) != o for b, o in zip(ids, offs)):
        raise RuntimeError("a local-time offset change inside a 900-s bucket")
    return np.ascontiguousarray(ids, np.int64), offs


def position_doc_cfg(provider_uniques, vehicle_uniques, ts_us, bucket_ids=None):
    """hm_position_doc_cfg for a batch's string dictionaries (pandas.factorize uniques in the order the vkeys were
    built, or (n, offsets, bytes) as decode_json returns them) and the eventTs of its latest rows (or their 900-s
    buckets); the returned tuple keeps the arrays alive."""
    np_, po, pb = provider_uniques if isinstance(provider_uniques, tuple) else _dictionary(provider_uniques)
    nv, vo, vb = vehicle_uniques if isinstance(vehicle_uniques, tuple) else _dictionary(vehicle_uniques)
    bi, bo = time_buckets(ts_us, bucket_ids)
    cfg = HmPositionDocCfg(n_providers=np_, provider_offsets=ptr(po), provider_bytes=ptr(pb), n_vehicles=max(nv, 1),
                           vehicle_offsets=ptr(vo), vehicle_bytes=ptr(vb), n_buckets=bi.size,
                           bucket_ids=ptr(bi) if bi.size else None, bucket_offset_s=ptr(bo) if bo.size else None)
    if nv == 0:   # (no valid row: an empty dictionary of one empty string keeps the offsets well formed)
        vo2 = np.zeros(2, np.int64)
        cfg.vehicle_offsets = ptr(vo2)
        return cfg, (po, pb, vo, vb, bi, bo, vo2)
    return cfg, (po, pb, vo, vb, bi, bo)


def position_statements_selftest(provider_uniques, vehicle_uniques, vkey, ts_us, lat, lon):
    """Host execution of the GPU positions encoder on rows (no GPU): (bytes uint8, offsets int64)."""
    lib = load()
    vkey = np.ascontiguousarray(vkey, dtype=np.uint64)
    ts_us = np.ascontiguousarray(ts_us, dtype=np.int64)
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    lon = np.ascontiguousarray(lon, dtype=np.float64)
    n = vkey.size
    cfg, keep = position_doc_cfg(provider_uniques, vehicle_uniques, ts_us)
    cap = 1024 * max(n, 1) + 8 * int(keep[1].size + keep[3].size)
    buf = np.zeros(cap, np.uint8)
    offs = np.zeros(n + 1, np.int64)
    check(lib.hm_selftest_position_statements(ctypes.byref(cfg), ptr(vkey), ptr(ts_us), ptr(lat), ptr(lon), n, ptr(buf),
                                              cap, ptr(offs)), None, "hm_selftest_position_statements")
    return buf[:offs[-1]].copy(), offs


# ---- Kafka values (row f1) ----
JF = dict(LAT=1, LON=2, SPEED=4, TS=8, PROV=16, VEH=32, BEARING=64, ACC=128, PROV_ESC=256, VEH_ESC=512,
          MALFORMED=1 << 16, UNSUPPORTED=1 << 17)   # json_decode.h


def pack_values(values):
    """A list of bytes (Kafka values) -> (bytes uint8 with 16 spare bytes, offsets int64[n+1]) in Arrow's layout."""
    lens = np.fromiter((len(v) for v in values), dtype=np.int64, count=len(values))
    offs = np.zeros(len(values) + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    buf = np.zeros(int(offs[-1]) + 16, np.uint8)
    if len(values):
        buf[:offs[-1]] = np.frombuffer(b"".join(values), np.uint8)
    return buf, offs


def json_records_selftest(values):
    """Host execution of the device record decoder (json_decode.h): per-record fields + decoded strings."""
    lib = load()
    buf, offs = pack_values(values)
    n = len(values)
    scratch = np.zeros_like(buf)
    o = {k: np.zeros(max(n, 1), dt) for k, dt in (("lat", np.float64), ("lon", np.float64), ("speed", np.float64),
                                                  ("ts_us", np.int64), ("bearing", np.int32), ("accuracy", np.int32),
                                                  ("p_off", np.int64), ("p_len", np.int32), ("v_off", np.int64),
                                                  ("v_len", np.int32), ("flags", np.uint32))}
    check(lib.hm_selftest_json_records(ptr(buf), ptr(offs), n, ptr(scratch), *[ptr(o[k]) for k in
                                       ("lat", "lon", "speed", "ts_us", "bearing", "accuracy", "p_off", "p_len", "v_off",
                                        "v_len", "flags")]), None, "hm_selftest_json_records")
    o = {k: v[:n] for k, v in o.items()}

    def strs(off, ln, esc_bit, present_bit):
        out = []
        for k in range(n):
            if not o["flags"][k] & present_bit:
                out.append(None)
                continue
            src = scratch if o["flags"][k] & esc_bit else buf
            out.append(bytes(src[o[off][k]:o[off][k] + o[ln][k]]))
        return out
    o["provider"] = strs("p_off", "p_len", JF["PROV_ESC"], JF["PROV"])
    o["vehicleId"] = strs("v_off", "v_len", JF["VEH_ESC"], JF["VEH"])
    return o


def decimal_to_double_selftest(w, q):
    lib = load()
    w = np.ascontiguousarray(w, dtype=np.uint64)
    q = np.ascontiguousarray(q, dtype=np.int64)
    out = np.empty(w.size, np.uint64)
    check(lib.hm_selftest_decimal_to_double(ptr(w), ptr(q), w.size, ptr(out)), None, "hm_selftest_decimal_to_double")
    return out


def cells_to_boundary_host_selftest(cells):
    """Host execution of the device cellToBoundary: (lat [n, 10], lng [n, 10], nverts [n])."""
    lib = load()
    cells = np.ascontiguousarray(cells, dtype=np.uint64)
    la = np.empty((cells.size, 10))
    lo = np.empty((cells.size, 10))
    nv = np.empty(cells.size, np.int32)
    check(lib.hm_selftest_cells_to_boundary_host(ptr(cells), cells.size, ptr(la), ptr(lo), ptr(nv)), None,
          "hm_selftest_cells_to_boundary_host")
    return la, lo, nv
