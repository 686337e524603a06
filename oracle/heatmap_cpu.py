"""ORACLE -- test infrastructure only (bench.py's cpu_baseline leg and tests/; never imported by the product path).

ctypes wrapper of oracle/heatmap_cpu.c: the whole micro-batch of the reference's Spark plan (filter, latLngToCell,
window, watermark, update-mode aggregation, eviction, latest rows per vehicle) as multi-threaded C (OpenMP), with
oracle/spark_oracle.py's semantics (tests/test_cpu_restatement.py).
"""
import ctypes

import numpy as np

from . import h3_oracle

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_bound = False


def _lib():
    global _bound
    L = h3_oracle.load()
    if not _bound:
        L.hmcpu_create.restype = _P
        L.hmcpu_create.argtypes = [ctypes.c_int, _I64, _I64]
        L.hmcpu_destroy.argtypes = [_P]
        L.hmcpu_process.restype = ctypes.c_int
        L.hmcpu_process.argtypes = [_P, _I64, _P, _P, _P, _P, _P, _P, _P, ctypes.c_int]
        L.hmcpu_n_tiles.restype = _I64
        L.hmcpu_n_tiles.argtypes = [_P]
        L.hmcpu_tiles.argtypes = [_P] + [_P] * 7
        L.hmcpu_n_latest.restype = _I64
        L.hmcpu_n_latest.argtypes = [_P]
        L.hmcpu_latest.argtypes = [_P, _P]
        L.hmcpu_stats.argtypes = [_P, _P]
        _bound = True
    return L


def _ptr(a):
    return None if a is None else a.ctypes.data


class CpuHeatmap:
    """One stream's state; process_batch returns the batch's tiles (arrays, unordered), latest rows and stats."""

    def __init__(self, h3_res=8, tile_minutes=5, watermark_delay_ms=600_000, threads=0):
        self.L = _lib()
        self.threads = int(threads)
        self.h = self.L.hmcpu_create(int(h3_res), int(tile_minutes) * 60_000_000, int(watermark_delay_ms))
        if not self.h:
            raise MemoryError("hmcpu_create")

    def close(self):
        if self.h:
            self.L.hmcpu_destroy(self.h)
            self.h = None

    __del__ = close

    def process_batch(self, lat, lon, ts_us, speed=None, speed_valid=None, vkey=None, row_valid=None, arrays=True):
        lat = np.ascontiguousarray(lat, np.float64)
        lon = np.ascontiguousarray(lon, np.float64)
        ts = np.ascontiguousarray(ts_us, np.int64)
        sp = None if speed is None else np.ascontiguousarray(speed, np.float64)
        sv = None if speed is None or speed_valid is None else np.ascontiguousarray(speed_valid, np.uint8)
        vk = None if vkey is None else np.ascontiguousarray(vkey, np.uint64)
        rv = None if row_valid is None else np.ascontiguousarray(row_valid, np.uint8)
        rc = self.L.hmcpu_process(self.h, lat.size, _ptr(lat), _ptr(lon), _ptr(ts), _ptr(sp), _ptr(sv), _ptr(vk), _ptr(rv),
                                  self.threads)
        if rc:
            raise MemoryError("hmcpu_process")
        if not arrays:
            return None
        m = self.L.hmcpu_n_tiles(self.h)
        t = dict(cell=np.empty(m, np.uint64), window_start_us=np.empty(m, np.int64), count=np.empty(m, np.int64),
                 avg_speed=np.empty(m), speed_null=np.empty(m, np.uint8), avg_lat=np.empty(m), avg_lon=np.empty(m))
        self.L.hmcpu_tiles(self.h, *(t[k].ctypes.data for k in ("cell", "window_start_us", "count", "avg_speed",
                                                                "speed_null", "avg_lat", "avg_lon")))
        latest = np.empty(self.L.hmcpu_n_latest(self.h), np.int64)
        self.L.hmcpu_latest(self.h, latest.ctypes.data)
        st = np.empty(6, np.int64)
        self.L.hmcpu_stats(self.h, st.ctypes.data)
        return dict(tiles=t, latest_rows=latest, n_valid=int(st[0]), n_late=int(st[1]), batch_max_event_ms=int(st[2]),
                    watermark_ms=int(st[3]), late_watermark_ms=int(st[4]), n_state=int(st[5]))
