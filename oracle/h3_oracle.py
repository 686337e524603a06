"""ORACLE -- test infrastructure only (never imported by the product path).

ctypes wrapper of oracle/libh3oracle.so, the C restatement of H3 v4 latLngToCell / cellToLatLng / cellToBoundary
(see h3_oracle.c for provenance).  Builds the library with `make -C oracle` when it is missing.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libh3oracle.so")
_lib = None


def build(force=False):
    srcs = ("h3_oracle.c", "h3_tables_oracle.h", "h3_tables_derive.c", "heatmap_cpu.c")
    if force or not os.path.exists(LIB) or any(os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, s)) for s in srcs):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        L.oracle_latlng_to_cell.restype = ctypes.c_uint64
        L.oracle_latlng_to_cell.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int]
        L.oracle_latlng_to_cell_batch.restype = None
        L.oracle_latlng_to_cell_batch.argtypes = [P, P, ctypes.c_int64, ctypes.c_int, P]
        L.oracle_latlng_to_cell_perturbed_batch.restype = None
        L.oracle_latlng_to_cell_perturbed_batch.argtypes = [P, P, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
        L.oracle_cell_to_latlng_batch.restype = None
        L.oracle_cell_to_latlng_batch.argtypes = [P, ctypes.c_int64, P, P]
        L.oracle_cell_to_boundary_batch.restype = None
        L.oracle_cell_to_boundary_batch.argtypes = [P, ctypes.c_int64, P, P, P]
        L.oracle_tables.restype = ctypes.c_int
        L.oracle_tables.argtypes = [P, P, P, ctypes.POINTER(ctypes.c_char_p)]
        L.oracle_latlng_to_cell_args_batch.restype = None
        L.oracle_latlng_to_cell_args_batch.argtypes = [P, P, ctypes.c_int64, ctypes.c_int, P]
        L.oracle_libm_batch.restype = None
        L.oracle_libm_batch.argtypes = [ctypes.c_int, P, P, ctypes.c_int64, P, P]
        L.oracle_ld_ops.restype = None
        L.oracle_ld_ops.argtypes = [P, ctypes.c_int64, ctypes.c_int, P]
        _lib = L
        tables()   # the tables are derived at load: fail loudly if a derivation check failed on this host
    return _lib


def latlng_to_cell(lat, lon, res):
    """h3.latlng_to_cell for arrays (degrees); 0 where h3 would fail (non-finite / bad res)."""
    L = load()
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    lon = np.ascontiguousarray(lon, dtype=np.float64)
    out = np.empty(lat.size, dtype=np.uint64)
    L.oracle_latlng_to_cell_batch(lat.ctypes.data, lon.ctypes.data, lat.size, int(res), out.ctypes.data)
    return out


LIBM_FNS = {"sincos": 0, "acos": 1, "atan2": 2, "tan": 3, "asin": 4, "atan": 5}


def libm(fn, a, b=None):
    """glibc's sincos (-> (sin, cos)), acos, atan2(a, b), tan, asin or atan of each element, through this process's libm."""
    L = load()
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
    out = np.empty(a.size)
    out2 = np.empty(a.size) if fn == "sincos" else None
    L.oracle_libm_batch(LIBM_FNS[fn], a.ctypes.data, None if b is None else b.ctypes.data, a.size, out.ctypes.data,
                        None if out2 is None else out2.ctypes.data)
    return (out, out2) if fn == "sincos" else out


def latlng_to_cell_args(lat, lon, res):
    """The arguments latLngToCell passes to glibc for each point: (n, 8) array -- sincos(lat), sincos(lng), acos,
    sincos(dlng), atan2 y, atan2 x, tan, sincos(theta); NaN where the call is not reached."""
    L = load()
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    lon = np.ascontiguousarray(lon, dtype=np.float64)
    out = np.empty((lat.size, 8))
    L.oracle_latlng_to_cell_args_batch(lat.ctypes.data, lon.ctypes.data, lat.size, int(res), out.ctypes.data)
    return out


N_LIBM_SITES = 11   # transcendental call sites of the forward path (h3_oracle.c PT)


def libm_alternatives(lat, lon, res, max_ulps=2):
    """[k, n] cells of latLngToCell with one transcendental call site's result moved by +-1..max_ulps ulps (k =
    N_LIBM_SITES * 2 * max_ulps): the cells another libm (last-bit differences) could make h3 return."""
    L = load()
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    lon = np.ascontiguousarray(lon, dtype=np.float64)
    alts = []
    for site in range(N_LIBM_SITES):
        for u in range(1, max_ulps + 1):
            for sg in (-1, 1):
                out = np.empty(lat.size, dtype=np.uint64)
                L.oracle_latlng_to_cell_perturbed_batch(lat.ctypes.data, lon.ctypes.data, lat.size, int(res), site, sg * u,
                                                       out.ctypes.data)
                alts.append(out)
    return np.stack(alts) if alts else np.empty((0, lat.size), np.uint64)


NEIGHBOURHOOD_ULPS = (-32, -16, -8, -4, -2, -1, 0, 1, 2, 4, 8, 16, 32)


def neighbourhood_cells(lat, lon, res, steps=NEIGHBOURHOOD_ULPS):
    """[k, n] cells of the inputs moved by (i, j) units in (lat, lon) for i, j in steps (k = len(steps)^2), a unit being
    one ulp of max(|coordinate|, 45) degrees (7.1e-15 degrees, ~1e-16 rad: the absolute scale of a last-bit error of
    sin/cos/atan2, whatever the coordinate's own magnitude): the cells whose boundary passes within a few such errors
    of the point -- where last-bit differences of the libm can land it."""
    lat = np.asarray(lat, dtype=np.float64)
    lon = np.asarray(lon, dtype=np.float64)
    ua, uo = np.spacing(np.maximum(np.abs(lat), 45.0)), np.spacing(np.maximum(np.abs(lon), 45.0))
    out = []
    for i in steps:
        for j in steps:
            out.append(latlng_to_cell(lat + i * ua, lon + j * uo, res))
    return np.stack(out)


def cell_to_latlng(cells):
    L = load()
    cells = np.ascontiguousarray(cells, dtype=np.uint64)
    la = np.empty(cells.size)
    lo = np.empty(cells.size)
    L.oracle_cell_to_latlng_batch(cells.ctypes.data, cells.size, la.ctypes.data, lo.ctypes.data)
    return la, lo


def cell_to_boundary(cells):
    """h3.cell_to_boundary for arrays of cells: (lat [n, 10], lng [n, 10], nverts [n]); nverts -1 = invalid."""
    L = load()
    cells = np.ascontiguousarray(cells, dtype=np.uint64)
    la = np.full((cells.size, 10), np.nan)
    lo = np.full((cells.size, 10), np.nan)
    nv = np.zeros(cells.size, np.int32)
    L.oracle_cell_to_boundary_batch(cells.ctypes.data, cells.size, la.ctypes.data, lo.ctypes.data, nv.ctypes.data)
    return la, lo, nv


def ld_ops(a, op):
    """x87 long-double reference for the kernels' emulation (op codes as hm_selftest_ld_ops)."""
    L = load()
    a = np.ascontiguousarray(a, dtype=np.float64)
    out = np.empty_like(a)
    L.oracle_ld_ops(a.ctypes.data, a.size, int(op), out.ctypes.data)
    return out


def tables():
    """The oracle's own derived res-0 tables (h3_tables_derive.c): (baseCellData [122, 7], faceIjkBaseCells
    [20, 3, 3, 3, 2], faceNeighbors [20, 4, 5]); raises if one of the derivation's checks failed."""
    L = load()
    bcd = np.zeros((122, 7), np.int32)
    fib = np.zeros((20, 3, 3, 3, 2), np.int32)
    fn = np.zeros((20, 4, 5), np.int32)
    err = ctypes.c_char_p()
    if L.oracle_tables(bcd.ctypes.data, fib.ctypes.data, fn.ctypes.data, ctypes.byref(err)) != 0:
        raise RuntimeError("oracle table derivation failed: " + err.value.decode())
    return bcd, fib, fn
