"""glibc's sincos / acos / atan2 / tan (the exact latLngToCell path) and asin / atan (cellToBoundary, with sincos and
atan2) as csrc/glibc_libm.h restates them, against the running glibc (oracle.h3_oracle.libm, the same libm the
reference's h3 calls: heatmap_stream.py:65-75, app.py:19-41).

Bar: bit-identical results.  Arguments: >= 1e7 per function over the domain latLngToCell uses (and beyond), plus the
exact arguments latLngToCell hands glibc for the constructed near-tie inputs of every resolution (cell vertices, edge
midpoints, icosahedron vertices, nudged by 1-8 ulp: tests/test_gpu_boundary.py), captured from the oracle."""
import numpy as np
import pytest

from mobheat import _lib
from oracle import h3_oracle

import test_gpu_boundary as near


def _args(seed, n):
    rng = np.random.default_rng(seed)
    q = n // 4
    sc = np.concatenate([rng.uniform(-2 * np.pi, 2 * np.pi, q), rng.uniform(-np.pi / 2, np.pi / 2, q),
                         rng.uniform(-3.2, 3.2, q), rng.uniform(-1e-2, 1e-2, q // 4), rng.uniform(-1e7, 1e7, q // 4),
                         np.ldexp(rng.uniform(0.5, 1, q // 8), rng.integers(-60, 0, q // 8))])
    ac = np.concatenate([rng.uniform(-1, 1, q), rng.uniform(0.79, 1, 2 * q), 1 - np.ldexp(rng.uniform(0, 1, q // 2),
                         rng.integers(-53, -5, q // 2)), np.array([1.0, -1.0, 0.0, -0.0, 0.5, 0.75, 0.96875])])
    tn = np.concatenate([rng.uniform(-0.786, 0.786, q), rng.uniform(0, 0.66, 2 * q), rng.uniform(-0.07, 0.07, q // 2),
                         np.ldexp(rng.uniform(0.5, 1, q // 8), rng.integers(-40, -1, q // 8))])
    m = 2 * q
    y = rng.standard_normal(m) * np.exp(rng.uniform(-8, 8, m))
    x = rng.standard_normal(m) * np.exp(rng.uniform(-8, 8, m))
    y[: m // 8] *= 1e-30   # the |y| << |x| and |x| << |y| branches
    x[m // 8: m // 4] *= 1e-30
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf])
    y = np.concatenate([y, np.repeat(sp, sp.size), rng.uniform(-1, 1, q)])
    x = np.concatenate([x, np.tile(sp, sp.size), rng.uniform(-1, 1, q)])
    return sc, ac, tn, y, x


def _args_boundary(seed, n):
    """asin over [-1, 1] (every interval of e_asin.c, the Taylor and tiny ranges, 1 - 2^-k), atan over every branch
    of s_atan.c (|x| < 2^-27 .. 1/16 .. 1 .. 16 .. E and beyond, +-0, +-inf)"""
    rng = np.random.default_rng(seed)
    q = n // 4
    asn = np.concatenate([rng.uniform(-1, 1, q), rng.uniform(0.9, 1, q), -rng.uniform(0.5, 1, q // 2),
                          1 - np.ldexp(rng.uniform(0, 1, q // 2), rng.integers(-53, -5, q // 2)), rng.uniform(-0.13, 0.13, q // 2),
                          np.ldexp(rng.uniform(0.5, 1, q // 4), rng.integers(-60, -2, q // 4)),
                          np.array([1.0, -1.0, 0.0, -0.0, 0.125, 0.25, 0.5, 0.75, 0.921875, 0.953125, 0.96875])])
    m = 2 * q
    atn = np.concatenate([rng.standard_normal(m) * np.exp(rng.uniform(-45, 45, m)), rng.uniform(-20, 20, q),
                          rng.uniform(-1, 1, q // 2), np.array([0.0, -0.0, np.inf, -np.inf, 1.0, -1.0, 16.0, 0.0625, 1e16])])
    return asn, atn


def _same(name, got, exp, args):
    g = np.asarray(got, np.float64).view(np.uint64)
    e = np.asarray(exp, np.float64).view(np.uint64)
    bad = np.nonzero(g != e)[0]
    assert bad.size == 0, f"{name}: {bad.size} of {g.size} differ, e.g. " + ", ".join(
        f"{tuple(float(a[i]).hex() for a in args)} -> {float(got[i]).hex()} vs {float(exp[i]).hex()}" for i in bad[:4])


def _check(fn, a, b=None, device=None):
    got = _lib.glibc_libm_selftest(fn, a, b, device=device)
    exp = h3_oracle.libm(fn, a, b)
    args = (a,) if b is None else (a, b)
    if fn == "sincos":
        _same("sin", got[0], exp[0], args)
        _same("cos", got[1], exp[1], args)
    else:
        _same(fn, got, exp, args)
    return a.size


def _near_tie_args():
    cols = []
    for res in range(16):
        lat, lon = near._near_tie_points(res)
        ok = (np.abs(lat) <= 90) & (np.abs(lon) <= 180)
        cols.append(h3_oracle.latlng_to_cell_args(lat[ok], lon[ok], res))
    A = np.concatenate(cols)
    sc = np.concatenate([A[:, 0], A[:, 1], A[:, 3], A[:, 7]])
    at = A[:, 4:6][~np.isnan(A[:, 4])]
    return (sc[~np.isnan(sc)], A[:, 2][~np.isnan(A[:, 2])], A[:, 6][~np.isnan(A[:, 6])], at[:, 0], at[:, 1])


def test_host_restatement_equals_glibc_1e7_per_function():
    sc, ac, tn, y, x = _args(7, 14_000_000)
    n = [_check("sincos", sc), _check("acos", ac), _check("tan", tn), _check("atan2", y, x)]
    asn, atn = _args_boundary(9, 14_000_000)
    n += [_check("asin", asn), _check("atan", atn)]
    assert min(n) >= 10_000_000, n


def test_host_restatement_equals_glibc_on_near_tie_arguments():
    sc, ac, tn, y, x = _near_tie_args()
    n = [_check("sincos", sc), _check("acos", ac), _check("tan", tn), _check("atan2", y, x)]
    print("near-tie arguments checked per function:", n)


def test_host_exact_path_equals_oracle_on_near_ties():
    """The whole exact latLngToCell path (fast path + exact fallback, executed on the host) on the constructed near-tie
    inputs of every resolution: cell ids identical to the glibc-linked oracle's."""
    for res in range(16):
        lat, lon = near._near_tie_points(res)
        ok = (np.abs(lat) <= 90) & (np.abs(lon) <= 180)
        got, fell_back = _lib.latlng_to_cell_fast_host_selftest(lat[ok], lon[ok], res)
        exact = _lib.latlng_to_cell_host_selftest(lat[ok], lon[ok], res)
        exp = h3_oracle.latlng_to_cell(lat[ok], lon[ok], res)
        assert np.array_equal(got, exp) and np.array_equal(exact, exp), res
        assert fell_back.any(), res


@pytest.mark.gpu
def test_device_restatement_equals_glibc():
    sc, ac, tn, y, x = _args(8, 14_000_000)
    asn, atn = _args_boundary(10, 14_000_000)
    for fn, a, b in [("sincos", sc, None), ("acos", ac, None), ("tan", tn, None), ("atan2", y, x), ("asin", asn, None),
                     ("atan", atn, None)]:
        _check(fn, a, b, device=0)
    sc, ac, tn, y, x = _near_tie_args()
    for fn, a, b in [("sincos", sc, None), ("acos", ac, None), ("tan", tn, None), ("atan2", y, x)]:
        _check(fn, a, b, device=0)
