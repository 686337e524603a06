"""CPU: the kernels' numerics, executed on the host through libmobheat.so's self-test entry points.

1. hm::xld_* -- the integer emulation of upstream H3's x87 `long double` expressions -- must be bit-identical
   to real x87 arithmetic (oracle_ld_ops, compiled by gcc) for every op the kernels use.
2. The device latLngToCell code path, compiled for the host (host libm for sin/cos/acos/atan2/tan), must be
   bit-identical to the oracle at every resolution: this validates the kernel's port of the algorithm
   (operation order, tables, digit logic) independently of the GPU math library.
"""
import numpy as np
import pytest

OPS = {0: "a*M_PI_180", 1: "a*M_SQRT7", 2: "a*M_RSIN60", 3: "a+M_2PI", 4: "a-M_2PI", 5: "a-M_AP7_ROT", 6: "a+M_AP7_ROT"}


def _inputs(op):
    rng = np.random.default_rng(op)
    special = np.array([0.0, -0.0, 1.0, -1.0, 5e-324, -5e-324, 2.2250738585072014e-308, 1e-300, 1e-17, -1e-20,
                        np.pi, 2 * np.pi, -2 * np.pi, 6.283185307179586, 6.283185307179587, 0.3334731722518321,
                        180.0, -180.0, 90.0, -90.0, 1e300, np.inf, -np.inf, np.nan])
    # 2M uniform values put ~1000 exact products within 2^-12 ulp of a double-rounding midpoint, where the
    # fast path must round the tail to the 64-bit-mantissa grid correctly
    if op == 0:
        r = np.r_[rng.uniform(-180, 180, 2_000_000), rng.uniform(-1e-5, 1e-5, 20_000)]
    elif op in (1, 2):
        r = np.r_[rng.uniform(0, 3e6, 2_000_000), np.exp(rng.uniform(-700, 700, 20_000))]
    else:
        r = np.r_[rng.uniform(-7, 7, 2_000_000), rng.uniform(-1e-15, 1e-15, 20_000)]
    # values adjacent to representable neighbours of the constants
    return np.r_[special, r, np.nextafter(r[:1000], np.inf)]


@pytest.mark.parametrize("path", ["fast", "exact"])
@pytest.mark.parametrize("op", sorted(OPS))
def test_x87_emulation_bit_exact(oracle_h3, mobheat_lib, op, path):
    """fast = fp64 error-free path with exact fallback (what the kernels run); exact = 128-bit integer path."""
    from mobheat import _lib
    a = _inputs(op)
    got = _lib.ld_ops_selftest(a, op + (10 if path == "exact" else 0))
    exp = oracle_h3.ld_ops(a, op)
    same = (got.view(np.uint64) == exp.view(np.uint64)) | (np.isnan(got) & np.isnan(exp))
    assert same.all(), f"{OPS[op]}: {np.count_nonzero(~same)} mismatches, e.g. a={a[~same][:3]!r}"


@pytest.mark.parametrize("res", range(16))
def test_device_code_on_host_matches_oracle(oracle_h3, mobheat_lib, res):
    from mobheat import _lib, synth
    rng = np.random.default_rng(1000 + res)
    n = 30_000
    lat = np.r_[np.degrees(np.arcsin(rng.uniform(-1, 1, n))), synth.edge_points()[0]]
    lon = np.r_[rng.uniform(-180, 180, n), synth.edge_points()[1]]
    got = _lib.latlng_to_cell_host_selftest(lat, lon, res)
    exp = oracle_h3.latlng_to_cell(lat, lon, res)
    # the oracle returns a cell for any finite input; the UDF guard maps out-of-range rows to None (0)
    with np.errstate(invalid="ignore"):
        in_range = (lat >= -90) & (lat <= 90) & (lon >= -180) & (lon <= 180)
    exp = np.where(in_range, exp, 0)
    bad = got != exp
    assert not bad.any(), f"res {res}: {bad.sum()} mismatches at {list(zip(lat[bad][:3], lon[bad][:3]))}"
