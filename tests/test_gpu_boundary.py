"""GPU: row f4 (cellToBoundary, the read side of reference app.py:19-41) against the oracle, and latLngToCell on
constructed near-ties at every resolution (pentagon centres = icosahedron vertices, icosahedron
edge midpoints, face centres, cell centres, vertices and edge midpoints, each nudged by 1-8 ulp)."""
import numpy as np
import pytest

from mobheat import _lib
from oracle import h3_oracle

pytestmark = pytest.mark.gpu
PENTAGON_BASE_CELLS = [4, 14, 24, 38, 49, 58, 63, 72, 83, 97, 107, 117]
# boundary coordinates: bit-identical to the glibc-linked oracle's -- the kernel computes sincos/asin/atan2/atan as
# glibc's FMA variants do (csrc/glibc_libm.h), and upstream's long double constants with the x87 emulation


def _random_cells(res, n, seed):
    rng = np.random.default_rng(seed)
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, n)))
    lon = rng.uniform(-180, 180, n)
    return h3_oracle.latlng_to_cell(lat, lon, res)


@pytest.mark.parametrize("res", [0, 1, 2, 5, 7, 8, 9, 12, 15])
def test_cells_to_boundary_matches_oracle(res):
    from mobheat import readside
    cells = _random_cells(res, 100_000, res)
    base = np.array([(1 << 59) | (res << 52) | (bc << 45) | ((1 << (3 * (15 - res))) - 1) for bc in PENTAGON_BASE_CELLS],
                    np.uint64)   # the pentagons at this resolution (centre children of the 12 pentagon base cells)
    cells = np.concatenate([cells, base, np.array([0, 0x8a2a1072b59ffff | (1 << 63)], np.uint64)])
    la, lo, nv = readside.cells_to_boundary(cells)
    x, y, z = h3_oracle.cell_to_boundary(cells)
    z = np.maximum(z, 0)
    assert np.array_equal(nv, z)
    m = ~np.isnan(x)
    assert np.array_equal(np.isnan(la), np.isnan(x)) and np.array_equal(np.isnan(lo), np.isnan(y))
    bad = np.nonzero((la[m].view(np.uint64) != x[m].view(np.uint64)) | (lo[m].view(np.uint64) != y[m].view(np.uint64)))[0]
    print(f"res {res}: {cells.size} cells, {int(m.sum())} vertex coordinates, {bad.size} differ from the oracle")
    assert bad.size == 0, [(float(la[m][i]).hex(), float(x[m][i]).hex(), float(lo[m][i]).hex(), float(y[m][i]).hex())
                           for i in bad[:4]]


def test_boundary_geojson_ring_and_collection():
    import datetime
    from mobheat import readside
    ring = readside.h3_boundary_geojson("85283473fffffff")
    assert len(ring) == 7 and ring[0] == ring[-1]
    assert abs(ring[0][0] - -121.91508032705622) < 1e-12 and abs(ring[0][1] - 37.271355866731895) < 1e-12
    ws = datetime.datetime(2025, 10, 4, 10, 20)
    docs = [{"cellId": "882a1072b5fffff", "count": 3, "avgSpeedKmh": 12.5, "windowStart": ws,
             "windowEnd": ws + datetime.timedelta(minutes=5)}]
    fc = readside.tiles_latest_collection(docs)
    f = fc["features"][0]
    assert fc["type"] == "FeatureCollection" and f["geometry"]["type"] == "Polygon"
    assert f["properties"] == {"cellId": "882a1072b5fffff", "count": 3, "avgSpeedKmh": 12.5,
                               "windowStart": "2025-10-04T10:20:00", "windowEnd": "2025-10-04T10:25:00"}


def _nudged(lat, lon, k=8):
    """every point, and each moved by 1..k ulp up and down in lat, and in lon"""
    la, lo = [lat], [lon]
    for s in range(1, k + 1):
        for sg in (-1, 1):
            la.append(lat + sg * s * np.spacing(lat))
            lo.append(lon)
            la.append(lat)
            lo.append(lon + sg * s * np.spacing(lon))
    return np.concatenate(la), np.concatenate(lo)


def _near_tie_points(res):
    pent = np.array([(1 << 59) | (bc << 45) | ((1 << 45) - 1) for bc in PENTAGON_BASE_CELLS], np.uint64)
    plat, plon = h3_oracle.cell_to_latlng(pent)   # pentagon centres = the icosahedron's vertices
    v = np.stack([np.cos(np.radians(plat)) * np.cos(np.radians(plon)), np.cos(np.radians(plat)) * np.sin(np.radians(plon)),
                  np.sin(np.radians(plat))], 1)
    d = v @ v.T
    i, j = np.nonzero(np.triu(d > 0.4, 1))          # the 30 icosahedron edges (adjacent vertices)
    mid = v[i] + v[j]
    mid /= np.linalg.norm(mid, axis=1, keepdims=True)
    elat, elon = np.degrees(np.arcsin(mid[:, 2])), np.degrees(np.arctan2(mid[:, 1], mid[:, 0]))
    cells = _random_cells(res, 300, 1000 + res)
    clat, clon = h3_oracle.cell_to_latlng(cells)
    bla, blo, bnv = h3_oracle.cell_to_boundary(cells)
    vla = np.concatenate([bla[k, :bnv[k]] for k in range(cells.size)])
    vlo = np.concatenate([blo[k, :bnv[k]] for k in range(cells.size)])
    mla = np.concatenate([(bla[k, :bnv[k]] + np.roll(bla[k, :bnv[k]], -1)) / 2 for k in range(cells.size)])
    mlo = np.concatenate([(blo[k, :bnv[k]] + np.roll(blo[k, :bnv[k]], -1)) / 2 for k in range(cells.size)])
    lat = np.concatenate([plat, elat, clat, vla, mla])
    lon = np.concatenate([plon, elon, clon, vlo, mlo])
    return _nudged(lat, lon)


@pytest.mark.parametrize("res", range(16))
def test_latlng_to_cell_constructed_near_ties(res):
    """Bit-exact on knife-edge inputs: cell vertices, edge midpoints and icosahedron vertices,
    each nudged by 1-8 ulp, where the last bit of one transcendental decides the cell.  The fast path hands every
    input whose margins are below its error bound to the exact path, and the exact path evaluates upstream's sequence
    with glibc 2.35's own sincos/acos/atan2/tan restated for the device (csrc/glibc_libm.h; the routines the
    reference's h3 calls through the host libm, checked bit for bit by tests/test_glibc_libm.py), so the GPU's cell
    equals the glibc-linked oracle's on every input."""
    from mobheat import latlng_to_cell
    lat, lon = _near_tie_points(res)
    got = latlng_to_cell(lat, lon, res)
    n_exact = _lib.load().hm_latlng_to_cell_last_exact(0)
    exp = h3_oracle.latlng_to_cell(lat, lon, res)
    ok = (np.abs(lat) <= 90) & (np.abs(lon) <= 180)
    hf, fell_back = _lib.latlng_to_cell_fast_host_selftest(lat, lon, res)
    assert np.array_equal(hf[ok], exp[ok]), "host execution of the fast path + exact fallback differs from the oracle"
    diff = np.nonzero(ok & (got != exp))[0]
    assert diff.size == 0, [(lat[i].hex(), lon[i].hex(), hex(int(got[i])), hex(int(exp[i])), bool(fell_back[i]))
                            for i in diff[:5]]
    assert n_exact > 0, "no input reached the exact path"
    print(f"res {res}: {lat.size} near-tie inputs, {n_exact} through the exact path, 0 differences from the oracle")
