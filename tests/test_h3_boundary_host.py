"""CPU: row f4's cellToBoundary (csrc/h3_boundary.h, the read side of reference app.py:19-41) executed on the host
against the oracle's restatement (oracle/h3_oracle.c oracle_cell_to_boundary), and the oracle against a published
example.  The kernel's sincos/asin/atan2/atan are glibc's routines restated (csrc/glibc_libm.h), so its host execution
equals the glibc-linked oracle bit for bit -- and so does the GPU (tests/test_gpu_boundary.py)."""
import numpy as np
import pytest

from mobheat import _lib
from oracle import h3_oracle

PENTAGON_BASE_CELLS = [4, 14, 24, 38, 49, 58, 63, 72, 83, 97, 107, 117]


def _cells_near_pentagons(res, rng, per=200):
    """cells around the 12 pentagons at `res` (pentagon centres, their distortion-vertex neighbours)"""
    base = np.array([(1 << 59) | (bc << 45) | ((1 << 45) - 1) for bc in PENTAGON_BASE_CELLS], np.uint64)
    clat, clon = h3_oracle.cell_to_latlng(base)
    lat = np.repeat(clat, per) + rng.normal(0, 3.0 * 7 ** (-res / 2), per * 12)
    lon = np.repeat(clon, per) + rng.normal(0, 3.0 * 7 ** (-res / 2), per * 12)
    lat = np.clip(lat, -90, 90)
    lon = (lon + 180) % 360 - 180
    return np.unique(h3_oracle.latlng_to_cell(lat, lon, res))


def test_oracle_boundary_known_answer():
    """cellToBoundary(0x85283473fffffff) as the H3 documentation prints it (recalled; the docs' build rounds a few
    last bits differently, hence the 1e-12 degree bar), and the pentagon/distortion vertex counts of H3."""
    exp = [(37.271355866731895, -121.91508032705622), (37.353926450852256, -121.86222328902491),
           (37.42834118609435, -121.9235499963016), (37.42012867767778, -122.0377349642703),
           (37.33755608435298, -122.09042892904395), (37.26319797461824, -122.02910130919)]
    la, lo, nv = h3_oracle.cell_to_boundary(np.array([0x85283473fffffff], np.uint64))
    assert nv[0] == 6
    assert np.allclose(la[0, :6], [e[0] for e in exp], rtol=0, atol=1e-12)
    assert np.allclose(lo[0, :6], [e[1] for e in exp], rtol=0, atol=1e-12)
    # res-0 pentagons: 5 vertices; res-1 pentagons (Class III): 10 (each edge crosses an icosahedron edge)
    _, _, nv0 = h3_oracle.cell_to_boundary(np.array([(1 << 59) | (4 << 45) | ((1 << 45) - 1)], np.uint64))
    _, _, nv1 = h3_oracle.cell_to_boundary(np.array([(1 << 59) | (1 << 52) | (4 << 45) | ((1 << 42) - 1)], np.uint64))
    assert nv0[0] == 5 and nv1[0] == 10


@pytest.mark.parametrize("res", range(16))
def test_host_boundary_equals_oracle(res):
    rng = np.random.default_rng(100 + res)
    n = 4000
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, n)))
    lon = rng.uniform(-180, 180, n)
    cells = np.concatenate([h3_oracle.latlng_to_cell(lat, lon, res), _cells_near_pentagons(res, rng)])
    a, b, c = _lib.cells_to_boundary_host_selftest(cells)
    x, y, z = h3_oracle.cell_to_boundary(cells)
    assert np.array_equal(c, z)
    assert np.array_equal(a.view(np.uint64)[~np.isnan(x)], x.view(np.uint64)[~np.isnan(x)])
    assert np.array_equal(b.view(np.uint64)[~np.isnan(y)], y.view(np.uint64)[~np.isnan(y)])
    assert set(np.unique(c)) <= {5, 6, 7, 8, 9, 10}


def test_boundary_vertices_surround_the_centre():
    """Each cell's vertices, pulled 1e-6 of the way towards its centre, index back into the cell."""
    rng = np.random.default_rng(7)
    for res in (3, 8, 12):
        lat = np.degrees(np.arcsin(rng.uniform(-1, 1, 2000)))
        lon = rng.uniform(-180, 180, 2000)
        cells = h3_oracle.latlng_to_cell(lat, lon, res)
        clat, clon = h3_oracle.cell_to_latlng(cells)
        la, lo, nv = h3_oracle.cell_to_boundary(cells)
        for k in range(cells.size):
            if abs(clat[k]) > 80:
                continue
            for v in range(nv[k]):
                dl = ((lo[k, v] - clon[k] + 180) % 360) - 180
                p_lat = la[k, v] + (clat[k] - la[k, v]) * 1e-6
                p_lon = clon[k] + dl * (1 - 1e-6)
                assert h3_oracle.latlng_to_cell(np.array([p_lat]), np.array([p_lon]), res)[0] == cells[k]
