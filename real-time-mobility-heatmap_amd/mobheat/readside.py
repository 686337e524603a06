"""The read side's hot loop: the reference's web API turns every tile of the latest window into
a GeoJSON polygon, one h3.cell_to_boundary call per tile (reference app.py:19-41 h3_boundary_geojson, :45-69
api_tiles_latest).  Here the boundaries of all the window's cells come from one GPU launch (hm_cells_to_boundary,
csrc/h3_boundary.h); the Flask app, MongoDB queries and the Leaflet page stay out of scope.

Mirrors the reference's helper names and output shapes:
  h3_boundary_geojson(cell_id) -> [[lng, lat], ..., [lng, lat]] closed ring (app.py:19-41)
  tiles_latest_collection(docs) -> the FeatureCollection dict api_tiles_latest returns for a window's tile docs
"""
import numpy as np

from . import _lib
from ._lib import HM_MEM_HOST, check, ptr


def cells_to_boundary(cells, device=0):
    """cellToBoundary of an array of cells on the GPU: (lat [n, 10], lng [n, 10], nverts [n]) in degrees,
    upstream's vertex order; nverts 0 for an invalid index."""
    lib = _lib.load()
    cells = np.ascontiguousarray(cells, dtype=np.uint64)
    lat = np.empty((cells.size, 10))
    lng = np.empty((cells.size, 10))
    nv = np.empty(cells.size, np.int32)
    if cells.size:
        check(lib.hm_cells_to_boundary(ptr(cells), cells.size, HM_MEM_HOST, int(device), ptr(lat), ptr(lng), ptr(nv)),
              None, "hm_cells_to_boundary")
    return lat, lng, nv


def _cell_int(cell_id):
    return int(cell_id, 16) if isinstance(cell_id, str) else int(cell_id)


def rings(cells, device=0):
    """GeoJSON rings of many cells: [[lng, lat], ...] closed (first vertex repeated), as h3_boundary_geojson."""
    lat, lng, nv = cells_to_boundary(np.array([_cell_int(c) for c in cells], dtype=np.uint64), device)
    out = []
    for k in range(len(nv)):
        ring = [[float(lng[k, v]), float(lat[k, v])] for v in range(nv[k])]
        if ring and ring[0] != ring[-1]:
            ring.append(ring[0])
        out.append(ring)
    return out


def h3_boundary_geojson(cell_id, device=0):
    """Closed GeoJSON ring [[lng, lat], ...] of one cell (reference app.py:19-41); cell_id as h3-py's hex string."""
    return rings([cell_id], device)[0]


def tiles_latest_collection(docs, device=0):
    """The FeatureCollection of reference app.py:45-69 for the tile documents of the latest window (dicts with
    cellId, count, avgSpeedKmh, windowStart, windowEnd as the tiles collection stores them)."""
    docs = list(docs)
    geoms = rings([d["cellId"] for d in docs], device)
    features = []
    for d, ring in zip(docs, geoms):
        props = {"cellId": d["cellId"], "count": int(d.get("count", 0)), "avgSpeedKmh": float(d.get("avgSpeedKmh", 0.0)),
                 "windowStart": d["windowStart"].isoformat(), "windowEnd": d["windowEnd"].isoformat()}
        features.append({"type": "Feature", "geometry": {"type": "Polygon", "coordinates": [ring]},
                         "properties": props})
    return {"type": "FeatureCollection", "features": features}

