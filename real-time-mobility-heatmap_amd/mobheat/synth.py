"""Synthetic micro-batches shaped like BASELINE.json's configs (no network, no datasets).

Message shape and value ranges follow the reference producer (mbta_to_kafka.py:66-74: provider, vehicleId,
lat, lon, speedKmh (often null), ts as '...Z' seconds) and the Boston view of the reference UI (app.py:121).

Every generator returns a dict of numpy SoA columns ready for HeatmapEngine.process_batch:
    lat, lon (float64 deg), ts_us (int64), speed (float64), speed_valid (bool), vkey (uint64), row_valid (bool)
"""
import numpy as np

T0_C1 = 1759573470 * 1_000_000     # 2025-10-04T10:24:30Z in microseconds
T0 = 1759572000 * 1_000_000        # 2025-10-04T10:00:00Z
ATHENS = (37.9838, 23.7275)         # CITY default "ath" (reference heatmap_stream.py:23)


def _speeds(rng, n, null_frac):
    speed = rng.uniform(0.0, 80.0, n)
    valid = rng.random(n) >= null_frac
    speed[~valid] = 0.0
    return speed, valid


def c1_boston(seed=0, n=10_000, invalid_frac=0.01):
    """C1: 10k vehicles x 1 micro-batch around Boston; ts crosses a 5-minute edge; 15% null speeds."""
    rng = np.random.default_rng(seed)
    lat = rng.uniform(42.20, 42.45, n)
    lon = rng.uniform(-71.20, -70.95, n)
    ts = T0_C1 + rng.integers(0, 60, n) * 1_000_000
    speed, sv = _speeds(rng, n, 0.15)
    vkey = np.arange(n, dtype=np.uint64)
    row_valid = np.ones(n, bool)
    k = max(4, int(n * invalid_frac))
    bad = rng.choice(n, k, replace=False)
    q = k // 4
    lat[bad[:q]] = 91.0
    lon[bad[q:2 * q]] = -181.0
    lat[bad[2 * q:3 * q]] = np.nan
    row_valid[bad[3 * q:]] = False          # null vehicleId
    return dict(lat=lat, lon=lon, ts_us=ts, speed=speed, speed_valid=sv, vkey=vkey, row_valid=row_valid)


def c2_global(seed=1, n=100_000_000, n_vehicles=50_000):
    """C2: events uniform on the sphere, ICAO-like vehicle ids, 15 minutes of timestamps (3 windows)."""
    rng = np.random.default_rng(seed)
    lat = np.degrees(np.arcsin(rng.uniform(-1.0, 1.0, n)))
    lon = rng.uniform(-180.0, 180.0, n)
    ts = T0 + rng.integers(0, 15 * 60 * 1_000_000, n)
    speed, sv = _speeds(rng, n, 0.10)
    vkey = rng.integers(0, n_vehicles, n).astype(np.uint64)
    return dict(lat=lat, lon=lon, ts_us=ts, speed=speed, speed_valid=sv, vkey=vkey, row_valid=np.ones(n, bool))


def _box(center, km):
    dlat = km / 2 / 111.32
    dlon = km / 2 / (111.32 * np.cos(np.radians(center[0])))
    return center[0] - dlat, center[0] + dlat, center[1] - dlon, center[1] + dlon


def c3_city(seed=2, n=1_000_000_000, hotspots=2000, zipf_s=1.1, sigma_m=200.0, span_min=10, n_vehicles=200_000):
    """C3: city-scale, Zipf(1.1) over hot spots with 200 m Gaussian jitter in a 50x50 km box (Athens)."""
    rng = np.random.default_rng(seed)
    la0, la1, lo0, lo1 = _box(ATHENS, 50.0)
    hs_lat = rng.uniform(la0, la1, hotspots)
    hs_lon = rng.uniform(lo0, lo1, hotspots)
    w = 1.0 / np.arange(1, hotspots + 1) ** zipf_s
    h = rng.choice(hotspots, n, p=w / w.sum())
    lat = hs_lat[h] + rng.normal(0.0, sigma_m / 111_320.0, n)
    lon = hs_lon[h] + rng.normal(0.0, sigma_m / (111_320.0 * np.cos(np.radians(ATHENS[0]))), n)
    ts = T0 + rng.integers(0, span_min * 60 * 1_000_000, n)
    speed, sv = _speeds(rng, n, 0.15)
    vkey = rng.integers(0, n_vehicles, n).astype(np.uint64)
    return dict(lat=lat, lon=lon, ts_us=ts, speed=speed, speed_valid=sv, vkey=vkey, row_valid=np.ones(n, bool))


def c4_high_cardinality(seed=3, n=500_000_000, span_min=60, late_frac=0.05, n_vehicles=1_000_000):
    """C4: uniform over a 50x50 km box, 12 windows, as two data batches; batch 2 holds late_frac rows whose
    window ends at or before the watermark (exercises late-row dropping). Returns [batch1, batch2].
    Under Spark 3.5 the late filter of a batch uses the PREVIOUS batch's watermark, so run the no-data batch
    Spark inserts when the watermark advances (an empty batch) between the two."""
    rng = np.random.default_rng(seed)
    la0, la1, lo0, lo1 = _box(ATHENS, 50.0)
    half = n // 2
    out = []
    for b in range(2):
        m = half if b == 0 else n - half
        lat = rng.uniform(la0, la1, m)
        lon = rng.uniform(lo0, lo1, m)
        if b == 0:
            ts = T0 + rng.integers(0, span_min * 60 * 1_000_000, m)
        else:
            ts = T0 + span_min * 60 * 1_000_000 + rng.integers(0, span_min * 60 * 1_000_000, m)
            k = int(m * late_frac)
            ts[:k] = T0 + rng.integers(0, 10 * 60 * 1_000_000, k)     # first 2 windows: late by then
            p = rng.permutation(m)
            ts = ts[p]
        speed, sv = _speeds(rng, m, 0.10)
        vkey = rng.integers(0, n_vehicles, m).astype(np.uint64)
        out.append(dict(lat=lat, lon=lon, ts_us=ts, speed=speed, speed_valid=sv, vkey=vkey, row_valid=np.ones(m, bool)))
    return out


def c5_dedup(seed=4, n_vehicles=10_000_000, updates=50, tie_frac=0.01):
    """C5: n_vehicles x updates, distinct timestamps per vehicle except a tie subset; randomly permuted."""
    rng = np.random.default_rng(seed)
    n = n_vehicles * updates
    vkey = np.repeat(np.arange(n_vehicles, dtype=np.uint64), updates)
    step = np.tile(np.arange(updates, dtype=np.int64), n_vehicles)
    ts = T0 + step * 3_000_000 + rng.integers(0, 1_000_000, n_vehicles).repeat(updates)
    ties = rng.random(n_vehicles) < tie_frac
    last = np.arange(n_vehicles) * updates + updates - 1
    ts[last[ties] - 1] = ts[last[ties]]          # two rows share the max timestamp
    lat = rng.uniform(42.20, 42.45, n)
    lon = rng.uniform(-71.20, -70.95, n)
    speed, sv = _speeds(rng, n, 0.15)
    p = rng.permutation(n)
    return dict(lat=lat[p], lon=lon[p], ts_us=ts[p], speed=speed[p], speed_valid=sv[p], vkey=vkey[p],
                row_valid=np.ones(n, bool))


def edge_points():
    """Edge set for the UDF: poles, the antimeridian, the equator/prime meridian, sub-normals, signed zeros,
    range limits, just-outside values and non-finite values (the latter must map to None / 0)."""
    lat = [90.0, -90.0, 0.0, -0.0, 89.999999999, -89.999999999, 45.0, 5e-324, -5e-324, 1e-300, 90.0, -90.0,
           0.0, 0.0, 0.0, 0.0, 12.5, 12.5, 90.0000000001, -90.0000000001, np.nan, np.inf, -np.inf, 10.0, 10.0]
    lon = [0.0, 0.0, 180.0, -180.0, 179.999999999, -179.999999999, 0.0, 0.0, 0.0, 1e-300, 180.0, -180.0,
           0.0, -0.0, 5e-324, 1e-310, 180.0, -180.0, 0.0, 0.0, 0.0, 0.0, 0.0, 180.0000000001, np.nan]
    return np.array(lat), np.array(lon)
