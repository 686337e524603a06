#!/usr/bin/env python3
"""Generate the committed golden fixtures (inputs + expected outputs) under tests/golden/.

Provenance: expected outputs come from the repo's CPU ORACLE (oracle/h3_oracle.c + oracle/spark_oracle.py),
i.e. they are RESTATEMENT-DERIVED, not produced by the reference (h3-py / pyspark are not importable here and
the reference ships no fixtures -- SURVEY.md §8c).  They pin the oracle against regressions and give the GPU
parity tests fixed expected values.  The H3 part is anchored by the public known-answer vectors in
tests/test_h3_oracle.py.

Run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-mobility-heatmap_amd")]

from mobheat import synth  # noqa: E402
from oracle import h3_oracle, spark_oracle  # noqa: E402


def h3_cells():
    rng = np.random.default_rng(2024)
    n = 2000
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, n)))
    lon = rng.uniform(-180, 180, n)
    el, eo = synth.edge_points()
    kat_lat = np.array([40.689167, 37.769377, 37.3615593])
    kat_lon = np.array([-74.044444, -122.388903, -122.0553238])
    lat = np.concatenate([kat_lat, el, lat])
    lon = np.concatenate([kat_lon, eo, lon])
    out = dict(lat=lat, lon=lon)
    for res in range(16):
        out[f"cells_r{res}"] = h3_oracle.latlng_to_cell(lat, lon, res)
    np.savez_compressed(os.path.join(HERE, "h3_cells.npz"), **out)


def c1_batch():
    b = synth.c1_boston()
    o = spark_oracle.SparkHeatmapOracle(h3_res=8)
    r = o.process_batch(**b)
    t = r["tiles"]
    np.savez_compressed(
        os.path.join(HERE, "c1_batch.npz"), **{f"in_{k}": v for k, v in b.items()},
        t_cell=np.array([x["cell"] for x in t], np.uint64), t_ws=np.array([x["window_start_us"] for x in t], np.int64),
        t_count=np.array([x["count"] for x in t], np.int64),
        t_speed=np.array([np.nan if x["avg_speed"] is None else x["avg_speed"] for x in t]),
        t_speed_null=np.array([x["avg_speed"] is None for x in t]),
        t_lon=np.array([x["avg_lon"] for x in t]), t_lat=np.array([x["avg_lat"] for x in t]),
        latest=r["latest_rows"], n_valid=r["n_valid"])


if __name__ == "__main__":
    h3_cells()
    c1_batch()
    print("golden fixtures written to", HERE)
