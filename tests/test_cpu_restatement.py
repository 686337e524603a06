"""The bench's CPU baseline, oracle/heatmap_cpu.c (the whole micro-batch in C with OpenMP), against the Spark-semantics
oracle (oracle/spark_oracle.py) batch by batch: tiles (count exact, averages within 1e-9 relative), latest rows,
watermarks, late rows and the live state -- on 1 and 4 threads."""
import math

import numpy as np
import pytest

from oracle.heatmap_cpu import CpuHeatmap
from oracle.spark_oracle import SparkHeatmapOracle

T0 = 1_759_572_000_000_000


def _batches(seed, n=20_000, nb=6):
    rng = np.random.default_rng(seed)
    out = []
    for b in range(nb):
        lat = np.degrees(np.arcsin(rng.uniform(-1, 1, n)))
        lon = rng.uniform(-180, 180, n)
        hot = rng.random(n) < 0.5   # repeated keys within and across batches
        lat[hot] = rng.choice(np.linspace(-60, 60, 40), hot.sum())
        lon[hot] = rng.choice(np.linspace(-170, 170, 40), hot.sum())
        # 4 minutes per batch, advancing 4 minutes, 3% of the rows 25 minutes old (late from the third batch on)
        ts = T0 + b * 240_000_000 + rng.integers(0, 240_000_000, n)
        old = rng.random(n) < 0.03
        ts[old] -= 25 * 60_000_000
        speed = rng.uniform(0, 90, n)
        speed[rng.random(n) < 0.02] = np.nan
        sv = rng.random(n) > 0.1
        vkey = rng.integers(0, 3000, n).astype(np.uint64)
        tie = rng.random(n) < 0.05
        ts[tie] = T0 + b * 240_000_000 + 239_000_000   # tied maxima
        lat[rng.random(n) < 0.01] = np.nan
        lon[rng.random(n) < 0.01] = 181.0
        rv = rng.random(n) > 0.01
        out.append(dict(lat=lat, lon=lon, ts_us=ts, speed=speed, speed_valid=sv, vkey=vkey, row_valid=rv))
    return out


def _close(a, b):
    return a == b or (math.isnan(a) and math.isnan(b)) or abs(a - b) <= 1e-9 * max(abs(a), abs(b))


@pytest.mark.parametrize("threads", [1, 4])
def test_cpu_restatement_equals_spark_oracle(threads):
    ora = SparkHeatmapOracle(h3_res=8)
    cpu = CpuHeatmap(h3_res=8, threads=threads)
    for b in _batches(5):
        e = ora.process_batch(**b)
        g = cpu.process_batch(**b)
        for k in ("n_valid", "n_late", "batch_max_event_ms", "watermark_ms", "late_watermark_ms", "n_state"):
            assert g[k] == e[k], k
        assert np.array_equal(g["latest_rows"], e["latest_rows"])
        t = g["tiles"]
        got = {(int(t["cell"][i]), int(t["window_start_us"][i])): i for i in range(t["cell"].size)}
        assert len(got) == t["cell"].size == len(e["tiles"])
        for x in e["tiles"]:
            i = got[(x["cell"], x["window_start_us"])]
            assert t["count"][i] == x["count"]
            assert bool(t["speed_null"][i]) == (x["avg_speed"] is None)
            if x["avg_speed"] is not None:
                assert _close(t["avg_speed"][i], x["avg_speed"])
            assert _close(t["avg_lat"][i], x["avg_lat"]) and _close(t["avg_lon"][i], x["avg_lon"])
    assert e["n_late"] > 0 and e["n_state"] > 0
    cpu.close()


def test_cpu_restatement_without_optional_columns():
    b = _batches(9, n=5000, nb=1)[0]
    e = SparkHeatmapOracle(h3_res=5).process_batch(b["lat"], b["lon"], b["ts_us"])
    g = CpuHeatmap(h3_res=5, threads=3).process_batch(b["lat"], b["lon"], b["ts_us"])
    assert g["tiles"]["cell"].size == len(e["tiles"]) and g["tiles"]["speed_null"].all()
    assert np.array_equal(g["latest_rows"], e["latest_rows"])
