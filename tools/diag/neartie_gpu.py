"""Diagnostic (GPU box): where the device latLngToCell differs from the oracle on the constructed near-tie inputs of
tests/test_gpu_boundary.py; prints each mismatch with the host execution of the same device code (fast + exact path)
and whether this host's CPU has FMA (glibc picks its FMA variants of sin/cos/atan2/... then)."""
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-mobility-heatmap_amd")]
from mobheat import _lib, latlng_to_cell  # noqa: E402
from oracle import h3_oracle  # noqa: E402

h3_oracle.load()
spec = importlib.util.spec_from_file_location("tb", os.path.join(ROOT, "tests", "test_gpu_boundary.py"))
tb = importlib.util.module_from_spec(spec)
spec.loader.exec_module(tb)
flags = open("/proc/cpuinfo").read().split("flags")[1].split("\n")[0]
print("host cpu fma:", " fma " in flags + " ", "avx2:", " avx2 " in flags + " ")
for res in range(16):
    lat, lon = tb._near_tie_points(res)
    ok = (np.abs(lat) <= 90) & (np.abs(lon) <= 180)
    got = latlng_to_cell(lat, lon, res)
    n_exact = _lib.load().hm_latlng_to_cell_last_exact(0)
    exp = h3_oracle.latlng_to_cell(lat, lon, res)
    hf, fb = _lib.latlng_to_cell_fast_host_selftest(lat, lon, res)
    bad = np.nonzero(ok & (got != exp))[0]
    print(f"res {res}: n {lat.size} exact-path {n_exact} mismatches {bad.size} host-fast-vs-oracle "
          f"{int((ok & (hf != exp)).sum())}", flush=True)
    for i in bad[:6]:
        print(f"   lat {lat[i].hex()} lon {lon[i].hex()} gpu {int(got[i]):x} oracle {int(exp[i]):x} "
              f"host {int(hf[i]):x} host-fell-back {bool(fb[i])}", flush=True)
