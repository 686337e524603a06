"""Diagnostic (GPU box host): the oracle's table derivation status and its agreement with the product's tables."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
from oracle import h3_oracle  # noqa: E402
from test_h3_oracle import _product_tables  # noqa: E402

flags = open("/proc/cpuinfo").read().split("flags")[1].split("\n")[0]
print("host cpu fma:", " fma " in flags + " ", flush=True)
try:
    ob, of, on = h3_oracle.tables()
    pb, pf, pn = _product_tables()
    for name, o, p in (("baseCellData", ob, pb), ("faceIjkBaseCells", of, pf), ("faceNeighbors", on, pn)):
        bad = np.argwhere(o != p)
        print(name, "differences:", len(bad), bad[:10].tolist(), flush=True)
except RuntimeError as e:
    print("derivation failed:", e, flush=True)
