"""GPU: BASELINE.json's full-size configurations on one MI355X, device-generated, checked through size-independent
properties (the oracle cannot run these sizes; tools/scale_check.py holds the generators and the checks):

  C2 configs[1]  1e8 events uniform on the sphere at res 7 (its own resolution), one batch;
  C4 configs[3]  5e8 events at res 12 over a 50x50 km box, 12 windows per batch, two batches of 2.5e8 with Spark's
                 no-data batch between them, 5% of batch 2 late (exactly those rows dropped);
  C5 configs[4]  1e7 vehicles x 50 updates, permuted, a 1% tie subset (both tied rows kept);
  C3 configs[2]  one GPU's 1.25e8-event shard of the city-scale batch, eight batches advancing 10 min.
Each asserts: counts add up to the aggregated rows, no key emitted twice, window starts in range, the late rows
dropped exactly, and the latest rows (one per vehicle at its max, two for ties).  
"""
import json
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.fixture(scope="module")
def dev():
    import torch
    d = torch.device("cuda", 0)
    torch.cuda.set_device(d)
    yield d
    torch.cuda.empty_cache()


@pytest.mark.parametrize("config", ["c2", "c4", "c5", "c3"])
def test_full_size_config(config, dev, capsys):
    import torch
    import scale_check
    r = {"c2": scale_check.run_c2, "c3": scale_check.run_c3, "c4": scale_check.run_c4,
         "c5": scale_check.run_c5}[config](dev, 1.0)
    torch.cuda.empty_cache()
    assert r["ok"]
    with capsys.disabled():
        print("\n" + json.dumps(r))
