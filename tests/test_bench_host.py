"""bench.py's host-side accounting (no GPU): the stage its roofline prices and the algorithmic bytes per stage
(DESIGN.md §5, §7)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_dominant_stage_skips_the_concurrent_dedup():
    b = _bench()
    ms = {"ingest": 3.6, "aggregate": 0.08, "send": 0.0, "partition": 3.78, "merge": 3.84, "emit": 0.13, "dedup": 3.85}
    assert b.dominant_stage(ms) == "merge"           # the dedup's side-stream span is longer, but concurrent
    ms["partition"] = 3.9
    assert b.dominant_stage(ms) == "partition"
    assert "dedup" in b.CONCURRENT_STAGES


def test_stage_bytes_direct_path():
    b = _bench()
    n = 100_000_000
    c = {"partials": n, "tiles": 97_590_394, "state_new": 97_590_394, "table_mode": False, "sent": 0}
    s = b.stage_bytes(n, c)
    assert s["ingest"] == 42 * n
    # k_ev_hist reads the key (8); k_ev_scatter_rec reads key, speed, speed_valid, lat, lon (33) and writes 32
    assert s["partition"] == (8 + 33 + 32) * n
    assert s["merge"] == 32 * n + 113 * c["tiles"]   # no key existed before the batch
    assert s["emit"] == 98 * (n - c["tiles"])


def test_stage_bytes_multi_gpu_owner():
    b = _bench()
    n, R, S = 50_000_000, 49_000_000, 50_000_000
    c = {"partials": R, "tiles": R, "state_new": R, "table_mode": False, "sent": S}
    s = b.stage_bytes(n, c, world=2)
    # the sender's partition by region field (keys read twice; columns read, the 32-B record written), then each
    # record read from its bin and written into its destination's chunk; the owner merges without a partition
    assert s["partition"] == 16 * n + (25 + 32) * S
    assert s["send"] == (32 + 32) * S
    assert s["merge"] == 32 * R + 113 * R
    s = b.stage_bytes(n, dict(c, binned=1), world=2)
    assert s["partition"] == 0 and s["ingest"] == 43 * n + 32 * S and s["send"] == 64 * S


def test_stage_bytes_self_held_records():
    """The records of the bins a rank owns stay in its slabs (binned): only their keys are read (census), 8 B each;
    the bench's --sharded run prices the stage API at world 1 too."""
    b = _bench()
    n, S, H = 50_000_000, 50_000_000, 25_000_000
    c = {"partials": S, "tiles": S, "state_new": S, "table_mode": False, "sent": S, "binned": 1, "self_held": H}
    assert b.stage_bytes(n, c, world=2)["send"] == 64 * (S - H) + 8 * H
    c1 = dict(c, self_held=S)
    assert b.stage_bytes(n, c1, world=1, staged=True)["send"] == 8 * S
    assert b.stage_bytes(n, c1, world=1)["send"] == 0   # (hm_process_batch: no stage API)
