"""CPU: the checkpoint file writer (engine.save_state_file) in its streamed form -- the records filled slice by slice by a
copier thread (Engine.export_begin's fill: hm_state_export_copy) while the slices that landed are written, with
O_DIRECT writes from the page-aligned export buffer (header padded to 4 KiB, last block zero-padded, file truncated)
or buffered + fsync -- reads back exactly what the one-shot buffered writer writes (reference heatmap_stream.py:37,244:
the state store behind checkpointLocation)."""
import mmap
import os

import numpy as np
import pytest

from mobheat import engine as E


def _records(n, seed):
    rng = np.random.default_rng(seed)
    r = np.zeros(n, E.STATE_REC_DTYPE)
    r["cell"] = rng.integers(1, 2**62, n, dtype=np.uint64)
    r["window_start_us"] = rng.integers(0, 10**15, n)
    r["count"] = rng.integers(1, 100, n)
    r["n_speed"] = r["count"] // 2
    r["sum_speed"] = rng.uniform(0, 1e4, n)
    r["sum_lat"] = rng.uniform(-90, 90, n)
    r["sum_lon"] = rng.uniform(-180, 180, n)
    return r


INFO = {k: 7 for k in E._INFO_FIELDS}


@pytest.mark.parametrize("n", [0, 1, 63, 64, 1000, 4097])
@pytest.mark.parametrize("direct", ["1", "0"])
def test_streamed_state_file_reads_back(tmp_path, monkeypatch, n, direct):
    monkeypatch.setenv("MOBHEAT_CKPT_DIRECT", direct)
    monkeypatch.setattr(E._Slices, "SLICE", 256)   # (several slices, the last one partial)
    src = _records(n, n)
    need = -(-max(n, 1) * 64 // 4096) * 4096
    buf = mmap.mmap(-1, need + 4096)
    raw = np.frombuffer(buf, np.uint8)
    raw[:] = 0xAB   # (the bytes past the records: the writer pads the last block with zeros, the file ends at n)
    recs = raw[: n * 64].view(E.STATE_REC_DTYPE)
    calls = []

    def fill(first, count):
        calls.append((first, count))
        recs[first:first + count] = src[first:first + count]
    path = str(tmp_path / "delta-3.r0of1.mhs")
    E.save_state_file(path, INFO, recs, meta='{"x": 1}', fill=fill, raw=raw)
    info, got = E.load_state_file(path)
    assert info == INFO and got.tobytes() == src.tobytes()
    assert E.read_state_meta(path) == '{"x": 1}'
    assert calls == [(lo, min(256, n - lo)) for lo in range(0, n, 256)]
    head = 4096 if direct == "1" else None
    size = os.path.getsize(path)
    assert size % 64 == 0 and (head is None or size == head + 64 * n)
    # the one-shot buffered writer: the same records and header fields
    ref = str(tmp_path / "ref.mhs")
    E.save_state_file(ref, INFO, src, meta='{"x": 1}')
    assert E.load_state_file(ref)[1].tobytes() == got.tobytes()
    assert not [f for f in os.listdir(tmp_path) if ".tmp" in f]
    del recs, raw
    buf.close()


def test_streamed_state_file_fill_error_leaves_no_file(tmp_path, monkeypatch):
    monkeypatch.setattr(E._Slices, "SLICE", 64)
    n = 500
    buf = mmap.mmap(-1, 64 * 1024)
    raw = np.frombuffer(buf, np.uint8)
    recs = raw[: n * 64].view(E.STATE_REC_DTYPE)

    def fill(first, count):
        if first >= 256:
            raise RuntimeError("hm_state_export_copy: failed")
    path = str(tmp_path / "state-1.r0of1.mhs")
    with pytest.raises(RuntimeError, match="export_copy"):
        E.save_state_file(path, INFO, recs, meta=None, fill=fill, raw=raw)
    assert os.listdir(tmp_path) == []
