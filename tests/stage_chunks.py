"""Test helper: the multi-GPU exchange chunk (include/mobheat.h, csrc/k_stage.h ChunkHdr / chunk_layout) written and
read in numpy, so that the oracle stage backend (tests/test_distributed_gloo.py OracleStages) speaks the library's wire
format.  One chunk per (sender, destination): a 64-B header (8 int64: magic, records, candidates, record bytes, bins,
records offset, candidates offset, bytes); direct path: u32 counts[bins] and u32 census[4096], each padded to 32 B;
the records (32-B EventRec grouped by region field, or 48-B tile partials); the 32-B candidates."""
import numpy as np

MAGIC = 0x314B4E5548434D48
CENSUS_WORDS = 4096
EVENT_DT = np.dtype([("key", "<u8"), ("sp", "<u8"), ("lat", "<f8"), ("lon", "<f8")])
TILE_DT = np.dtype([("cell", "<u8"), ("ws", "<i8"), ("count", "<u4"), ("nsp", "<u4"), ("ssp", "<f8"), ("slat", "<f8"),
                    ("slon", "<f8")])
CAND_DT = np.dtype([("vkey", "<u8"), ("ts", "<i8"), ("row", "<i8"), ("origin", "<i8")])


def pad32(b):
    return (int(b) + 31) & ~31


def layout(records, cands, rec_bytes, bins):
    recs_off = 64 + ((pad32(bins * 4) + pad32(CENSUS_WORDS * 4)) if bins > 0 else 0)
    cands_off = recs_off + pad32(records * rec_bytes)
    return dict(records=int(records), cands=int(cands), rec_bytes=int(rec_bytes), bins=int(bins), recs_off=recs_off,
                cands_off=cands_off, bytes=cands_off + int(cands) * 32)


def pack(recs, cands, bins=None, counts=None, census=None):
    """One chunk: recs (EVENT_DT or TILE_DT array), cands (CAND_DT); direct path: bins, counts[bins], census[4096]."""
    direct = recs.dtype == EVENT_DT
    b = int(bins) if direct else 0
    L = layout(recs.size, cands.size, recs.dtype.itemsize, b)
    out = np.zeros(L["bytes"], np.uint8)
    out[:64].view(np.int64)[:] = [MAGIC, L["records"], L["cands"], L["rec_bytes"], L["bins"], L["recs_off"],
                                  L["cands_off"], L["bytes"]]
    if direct:
        out[64: 64 + 4 * b].view(np.uint32)[:] = counts
        c0 = 64 + pad32(4 * b)
        out[c0: c0 + 4 * CENSUS_WORDS].view(np.uint32)[:] = census
    out[L["recs_off"]: L["recs_off"] + recs.nbytes] = recs.view(np.uint8)
    out[L["cands_off"]: L["cands_off"] + cands.nbytes] = cands.view(np.uint8)
    return out


def unpack(buf, sizes, direct):
    """The chunks of every sender, in order -> (records concatenated, candidates concatenated, per-chunk headers)."""
    buf = np.asarray(buf, np.uint8)
    off, recs, cands, hdrs = 0, [], [], []
    dt = EVENT_DT if direct else TILE_DT
    for n in sizes:
        c = buf[off: off + n]
        h = c[:64].view(np.int64)
        assert h[0] == MAGIC and h[7] == n, (h, n)
        recs.append(c[h[5]: h[5] + h[1] * h[3]].view(dt))
        cands.append(c[h[6]: h[6] + h[2] * 32].view(CAND_DT))
        hdrs.append(h.copy())
        off += n
    return (np.concatenate(recs) if recs else np.zeros(0, dt), np.concatenate(cands) if cands else np.zeros(0, CAND_DT),
            hdrs)
