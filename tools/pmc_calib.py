"""rocprofv3's FETCH_SIZE / WRITE_SIZE on known byte counts in k_ingest<true>'s own access patterns
(tools/microbench/pmc_calib.hip), and the calibrated HBM traffic of a bench PMC file's k_ingest.

usage: python tools/pmc_calib.py --calib <fetch pass dir> <write pass dir> [--rows N]
                                 [--pmc profiles/r5/kernel_pmc.json --records R]   (adds k_ingest's calibrated bytes)

Patterns (per dispatch, N rows): k_nt8 reads 42 N (8-B non-temporal loads of 5 columns + two 1-B columns, k_ingest's
columns); k_st9 writes 9 N (1-B flag + 8-B key per row); k_atom makes N returned 32-bit atomics on 8192 counters (no
data); k_scat32 writes 32 N (two 16-B stores per row at scattered slots: the binned records).
k_ingest<true> calibrated = FETCH_SIZE / (nt8 counted / known)  +  (WRITE_SIZE - R x atom bytes per atomic) with the
flag/key and record stores each divided by their pattern's counted / known ratio (R = records binned).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def mean(v):
    return sum(v) / len(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calib", nargs=2, required=True, metavar=("FETCH_DIR", "WRITE_DIR"))
    ap.add_argument("--rows", type=int, default=100000000 // 8192 * 8192)
    ap.add_argument("--pmc", help="a kernel_pmc.json (tools/ingest_pmc.py) to add k_ingest's calibrated bytes to")
    ap.add_argument("--records", type=int, default=None, help="records k_ingest binned per dispatch (default: rows)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    f, _ = load([a.calib[0]])
    w, _ = load([a.calib[1]])
    n = a.rows
    fetch = {k: mean(v["FETCH_SIZE"]) * 1024 for k, v in f.items() if "FETCH_SIZE" in v}
    write = {k: mean(v["WRITE_SIZE"]) * 1024 for k, v in w.items() if "WRITE_SIZE" in v}
    cal = {
        "rows": n,
        "nt8_fetch_per_known_read": fetch["k_nt8"] / (42 * n),
        "st9_write_per_known_write": write["k_st9"] / (9 * n),
        "scat32_write_per_known_write": write["k_scat32"] / (32 * n),
        "atom_write_bytes_per_atomic": write["k_atom"] / n,
        "atom_fetch_bytes_per_atomic": fetch.get("k_atom", 0.0) / n,
        "scat32_fetch_bytes_per_record": fetch.get("k_scat32", 0.0) / n,
        "raw": {"fetch": fetch, "write": write},
        "source": [os.path.relpath(x) for x in a.calib],
    }
    out = {"calibration": cal}
    if a.pmc:
        d = json.load(open(a.pmc))
        ev = d["events_per_dispatch"]
        R = a.records if a.records is not None else ev
        k = d["kernels"]["k_ingest"]
        f_raw, w_raw = k["fetch_bytes_raw"], k["write_bytes"]
        reads = f_raw / cal["nt8_fetch_per_known_read"]
        w_atom = R * cal["atom_write_bytes_per_atomic"]
        # the writes left once the atomics' counted bytes are taken out: flags (1 B per event; the 8-B event key only
        # for exception and sampled rows since round 5) and records (32 B per record), each at its pattern's counted /
        # known ratio (the coalesced row-order pattern: st9's)
        w_data = w_raw - w_atom
        w_model = cal["st9_write_per_known_write"] * 1 * ev + cal["scat32_write_per_known_write"] * 32 * R
        writes = 1 * ev + 32 * R + (w_data - w_model)   # (the residual: counted writes the patterns do not explain)
        k["calibrated"] = {"read_bytes": reads, "write_bytes": writes, "hbm_bytes": reads + writes,
                           "atomics_counted_write_bytes": w_atom, "unexplained_write_bytes": w_data - w_model,
                           "algorithmic_bytes": 43 * ev + 32 * R, "records": R}
        d["calibration"] = cal
        json.dump(d, open(a.out or a.pmc, "w"), indent=1)
        out["k_ingest_calibrated"] = k["calibrated"]
    print(json.dumps(out, indent=1, default=float))


if __name__ == "__main__":
    main()
