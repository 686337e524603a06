"""Reduce rocprofv3 PMC passes of `bench.py` to k_ingest's per-event fp64 FLOPs and HBM bytes, and every other
kernel's HBM bytes per dispatch (the `kernels` section: bench.py's roofline traffic for whichever stage dominates).

usage: python tools/ingest_pmc.py --res 8 --events 100000000 --out profiles/r1/kernel_pmc.json <pmc dirs...>

fp64 FLOPs: 64 x SQ_INSTS_VALU_FLOPS_FP64 (+ _TRANS), cross-checked against (2*FMA + ADD + MUL + TRANS)_F64 x 64 lanes.
HBM bytes: FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts half of a wide streaming read, MI355X_MICROARCH.md §HBM;
calibrated on this kernel's own input stream) + WRITE_SIZE; both reported by rocprofv3 in KB.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, required=True)
    ap.add_argument("--events", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("dirs", nargs="+")
    a = ap.parse_args()
    vals, dur = load(a.dirs)
    c = {k: sum(v) / len(v) for k, v in vals["k_ingest"].items()}
    n = a.events
    lanes = (2 * c.get("SQ_INSTS_VALU_FMA_F64", 0) + c.get("SQ_INSTS_VALU_ADD_F64", 0) + c.get("SQ_INSTS_VALU_MUL_F64", 0)
             + c.get("SQ_INSTS_VALU_TRANS_F64", 0)) * 64
    # the FLOPS counters tally per wave instruction (x64 lanes; cross-checks with the instruction counts)
    flops = 64 * (c.get("SQ_INSTS_VALU_FLOPS_FP64", 0) + c.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0))
    f64_insts = sum(c.get(k, 0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                          "SQ_INSTS_VALU_TRANS_F64"))
    fetch = c.get("FETCH_SIZE", 0) * 1024 * 2
    write = c.get("WRITE_SIZE", 0) * 1024
    kernels = {}
    for k, cv in vals.items():
        if "FETCH_SIZE" not in cv or "WRITE_SIZE" not in cv or not k.startswith("k_"):
            continue
        f = sum(cv["FETCH_SIZE"]) / len(cv["FETCH_SIZE"]) * 1024
        w = sum(cv["WRITE_SIZE"]) / len(cv["WRITE_SIZE"]) * 1024
        kernels[k] = {"dispatches": len(dur[k]), "mean_dispatch_ms": 1e3 * sum(dur[k].values()) / len(dur[k]),
                      "fetch_bytes_raw": f, "write_bytes": w, "hbm_bytes": 2 * f + w}
    i64 = c.get("SQ_INSTS_VALU_INT64", 0)
    cycles = c.get("GRBM_GUI_ACTIVE", 0) / 8   # the dispatch's shader cycles (rocprofv3 sums the 8 XCDs)
    d = {"h3_res": a.res, "events_per_dispatch": n,
         "fp64_flops_per_event": flops / n,
         "fp64_flops_per_event_from_inst_counts": lanes / n,
         # wave64 VALU instructions per 64 events (= lane-instructions per event)
         "valu_wave_insts_per_64_events": c.get("SQ_INSTS_VALU", 0) * 64 / n,
         "valu_f64_wave_insts_per_64_events": f64_insts * 64 / n,
         "valu_int64_wave_insts_per_64_events": i64 * 64 / n,
         "valu_other_wave_insts_per_64_events": (c.get("SQ_INSTS_VALU", 0) - f64_insts - i64) * 64 / n,
         "dispatch_cycles": cycles,
         # SQ_ACTIVE_INST_VALU counts one per VALU instruction (equal to SQ_INSTS_VALU in every valu_rate dispatch)
         # and SQ_BUSY_CU_CYCLES CU-cycles: VALU instructions per CU-cycle (ceiling 4 SIMDs / 2 cycles for 32-bit
         # ops, 4 / 4 for fp64 and 64-bit integer ops)
         "active_inst_valu_per_busy_cu_cycle": (c.get("SQ_ACTIVE_INST_VALU", 0) / c["SQ_BUSY_CU_CYCLES"]
                                                if c.get("SQ_BUSY_CU_CYCLES") else None),
         "hbm_bytes_per_event": (fetch + write) / n,
         "hbm_read_bytes_per_event": fetch / n, "hbm_write_bytes_per_event": write / n,
         "mean_dispatch_ms": 1e3 * sum(dur["k_ingest"].values()) / len(dur["k_ingest"]),
         "counters_mean_per_dispatch": c,
         "kernels": kernels,
         "source": [os.path.relpath(x) for x in a.dirs]}
    json.dump(d, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in d.items() if k != "counters_mean_per_dispatch"}, indent=1))


if __name__ == "__main__":
    main()
