#!/usr/bin/env python3
"""Reduce the rocprofv3 PMC run of tools/diag/ingest_phases to k_ingest's VALU instructions by phase.

usage: python tools/diag/ingest_phases.py <pmc dir> [--events 100000000]
Per kernel (mean over its dispatches): wave64 VALU instructions per 64 events (all, fp64, int64, other), SALU per 64
events, mean duration, and the SIMD-cycle estimate at 2 cycles per 32-bit op and 4 per fp64 / 64-bit integer op
(tools/microbench/valu_rate) over the dispatch's own cycles.  Then the phases as differences of successive kernels.
"""
import argparse
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pmc_summary import short  # noqa: E402

F64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--events", type=int, default=100_000_000)
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(dict))   # name -> dispatch -> counter -> value
    dur = defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(a.dir, "run_counter_collection.csv"))):
        name = r["Kernel_Name"]
        k = "k_phase<%s>" % name.split("k_phase<")[1][0] if "k_phase<" in name else \
            ("k_ingest<%s>" % ("true" if "<true" in name else "false") if "k_ingest<" in name else short(name))
        per[k][r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    n = a.events
    rows = {}
    for k, ds in per.items():
        if not (k.startswith("k_phase") or k.startswith("k_ingest<")):
            continue
        c = {cn: sum(d.get(cn, 0.0) for d in ds.values()) / len(ds) for cn in next(iter(ds.values()))}
        f64 = sum(c.get(x, 0.0) for x in F64)
        i64 = c.get("SQ_INSTS_VALU_INT64", 0.0)
        allv = c.get("SQ_INSTS_VALU", 0.0)
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
        simd = 4 * f64 + 4 * i64 + 2 * (allv - f64 - i64)
        rows[k] = dict(valu=allv * 64 / n, f64=f64 * 64 / n, i64=i64 * 64 / n, other=(allv - f64 - i64) * 64 / n,
                       salu=c.get("SQ_INSTS_SALU", 0.0) * 64 / n, ms=sum(dur[k].values()) / len(dur[k]),
                       issue=simd / (1024 * cyc) if cyc else 0.0)
    order = ["k_phase<0>", "k_phase<1>", "k_phase<2>", "k_phase<3>", "k_phase_digits", "k_ingest<false>", "k_ingest<true>"]
    label = {"k_phase<0>": "loads + loop", "k_phase<1>": "+ sincos x2, unit vector", "k_phase<2>": "+ closest face",
             "k_phase<3>": "+ projection, hex2d, digits", "k_phase_digits": "_faceIjkToH3 alone (+16-B load)",
             "k_ingest<false>": "k_ingest (window, registry, dedup, flags, keys)", "k_ingest<true>": "+ bin writes"}
    print(f"{'kernel':18s} {'what':48s} {'VALU/64ev':>9s} {'f64':>6s} {'i64':>6s} {'other':>6s} {'SALU':>6s} {'ms':>7s} {'issue':>6s}")
    for k in order:
        if k in rows:
            r = rows[k]
            print(f"{k:18s} {label[k]:48s} {r['valu']:9.1f} {r['f64']:6.1f} {r['i64']:6.1f} {r['other']:6.1f} {r['salu']:6.1f} "
                  f"{r['ms']:7.3f} {r['issue']:6.3f}")
    g = lambda k, f: rows[k][f] if k in rows else 0.0   # noqa: E731
    if all(k in rows for k in order[:6]):
        ph = [("loads + loop", g("k_phase<0>", "valu"), g("k_phase<0>", "ms")),
              ("sincos x2 + unit vector", g("k_phase<1>", "valu") - g("k_phase<0>", "valu"), g("k_phase<1>", "ms") - g("k_phase<0>", "ms")),
              ("closest face", g("k_phase<2>", "valu") - g("k_phase<1>", "valu"), g("k_phase<2>", "ms") - g("k_phase<1>", "ms")),
              ("projection + hex2d margins", g("k_phase<3>", "valu") - g("k_phase<2>", "valu") - (g("k_phase_digits", "valu") - g("k_phase<0>", "valu")), None),
              ("_faceIjkToH3 digits + base cell", g("k_phase_digits", "valu") - g("k_phase<0>", "valu"), None),
              ("window, registry, dedup, flags, keys", g("k_ingest<false>", "valu") - g("k_phase<3>", "valu"),
               g("k_ingest<false>", "ms") - g("k_phase<3>", "ms")),
              ("bin writes (k_ingest<true>)", g("k_ingest<true>", "valu") - g("k_ingest<false>", "valu"),
               g("k_ingest<true>", "ms") - g("k_ingest<false>", "ms"))]
        print("\nphases (wave64 VALU instructions per 64 events; ms where the kernels nest)")
        for nm, v, ms in ph:
            print(f"  {nm:40s} {v:8.1f}" + (f"   {ms:+.3f} ms" if ms is not None else ""))


if __name__ == "__main__":
    main()
