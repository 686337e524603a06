#!/usr/bin/env python3
"""Benchmark of the per-micro-batch hot path (BASELINE.json metric: events/s H3-snapped + window-aggregated).

Workload (N=1 and per rank for N>1, weak scaling): BASELINE.json configs[1] shape -- a synthetic
OpenSky-like global batch of 1e8 events uniform on the sphere, 50k vehicle ids, 15 minutes of event time
(3 five-minute windows), 10% null speeds -- at the metric's H3 resolution 8 (configs[1] quotes res 7;
--res 7 runs that).  One step = one micro-batch through the whole hot path on device-resident inputs:
one fused pass over the events (k_ingest: filter + latLngToCell + window + late test + per-vehicle max ts + one
event key per row + census of the rows per window, which sizes the per-window state tables), then either the direct
path (radix partition of the rows into (window, region) bins, the region-owned merge into the persistent
update-mode state that also writes the update-mode rows) or, for low-cardinality batches, table mode (two LDS
aggregation passes first); in-place densification of the rows (k_fill_gaps), eviction (whole window tables
released), and the latest-position flags + compaction.
Every step is a NEW micro-batch: its timestamps are the previous step's + 15 min (precomputed before the
timed region), so the stream advances, windows close and are evicted, and no row is late.  A second leg
(`state_read_leg`, N=1 only) times the regime where batches update open windows: 1 minute of event time per step,
advancing 1 minute, res 7.
For N>1 each rank runs the sharded path (mobheat.distributed: RCCL all-to-all of partials by owner).

Prints ONE JSON line (rank 0).  See DESIGN.md for the roofline's algorithmic-byte accounting.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-mobility-heatmap_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
T0 = 1759572000 * 1_000_000
SPAN_US = 15 * 60 * 1_000_000
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec
BIN_STORE_FLOOR_MS_PER_1E8 = 4.04   # 1e8 32-B records binned into 8192 bins, no other work (profiles/r5/r5mb3/)
FP64_PEAK_TFLOPS = 78.6   # MI355X fp64 vector peak: 1024 SIMDs x 16 FMA lanes x 2 x 2.4 GHz
SIMDS = 1024

# Algorithmic HBM bytes of each stage, from the batch's counts (hm_last_counts): n events, R partial
# records merged (direct path: one per aggregated row), T tiles emitted, E of them keys that existed before the batch
# (their 64-B state line is read); multi-GPU (stage API): S records this rank sent, R the records it merged as owner.
#   direct path   ingest 42/event (lat, lon, ts, vkey 8 each + row_valid 1 read; flags 1 + event key 8 written)
#                 partition 16/event (k_ev_hist and k_ev_scatter read the key) + 57/record (speed, speed_valid,
#                           lat, lon read: 25; the 32-B EventRec written)
#   binned        (the direct path's records written by k_ingest itself, hm_last_counts "binned") ingest 43/event (+ speed
#                 and speed_valid read; the event key not written -- the record carries it -- but for exception and
#                 sampled rows) + 32/record (the EventRec written into its bin); partition 0 (a scan of the 8192 bin
#                 counts)
#                 merge 32/record read + 113/tile (64-B state line + 49-B row written) + 64/pre-existing key read
#                 emit 98/gap (a 49-B row moved into a gap; gaps = R - T), dedup 20/event
#   multi-GPU     (stage API) the sender's records grouped by region field as above -- binned in k_ingest, or the
#                 partition with one bin per region field -- then send 64/sent record (k_stage_pack: the 32-B record
#                 read from its bin, written into its destination's chunk) -- except the H records of the bins the
#                 rank owns itself, kept in its slabs (binned; hm_last_counts "self_held"): 8/record, their keys read
#                 for the census; the owner merges each bin from its senders' segments and its own slabs: no partition
#                 (merge as above over the R records it received or kept)
#   table mode    aggregate 41/event + 48/record, partition 160/record (48 + 48 read, 64 written), merge 64/record
#                 read + 113/tile + 64/pre-existing key
def stage_bytes(n, c, world=1, staged=None):
    """staged: the batch ran through the stage API (default: world > 1; bench --sharded runs it at world 1 too)."""
    staged = world > 1 if staged is None else staged
    R, T = c["partials"], c["tiles"]
    E = max(T - c["state_new"], 0)
    b = {"ingest": 42 * n, "dedup": 20 * n, "emit": 98 * max(R - T, 0), "send": 0}
    if c["table_mode"]:
        b.update(aggregate=41 * n + 48 * R, partition=160 * R, merge=64 * R + 113 * T + 64 * E)
        return b
    S = c["sent"] if staged else R   # records this rank grouped (and sent)
    b.update(aggregate=0, merge=32 * R + 113 * T + 64 * E)
    if c.get("binned"):
        b.update(ingest=43 * n + 32 * S, partition=0)
    else:
        b.update(partition=16 * n + 57 * S)
    if staged:
        H = c.get("self_held", 0)
        b["send"] = 64 * (S - H) + 8 * H
    return b


def s8d_stage_bytes(n, c):
    """SURVEY.md section 8(d)'s bytes per stage of one step: 42 B per input event (k_ingest), 56 B per emitted tile + 2 x
    56 B per touched group (the merge's output and state read/write), 40 B per latest row (the dedup); the build's
    intermediate stages carry none."""
    b = {k: 0 for k in STAGES}
    b.update(ingest=42 * n, merge=3 * 56 * c["tiles"], dedup=40 * c.get("latest", 0))
    return b


def s8d(n, c, ms):
    b = 42 * n + (56 + 2 * 56) * c["tiles"]
    return {"bytes": b, "ms": ms, "achieved_gbs": b / (ms * 1e-3) / 1e9, "frac": b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}


STAGES = ["ingest", "aggregate", "send", "partition", "merge", "emit", "dedup"]
CONCURRENT_STAGES = ("dedup",)   # side stream (hm_process_batch): its kernel_ms is the side-stream span
# HBM traffic per dispatch of every kernel and k_ingest's VALU instruction mix per event of this workload, counted by
# rocprofv3 PMC passes of this same command (tools/ingest_pmc.py + tools/pmc_calib.py -> profiles/r5/kernel_pmc.json).
PMC_FILE = next((f for f in (os.path.join(ROOT, "profiles", r, "kernel_pmc.json") for r in ("r6", "r5")) if os.path.exists(f)),
                os.path.join(ROOT, "profiles", "r6", "kernel_pmc.json"))
STAGE_KERNELS = {"ingest": ["k_ingest"], "aggregate": ["k_agg", "k_bin_reduce"], "send": ["k_stage_pack"],
                 "partition": ["k_ev_hist", "k_ev_scatter_rec"], "merge": ["k_merge_owned"], "emit": ["k_fill_gaps"],
                 "dedup": ["k_dedup_flag"]}


def dominant_stage(avg_ms):
    """The stage the roofline prices: the longest of the serial stages on the main stream (the dedup runs on a side
    stream, concurrently with the partition and merge: its time is a span shared with them, not a stage of the step)."""
    return max((k for k in STAGES if k not in CONCURRENT_STAGES), key=lambda k: avg_ms[k])


def ingest_pmc(res, n, world):
    """The PMC file's counts, only when they were taken on this exact workload (one GPU, same res and batch)."""
    try:
        d = json.load(open(PMC_FILE))
    except (OSError, ValueError):
        return None
    return d if d.get("h3_res") == res and d.get("events_per_dispatch") == n and world == 1 else None


def gen_batch(n, steps, seed, dev, span_us=SPAN_US, advance_us=SPAN_US):
    """C2-shaped batch generated on the device (inputs resident in HBM before timing); step s's timestamps are
    step 0's + s * advance_us."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    lat = torch.rad2deg(torch.asin(torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 2 - 1))
    lon = torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 360.0 - 180.0
    base = T0 + torch.randint(0, span_us, (n,), generator=g, device=dev, dtype=torch.int64)
    ts = [base + s * advance_us for s in range(steps)]
    speed = torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 80.0
    sv = (torch.rand(n, generator=g, device=dev) >= 0.10).to(torch.uint8)
    vkey = torch.randint(0, 50_000, (n,), generator=g, device=dev, dtype=torch.int64)
    rv = torch.ones(n, dtype=torch.uint8, device=dev)
    return dict(lat=lat, lon=lon, ts=ts, speed=speed, sv=sv, vkey=vkey, rv=rv)


def spark_probe():
    """the CPU baseline is the reference's Spark plan under local[N] when pyspark 3.5.1, Java 17 and
    h3 are on this host; else the literal "Spark baseline unavailable" and the restatement (labelled so) instead."""
    import importlib.util
    import shutil
    missing = [m for m in ("pyspark", "h3") if importlib.util.find_spec(m) is None]
    if shutil.which("java") is None:
        missing.append("java")
    return ("Spark baseline unavailable" + (f" (not on this host: {', '.join(missing)})" if missing else
                                            " (the Spark plan itself is not part of this harness)"))


def _median_batches(make, res, threads, reps=5, fresh=False):
    """1 warm-up + the median of `reps` timed batches through oracle/heatmap_cpu.c on `threads` threads.  make(i) -> the
    i-th run's batches (the last one timed; earlier ones untimed, e.g. the batch before a late batch); fresh: a new stream
    per run (else one stream, each run's batches after the previous run's)."""
    from oracle.heatmap_cpu import CpuHeatmap
    c = None
    dts = []
    n = 0
    for i in range(reps + 1):
        if fresh or c is None:
            if c is not None:
                c.close()
            c = CpuHeatmap(h3_res=res, threads=threads)
        bs = make(i)
        for b in bs[:-1]:
            c.process_batch(**b, arrays=False)
        t = time.perf_counter()
        c.process_batch(**bs[-1], arrays=False)
        dt = time.perf_counter() - t
        n = bs[-1]["lat"].size
        if i:   # (run 0: the warm-up)
            dts.append(dt)
    c.close()
    med = sorted(dts)[len(dts) // 2]
    return {"value": n / med, "unit": "events/s", "cores": threads, "median_s": med, "events": n,
            "protocol": f"1 warm-up + median of {reps}", "kind": "port"}


def cpu_baseline(sample, res):
    """The oracle's C restatement of the whole micro-batch (oracle/heatmap_cpu.c: filter, latLngToCell, window,
    watermark, update-mode aggregation into hash-partitioned state tables, eviction, latest rows per vehicle; OpenMP)
    timed on this host on bounded samples, 1 warm-up + the median of 5, on every host thread this
    job may use (OMP_NUM_THREADS, else the CPU count) and on one thread: C2 (the bench's workload: one stream, each
    batch 15 min after the last, so its windows are new and the previous batch's evicted), and C3, C4, C5 samples."""
    from mobheat import synth
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))

    def c2(n):
        base = synth.c2_global(seed=11, n=n)

        def make(i):
            return [dict(base, ts_us=base["ts_us"] + i * SPAN_US)]
        return make

    out = _median_batches(c2(sample), res, threads)
    n1 = max(sample // 6, 10_000)
    one = _median_batches(c2(n1), res, 1)
    out.update({"kind": "port", "spark": spark_probe(),
                "sample": f"restatement: oracle/heatmap_cpu.c (C + OpenMP, H3 from oracle/h3_oracle.c), {sample:,}-event "
                          f"C2-shaped batches (seed 11, res {res}) of one stream 15 min apart, on {threads} threads: "
                          f"1 warm-up + median of 5, {out['median_s']:.2f} s per batch",
                "single_thread": dict(one, sample=f"the same on 1 thread, {n1:,}-event batches")})
    # BASELINE.md section 2's other configs, bounded samples of their shapes (each run a fresh stream)
    m = max(sample // 6, 100_000)
    c3 = synth.c3_city(seed=12, n=m)
    c4 = synth.c4_high_cardinality(seed=13, n=2 * m)
    c5 = synth.c5_dedup(seed=14, n_vehicles=max(m // 50, 1000), updates=50)
    empty = {k: v[:0] for k, v in c4[0].items()}
    configs = {
        "c3": (9, lambda i: [c3], f"C3 sample: {m:,} events, Zipf(1.1) over 2,000 hot spots in a 50x50 km box, res 9"),
        "c4": (12, lambda i: [c4[0], empty, c4[1]],
               f"C4 sample: {2 * m:,} events uniform in a 50x50 km box, res 12, 12 windows, two batches + Spark's no-data "
               f"batch between them, 5% of the second late; the second batch timed ({c4[1]['lat'].size:,} events)"),
        "c5": (8, lambda i: [c5], f"C5 sample: {c5['lat'].size // 50:,} vehicles x 50 updates, 1% max-ts ties, permuted, res 8"),
    }
    for name, (r, make, what) in configs.items():
        out[name] = dict(_median_batches(make, r, threads, fresh=True), sample=what)
    return out


def cpu_baseline_c1(reps=5):
    """BASELINE.md section 2's mandatory C1 CPU baseline: configs[0]'s Boston batch (10,000 events, one per vehicle, res
    8, crossing a 5-minute edge, 15% null speeds, 1% invalid rows; synth.c1_boston) through the oracle's C restatement of
    the micro-batch (oracle/heatmap_cpu.c) on every host thread this job may use and on one, then the reference-form
    UpdateOne ops of foreach_batch_func (stream.tile_ops / position_ops, heatmap_stream.py:159-235) built from its
    output and BSON-encoded as pymongo sends them (the sink itself replaced, as the plan says).  1 warm-up + the median
    of `reps`; each run a fresh stream (a new state), as the reference's first batch."""
    from mobheat import stream, synth
    from oracle.heatmap_cpu import CpuHeatmap
    b = synth.c1_boston(seed=0)
    n = b["lat"].size
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    cols = dict(provider=["mbta"] * n, vehicleId=[f"v{i:05d}" for i in range(n)], ts_us=b["ts_us"], lat=b["lat"],
                lon=b["lon"])

    def batch(th):
        c = CpuHeatmap(h3_res=8, threads=th)
        t = time.perf_counter()
        r = c.process_batch(**b)
        dt = time.perf_counter() - t
        c.close()
        return dt, r

    def ops(r):
        import bson
        import pandas as pd
        T = r["tiles"]
        tiles = _Tiles(dict(T, window_end_us=T["window_start_us"] + 300_000_000))
        t = time.perf_counter()
        o = stream.tile_ops(tiles, city="ath", h3_res=8, ttl_min=45) + \
            stream.position_ops({k: (pd.Series(v) if k in ("provider", "vehicleId") else v) for k, v in cols.items()},
                                r["latest_rows"])
        for op in o:   # the statement pymongo's bulk encodes for each UpdateOne
            bson.encode({"q": op._filter, "u": op._doc, "multi": False, "upsert": True})
        return time.perf_counter() - t, len(o)

    out = {"config": "C1: 10,000 Boston events (synth.c1_boston seed 0), one micro-batch, H3 res 8", "events": n,
           "protocol": f"1 warm-up + median of {reps}"}
    for th in (threads, 1):
        batch(th)
        runs = [batch(th) for _ in range(reps)]
        ts = sorted(x[0] for x in runs)
        med = ts[len(ts) // 2]
        out[f"restatement_{th}t"] = {"value": n / med, "unit": "events/s", "cores": th, "median_s": med,
                                     "kind": "port", "tiles": int(runs[0][1]["tiles"]["cell"].size)}
    r = runs[0][1]
    ops(r)
    ot = sorted(ops(r) for _ in range(reps))
    med_ops = ot[len(ot) // 2][0]
    out["foreach_ops_1t"] = {"median_s": med_ops, "ops": ot[0][1],
                             "note": "the reference's per-row UpdateOne build + BSON encode (heatmap_stream.py:159-235)"}
    one = out["restatement_1t"]["median_s"] + med_ops
    out["value"] = n / one
    out["unit"] = "events/s"
    out["cores"] = 1
    out["kind"] = "port"
    out["sample"] = "C1 batch through the restatement on 1 thread + the reference-form ops, median of 5"
    return out


class _Tiles:
    """tile_ops' view of a tiles dict (attribute access and len())."""

    def __init__(self, d):
        self.__dict__.update(d)

    def __len__(self):
        return len(self.cell)


def run_leg(args, n, res, span_us, advance_us, seed, dev, local, world, rank, arena_bytes=0, sharded=False):
    """Warmup + exactly K timed steps (barrier + synchronize on both sides, max over ranks); per-stage HIP-event
    times (the library's events on its own stream) and algorithmic bytes of the timed steps."""
    import mobheat
    from mobheat.distributed import LibStages, ShardedHeatmap
    total_steps = args.warmup + args.steps
    data = gen_batch(n, total_steps, seed=seed, dev=dev, span_us=span_us, advance_us=advance_us)
    eng = mobheat.HeatmapEngine(h3_res=res, device=local, batch_capacity_hint=n, state_arena_bytes=arena_bytes,
                                shard=(rank, world) if world > 1 else None)
    sharded = ShardedHeatmap(LibStages(eng), dev) if (world > 1 or sharded) else None

    def step(s):
        ptrs = dict(n=n, lat=data["lat"].data_ptr(), lon=data["lon"].data_ptr(), ts_us=data["ts"][s].data_ptr(),
                    speed=data["speed"].data_ptr(), speed_valid=data["sv"].data_ptr(), vkey=data["vkey"].data_ptr(),
                    row_valid=data["rv"].data_ptr())
        if sharded is None:
            return eng.process_batch_device(s, **ptrs)
        return sharded.process_batch(s, ptrs)

    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    kt = {k: 0.0 for k in STAGES}
    kb = {k: 0.0 for k in STAGES}
    step_ms = []
    host = []   # per step: the library call's host side (wall, syncs, allocations; single GPU)
    phases = []   # per step (sharded path): host wall ms of each stage phase (distributed.ShardedHeatmap)
    counts = None
    t0 = time.perf_counter()
    for s in range(args.warmup, total_steps):
        ts0 = time.perf_counter()
        step(s)
        step_ms.append((time.perf_counter() - ts0) * 1e3)
        if sharded is None:
            host.append(eng.last_host_timings())
        else:
            phases.append(dict(sharded.last_phase_ms))
        tm = eng.last_timings()
        counts = eng.last_counts()
        for k in STAGES:
            kt[k] += max(tm[k], 0.0)
        for k, v in stage_bytes(n, counts, world, staged=sharded is not None).items():
            kb[k] += v
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist.is_initialized():
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    eng.close()
    del data
    torch.cuda.empty_cache()
    K = args.steps
    return dict(elapsed=elapsed, step_ms=step_ms, kt={k: v / K for k, v in kt.items()},
                kb={k: v / K for k, v in kb.items()}, counts=counts, host=host,
                phases={k: round(float(np.median([p[k] for p in phases])), 3) for k in phases[0]} if phases else None)


def slowest_step(leg):
    """the slowest timed step: its wall ms and the library call's host side (where a step's time outside the
    kernels went: stream synchronizations -- the longest one and its library source line -- and allocations)"""
    if not leg["host"]:
        return None
    i = max(range(len(leg["step_ms"])), key=lambda k: leg["step_ms"][k])
    return dict(step=i, wall_ms=round(leg["step_ms"][i], 3), **{k: (round(v, 3) if isinstance(v, float) else v)
                                                               for k, v in leg["host"][i].items()},
                allocs_frees_per_step=[h["allocs_frees"] for h in leg["host"]])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--events", type=int, default=100_000_000, help="events per step per GPU")
    ap.add_argument("--res", type=int, default=8)
    ap.add_argument("--cpu-sample", type=int, default=12_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-state-leg", action="store_true", help="skip the 1-minute-advance state-read leg")
    ap.add_argument("--sharded", action="store_true",
                    help="run the multi-GPU stage path (mobheat.distributed over torch.distributed) even at --gpus 1: "
                         "at N=1 the exchange is RCCL's all-to-all of a rank with itself (the N>1 code path on one GPU)")
    ap.add_argument("--c1-baseline", action="store_true", help="only the C1 CPU baseline (BASELINE.md section 2)")
    args = ap.parse_args()
    if args.c1_baseline:
        print(json.dumps(cpu_baseline_c1()), flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # (ranks beyond the visible GPUs share them round-robin: lets a 1-GPU box rehearse the N>1 path)
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    sharded = world > 1 or args.sharded
    if sharded:
        # RCCL ("nccl") over xGMI; MOBHEAT_DIST_BACKEND=gloo only to rehearse several ranks on one GPU (RCCL
        # refuses two ranks on one device).  A --sharded N=1 run started without torchrun rendezvouses by itself.
        if "MASTER_ADDR" not in os.environ:
            import socket
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]), RANK="0", WORLD_SIZE="1")
            s.close()
        backend = os.environ.get("MOBHEAT_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, **({"device_id": dev} if backend == "nccl" else {}))

    n = args.events
    K = args.steps
    A = run_leg(args, n, args.res, SPAN_US, SPAN_US, 1 + 7919 * rank, dev, local, world, rank, sharded=sharded)
    elapsed, avg_ms, kb, c = A["elapsed"], A["kt"], A["kb"], A["counts"]
    ms_step = elapsed / K * 1e3
    # Roofline of the dominant stage by time, priced on HBM (the metric's "% HBM peak"), with the PMC-counted
    # traffic of its kernels when the PMC file was taken on this exact workload (tools/ingest_pmc.py).
    dom = dominant_stage(avg_ms)
    gbs = kb[dom] / (avg_ms[dom] * 1e-3) / 1e9 if avg_ms[dom] > 0 else 0.0
    # SURVEY.md section 8(d)'s own bytes for the dominant stage (independent of this build's intermediates): k_ingest
    # 42 B per input event; the merge 56 B per emitted tile + 2 x 56 B of state read and written per touched group
    s8 = s8d_stage_bytes(n, c)[dom]
    roof = {"bound": "hbm", "kernel": dom, "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gbs / HBM_PEAK_GBS, "frac_basis": "this build's algorithmic bytes (stage_bytes: the 32-B records "
                                                      "it writes and reads between its kernels counted)",
            "achieved_s8d": s8 / (avg_ms[dom] * 1e-3) / 1e9 if avg_ms[dom] > 0 else 0.0,
            "frac_s8d": s8 / (avg_ms[dom] * 1e-3) / 1e9 / HBM_PEAK_GBS if avg_ms[dom] > 0 else 0.0,
            "s8d_bytes_per_launch": s8, "traffic": None}
    pmc = ingest_pmc(args.res, n, world)
    if pmc is not None and all(k in pmc.get("kernels", {}) for k in STAGE_KERNELS[dom]):
        # FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE, per dispatch, summed over the stage's kernels; a kernel
        # whose patterns were calibrated (tools/pmc_calib.py: k_ingest's 8-B loads, returned atomics, scattered
        # records on known byte counts) counts its calibrated bytes, the counted ones beside them
        # `traffic` is the raw counted bytes (FETCH_SIZE x 2 + WRITE_SIZE): the calibration's account of them
        # (returned atomics as 31 B writes, the x 0.516 FETCH_SIZE of 8-B non-temporal loads) is beside it, labelled,
        # not substituted -- VERDICT r5: its residual write bytes came out negative
        ks = [pmc["kernels"][k] for k in STAGE_KERNELS[dom]]
        roof["traffic"] = sum(k["hbm_bytes"] for k in ks)
        if any("calibrated" in k for k in ks):
            roof["traffic_calibrated_model"] = sum(k.get("calibrated", {}).get("hbm_bytes", k["hbm_bytes"]) for k in ks)
        roof["traffic_source"] = os.path.relpath(PMC_FILE, ROOT)
    if pmc is not None:
        # k_ingest is bound by VALU issue and latency, not HBM: its VALU side from the same PMC file
        sec = avg_ms["ingest"] * 1e-3
        tf = pmc["fp64_flops_per_event"] * n / sec / 1e12
        # VALU issue: a wave64 instruction holds its SIMD-32 for 2 cycles (32-bit ops) or 4 (fp64 and 64-bit integer
        # ops), as tools/microbench/valu_rate measures at saturation (profiles/r4/valu_rate.txt); the cycles are the
        # PMC dispatch's own (GRBM_GUI_ACTIVE / 8), so the fraction comes from counters of one dispatch only
        f64, i64 = pmc["valu_f64_wave_insts_per_64_events"], pmc["valu_int64_wave_insts_per_64_events"]
        simd_cycles = (4 * f64 + 4 * i64 + 2 * pmc["valu_other_wave_insts_per_64_events"]) * n / 64
        roof["ingest_valu"] = {"fp64_tflops": tf, "fp64_peak_tflops": FP64_PEAK_TFLOPS, "fp64_frac": tf / FP64_PEAK_TFLOPS,
                               "issue_frac": simd_cycles / (SIMDS * pmc["dispatch_cycles"]),
                               "active_inst_valu_per_busy_cu_cycle": pmc["active_inst_valu_per_busy_cu_cycle"],
                               "valu_wave_insts_per_64_events": pmc["valu_wave_insts_per_64_events"],
                               "fp64_flops_per_event": pmc["fp64_flops_per_event"]}
    if dom == "ingest" and c.get("binned"):
        # what bounds the binned ingest instead of HBM bandwidth: its records' scattered 32-B
        # stores and bin-cursor atomics alone, 1e8 records into 8192 bins, measured by tools/microbench/bin_chunk.hip
        # ("direct" pattern, profiles/r5/r5mb3/direct_8192.txt) -- scaled to this launch's records
        floor_ms = BIN_STORE_FLOOR_MS_PER_1E8 * c["partials"] / 1e8
        roof["binning_floor"] = {"ms": floor_ms, "frac": floor_ms / avg_ms["ingest"] if avg_ms["ingest"] > 0 else None,
                                 "source": "profiles/r5/r5mb3/direct_8192.txt"}
    step_bytes = sum(kb.values())
    roof.update({"kernel_ms": {k: round(v, 3) for k, v in avg_ms.items()}, "concurrent_stages": list(CONCURRENT_STAGES),
                 "algorithmic_bytes_per_launch": kb[dom],
                 "units_per_launch": {"events": n, "records": c["partials"], "tiles": c["tiles"], "sent": c["sent"]},
                 # the whole step: every stage's algorithmic bytes / the step's wall time / 8 TB/s
                 "step": {"algorithmic_bytes": step_bytes, "ms": ms_step,
                          "achieved_gbs": step_bytes / (ms_step * 1e-3) / 1e9,
                          "frac": step_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS},
                 # SURVEY.md section 8(d)'s own bytes for the step, independent of this build's intermediates: 42 B per
                 # event in, 56 B per emitted tile, 2 x 56 B per touched state group (read + write)
                 "step_s8d": s8d(n, c, ms_step)})
    value = world * n * K / elapsed
    out = {
        "metric": METRIC, "value": value, "unit": "events/s", "n_gpus": world, "steps": K, "warmup": args.warmup,
        "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"C2-shaped global batch: {n:,} events/step/GPU uniform on the sphere, 50k vehicles, "
                               f"15 min of event time (3 windows) per step, advancing 15 min per step; H3 res {args.res}",
                   "events_per_step_per_gpu": n, "h3_res": args.res, "parallelism": f"dp{world}",
                   # the process group the exchange ran on, as torch.distributed reports it (None: one GPU, no exchange)
                   "dist_backend": dist.get_backend() if dist.is_initialized() else None,
                   "dist_world_size": dist.get_world_size() if dist.is_initialized() else 1,
                   "stage_path": sharded,
                   "binned_in_ingest": bool(c.get("binned")),
                   "tiles_emitted_last_step": c["tiles"], "partials_last_step": c["partials"],
                   "records_sent_last_step": c["sent"],
                   "table_mode": c["table_mode"]},
        "roofline": roof,
        "slowest_step": slowest_step(A),
    }
    if A["phases"]:   # the sharded path: median host wall ms per stage phase (rank 0)
        out["stage_phase_ms"] = A["phases"]
    B = None
    if world == 1 and not sharded and not args.no_state_leg:
        # second leg: the state-read regime of the reference's ~2-s trigger (README.md:134-135) -- each micro-batch
        # holds 1 minute of event time and the stream advances 1 minute per step, so consecutive batches update the
        # same open windows and the merge reads existing state lines.  res 7 (configs[1]'s resolution): 1e8 events
        # per minute re-touch most of a window's keys from its second batch on.
        # (its windows' tables come from a state arena reserved at create, so that no multi-GB table is allocated
        # inside a timed step: a window's table grows to 2^28 slots (17.4 GB) once its minutes have touched more than
        # 67M cells, and the leg holds up to three such tables plus the smaller ones it grew from -- ~700 B per event.
        # Round 3's per-step host timing found the leg's occasional multi-second stall in the step that allocated, with
        # 400 B per event, the table the arena no longer covered)
        B = run_leg(args, n, 7, 60_000_000, 60_000_000, 2, dev, local, world, rank, arena_bytes=700 * n)
        bms = B["elapsed"] / K * 1e3
        bb = sum(B["kb"].values())
        out["state_read_leg"] = {
            "value": n * K / B["elapsed"], "unit": "events/s", "ms_per_step": bms, "h3_res": 7,
            "workload": f"{n:,} events/step uniform on the sphere, 1 min of event time per step, advancing 1 min per step",
            "kernel_ms": {k: round(v, 3) for k, v in B["kt"].items()},
            "tiles_last_step": B["counts"]["tiles"], "state_keys_created_last_step": B["counts"]["state_new"],
            "step_frac": bb / (bms * 1e-3) / 1e9 / HBM_PEAK_GBS, "step_s8d": s8d(n, B["counts"], bms),
            "slowest_step": slowest_step(B)}
    if rank == 0 and world == 1 and not sharded and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_sample, args.res)
        out["cpu_baseline"]["c1"] = cpu_baseline_c1()
    if rank == 0:
        print("per-step ms (host wall, rank 0): " + " ".join(f"{x:.1f}" for x in A["step_ms"]), file=sys.stderr, flush=True)
        if B is not None:
            print("state-read leg per-step ms: " + " ".join(f"{x:.1f}" for x in B["step_ms"]), file=sys.stderr, flush=True)
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
