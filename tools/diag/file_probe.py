#!/usr/bin/env python3
"""How fast a checkpoint file of a 1e7-key delta (635 MB) reaches the disk on this box: one
write() vs pwrite() from T threads into the page cache, the fsync after each, and O_DIRECT writes from an aligned
buffer -- the numbers the checkpoint writer's layout is chosen from.

usage: python tools/diag/file_probe.py [--mb 635] [--dir /tmp]   (JSON lines)
"""
import argparse
import json
import mmap
import os
import tempfile
import threading
import time

import numpy as np


def pwrite_threads(fd, buf, threads, off0=0):
    n = len(buf)
    step = -(-n // threads)
    step = -(-step // 4096) * 4096
    errs = []

    def job(lo):
        try:
            mv = buf[lo:min(lo + step, n)]
            done = 0
            while done < len(mv):
                done += os.pwrite(fd, mv[done:], off0 + lo + done)
        except OSError as e:
            errs.append(e)
    ts = [threading.Thread(target=job, args=(lo,)) for lo in range(0, n, step)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=635)
    ap.add_argument("--dir", default=tempfile.gettempdir())
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pinned", action="store_true")
    a = ap.parse_args()
    nbytes = a.mb << 20
    mounts = [ln.split() for ln in open("/proc/mounts")]
    best = max((m for m in mounts if a.dir.startswith(m[1])), key=lambda m: len(m[1]))
    print(json.dumps({"dir": a.dir, "fs": best[2], "mount": best[1], "dev": best[0], "bytes": nbytes}), flush=True)
    raw = mmap.mmap(-1, nbytes)   # (page-aligned: usable for O_DIRECT)
    buf = memoryview(raw)
    np.frombuffer(raw, np.uint8)[:] = np.random.default_rng(0).integers(0, 256, nbytes, dtype=np.uint8)
    path = os.path.join(a.dir, "mobheat_file_probe.bin")
    bufs = {"mmap": buf}
    if a.pinned:   # page-locked host memory (hipHostMalloc, as the engine's export buffer): O_DIRECT from it
        import torch
        pt = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        pn = pt.numpy()
        pn[:] = np.frombuffer(raw, np.uint8)
        bufs["pinned"] = memoryview(pn)
    for rep in range(a.reps):
        for src, buf in bufs.items():
            for mode, threads in (("write", 1), ("pwrite", 4), ("direct", 1), ("direct", 4)):
                flags = os.O_WRONLY | os.O_CREAT | os.O_TRUNC
                if mode == "direct":
                    flags |= getattr(os, "O_DIRECT", 0)
                try:
                    fd = os.open(path, flags, 0o644)
                except OSError as e:
                    print(json.dumps({"mode": mode, "threads": threads, "error": repr(e)}), flush=True)
                    continue
                try:
                    t0 = time.perf_counter()
                    if mode == "write":
                        done = 0
                        while done < nbytes:
                            done += os.write(fd, buf[done:])
                    else:
                        pwrite_threads(fd, buf, threads)
                    t1 = time.perf_counter()
                    os.fsync(fd)
                    t2 = time.perf_counter()
                    print(json.dumps({"rep": rep, "src": src, "mode": mode, "threads": threads, "write_ms": round(1e3 * (t1 - t0), 1),
                                      "fsync_ms": round(1e3 * (t2 - t1), 1), "GBps": round(nbytes / (t2 - t0) / 1e9, 2)}),
                          flush=True)
                except OSError as e:
                    print(json.dumps({"mode": mode, "threads": threads, "error": repr(e)}), flush=True)
                finally:
                    os.close(fd)
                    os.remove(path)


if __name__ == "__main__":
    main()
