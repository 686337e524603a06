"""Timeline of one step from a rocprofv3 database (--kernel-trace [--memory-copy-trace], default rocpd output): every
kernel and copy of the step, in start order, with its offset from the step's first dispatch, its duration, its queue, and
the device-idle gaps (no kernel or copy running on any queue) -- where the host's synchronizations and launches show.

usage: python tools/trace_timeline.py <run_results.db> [--anchor k_ingest] [--step -2] [--min-gap-us 5]
A step starts at a dispatch whose kernel name contains --anchor; --step picks one (Python index: -2 = the last but one).
"""
import argparse
import sqlite3


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", default="k_ingest<true")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--min-gap-us", type=float, default=5.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ev = [(s, e, short(n), "q%s" % q) for s, e, n, q in c.execute("select start, end, name, queue_id from kernels")]
    try:
        ev += [(s, e, "copy %s %dB" % (n, sz), "q%s" % q)
               for s, e, n, sz, q in c.execute("select start, end, name, size, queue_id from memory_copies")]
    except sqlite3.Error:
        pass
    ev.sort()
    starts = [i for i, x in enumerate(ev) if a.anchor in x[2]]
    if len(starts) < 2:
        raise SystemExit("fewer than two steps found (anchor %r)" % a.anchor)
    k = starts[a.step]
    nxt = [i for i in starts if i > k]
    end = nxt[0] if nxt else len(ev)
    t0 = ev[k][0]
    busy_to = t0
    idle = 0.0
    print("%9s %9s  %-6s %s" % ("start_us", "dur_us", "queue", "name"))
    for s, e, n, q in ev[k:end]:
        if s > busy_to and (s - busy_to) / 1e3 >= a.min_gap_us:
            print("%9s %9.1f  %-6s -- idle" % ("", (s - busy_to) / 1e3, ""))
        if s > busy_to:
            idle += (s - busy_to) / 1e3
        busy_to = max(busy_to, e)
        print("%9.1f %9.1f  %-6s %s" % ((s - t0) / 1e3, (e - s) / 1e3, q, n))
    span = (ev[end][0] - t0) / 1e3 if end < len(ev) else (busy_to - t0) / 1e3
    print("step span %.1f us (to the next step's first dispatch), device idle %.1f us" % (span, idle))


if __name__ == "__main__":
    main()
