"""One batch's kernel timeline from a rocprofv3 kernel trace: start (us from the batch's k_ingest), duration, the gap
to the previous kernel's end (negative: concurrent, another queue), queue and kernel name.

    python3 tools/step_timeline.py <run_kernel_trace.csv> [batch index, default 4]
"""
import csv
import sys


def _is_ingest(name):   # (k_ingest<...> / k_ingest(...), not k_ingest_exact)
    name = name[5:] if name.startswith("void ") else name
    return name.startswith("k_ingest<") or name.startswith("k_ingest(")


def main(path, k):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if _is_ingest(r["Kernel_Name"])]
    i0, i1 = idx[k], idx[k + 1]
    t0 = int(rows[i0]["Start_Timestamp"])
    prev_end = None
    for r in rows[i0:i1 + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap:7.1f}  q{r['Queue_Id']}  {r['Kernel_Name'][:70]}")
        prev_end = max(prev_end or 0, e)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
