"""Compare two rocprofv3 kernel traces of the batch leg (bare vs after context churn): kernels per
(queue, stream), how the worker streams map to hardware queues, and per-stream busy time vs span.

usage: python tools/churn_compare.py <trace dir A> <trace dir B>
"""
import csv
import sys
from collections import defaultdict


def load(d):
    rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def report(name, rows):
    per = defaultdict(lambda: [0, 0.0, None, None])
    for r in rows:
        k = (r["Queue_Id"], r["Stream_Id"])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        p = per[k]
        p[0] += 1
        p[1] += (e - s) / 1e3
        p[2] = s if p[2] is None else min(p[2], s)
        p[3] = e if p[3] is None else max(p[3], e)
    print(f"## {name}: {len(rows)} kernels")
    print("| queue | stream | kernels | busy ms | span ms |")
    print("|---|---|---:|---:|---:|")
    for (q, st), (n, busy, a, b) in sorted(per.items(), key=lambda x: -x[1][0]):
        if n < 50:
            continue
        print(f"| {q} | {st} | {n} | {busy / 1e3:.1f} | {(b - a) / 1e6:.1f} |")
    streams_per_queue = defaultdict(set)
    for (q, st), v in per.items():
        if v[0] >= 50:
            streams_per_queue[q].add(st)
    print("streams per queue:", {q: sorted(s) for q, s in streams_per_queue.items()})
    print()


def main():
    for d in sys.argv[1:]:
        report(d, load(d))


if __name__ == "__main__":
    main()
