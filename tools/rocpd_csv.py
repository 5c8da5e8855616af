"""Convert a rocprofv3 SQLite output (run_results.db) into the CSV files the
other tools read: <dir>/<prefix>_kernel_trace.csv and <prefix>_kernel_stats.csv.

usage: python tools/rocpd_csv.py <dir> [prefix=run]
"""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    pre = sys.argv[2] if len(sys.argv) > 2 else "run"
    dbs = sorted(glob.glob(os.path.join(d, "**", "*results.db"), recursive=True))
    if not dbs:
        sys.exit(f"no rocpd database under {d}")
    rows = []
    for path in dbs:
        db = sqlite3.connect(path)
        for name, start, end, stream, queue in db.execute("select name, start, end, stream_id, queue_id from kernels"):
            rows.append((name, int(start), int(end), stream, queue))
    rows.sort(key=lambda r: r[1])
    with open(os.path.join(d, f"{pre}_kernel_trace.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Stream_Id", "Queue_Id"])
        for r in rows:
            w.writerow(r)
    agg = defaultdict(list)
    for name, s, e, _, _ in rows:
        agg[name].append(e - s)
    total = sum(sum(v) for v in agg.values()) or 1
    with open(os.path.join(d, f"{pre}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v)])
    print(f"{len(rows)} dispatches, {len(agg)} kernels -> {d}/{pre}_kernel_*.csv")


if __name__ == "__main__":
    main()
