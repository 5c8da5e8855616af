"""Summarize a rocprofv3 kernel trace: stats + the kernel sequence of the last align."""
import csv, sys
d = sys.argv[1]
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
for r in rows[:6]:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us  min {float(r['MinNs'])/1e3:7.1f} max {float(r['MaxNs'])/1e3:8.1f}")
t = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
seq = [(x['Kernel_Name'].split('(')[0].replace('void ', '').split('::')[-1][:14], (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3) for x in t]
idx = [i for i, s in enumerate(seq) if 'k_align_init' in s[0]][-1]
print(' | '.join(f"{n} {d:.1f}" for n, d in seq[idx:idx + 16]))
