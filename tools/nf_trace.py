"""Developer tool: the kernels of the last nanoflann tree build in a rocprofv3 kernel trace (start offset, gap, duration)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
starts = [i for i, r in enumerate(rows) if 'k_nf_unsort' in r['Kernel_Name']]
i0 = starts[-2]
seq = []
for r in rows[i0:]:
    seq.append(r)
    if 'k_nf_small_global' in r['Kernel_Name']:
        break
t0 = int(seq[0]['Start_Timestamp'])
prev = None
tot = {}
for r in seq:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    name = r['Kernel_Name'].split('(')[0].replace('ddlo::', '')[:28]
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{(s - t0) / 1e3:8.1f} +{gap:5.1f} dur {(e - s) / 1e3:6.1f}  {name}")
    tot[name] = tot.get(name, 0.0) + (e - s) / 1e3
    prev = e
print('total span', (int(seq[-1]['End_Timestamp']) - t0) / 1e3, 'us')
for k, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {k:28s} {v:7.1f}")
