"""Developer tool: per-kernel start offsets and gaps of the last graph aligns in a rocprofv3 kernel trace."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_align_init' in r['Kernel_Name']]
for i0 in idx[-14:-11]:
    j = i0 + 1
    while j < len(rows) and 'k_align_init' not in rows[j]['Kernel_Name']:
        j += 1
    seq = rows[i0:j]
    t0 = int(seq[0]['Start_Timestamp'])
    print('--- align')
    prev = None
    for r in seq[:16]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        gap = (s - prev) / 1e3 if prev else 0.0
        print(f"{(s - t0) / 1e3:8.1f} +{gap:5.1f} dur {(e - s) / 1e3:6.1f}  {r['Kernel_Name'][:40]}")
        prev = e
