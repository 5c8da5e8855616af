"""Summarize a rocprofv3 kernel trace: per outer iteration, search/moments/lm durations (us)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
cur = []
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ddlo::", "")
    t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if n.startswith("k_align_init"):
        if cur: print(" | ".join(cur))
        cur = []
        continue
    if n.startswith("k_nn") or n.startswith("k_moments") or n.startswith("k_lm_step"):
        if t > 8.0 or not n.startswith("k_lm"):
            cur.append(f"{n.split('<')[0]} {t:.1f}")
if cur: print(" | ".join(cur))
