"""Per-kernel averages of rocprofv3 --pmc counter passes.

usage: python tools/pmc_kernels.py <pass dir> [<pass dir> ...]
Each dir holds run_counter_collection.csv; prints counter averages per
dispatch for every kernel (active dispatches only: SQ_WAVES > 0 when known).
"""
import csv
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").split("::")[-1][:40]


def main():
    per = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> values per dispatch
    for d in sys.argv[1:]:
        rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
        disp = defaultdict(dict)
        for r in rows:
            k = (r.get("Dispatch_Id") or r.get("Correlation_Id"), short(r["Kernel_Name"]))
            disp[k][r["Counter_Name"]] = disp[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (_, kn), cv in disp.items():
            for c, v in cv.items():
                per[kn][c].append(v)
    for kn, cs in sorted(per.items()):
        n = max(len(v) for v in cs.values())
        print(f"{kn}  ({n} dispatches)")
        for c, v in sorted(cs.items()):
            big = sorted(v)[len(v) // 2:]   # upper half: active (non no-op) dispatches
            print(f"    {c:28s} mean {sum(v)/len(v):14.1f}   upper-half mean {sum(big)/max(1,len(big)):14.1f}")


if __name__ == "__main__":
    main()
