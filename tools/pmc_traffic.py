"""Per-launch HBM-side traffic of the linearize (k_nn_seed + k_nn_collect +
k_nn_scan + k_moments, or the single-kernel k_nn_search + k_moments) from
two rocprofv3 --pmc passes over bench.py (FETCH_SIZE, WRITE_SIZE; kB units).

Corrections (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports
half of the bytes of wide coalesced reads -> doubled here; WRITE_SIZE is
taken as reported.  Both count L2 -> fabric requests, i.e. Infinity-Cache
hits are included (upper bound of the HBM bytes).  Active iterations only:
search dispatches that together ran >= 20 us (no-op iterations exit at once).

usage: python tools/pmc_traffic.py fetch.csv write.csv [out.json]
"""
import csv
import json
import sys


SEARCH = ("k_nn_seed", "k_nn_collect", "k_nn_scan", "k_nn_search")


def per_iteration(path, counter):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    out = []
    val_s, dur_s = 0.0, 0.0
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        dur_us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        val = float(r["Counter_Value"]) * 1024.0  # kB -> bytes
        if any(k in name for k in SEARCH):
            val_s += val
            dur_s += dur_us
        elif "k_moments" in name:
            if dur_s >= 20.0:
                out.append((val_s, val))
            val_s, dur_s = 0.0, 0.0
    return out


def main():
    f = per_iteration(sys.argv[1], "FETCH_SIZE")
    w = per_iteration(sys.argv[2], "WRITE_SIZE")
    n = min(len(f), len(w))
    fetch_search = 2.0 * sum(x[0] for x in f[:n]) / n
    fetch_mom = 2.0 * sum(x[1] for x in f[:n]) / n
    write_search = sum(x[0] for x in w[:n]) / n
    write_mom = sum(x[1] for x in w[:n]) / n
    res = {"iterations": n,
           "bytes_per_linearize": round(fetch_search + fetch_mom + write_search + write_mom),
           "search": {"fetch": round(fetch_search), "write": round(write_search)},
           "moments": {"fetch": round(fetch_mom), "write": round(write_mom)},
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE x1; Infinity-Cache hits included"}
    print(json.dumps(res))
    if len(sys.argv) > 3:
        json.dump(res, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
