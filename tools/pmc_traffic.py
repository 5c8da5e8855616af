"""Per-launch HBM-side traffic of the linearize (k_moments with the fused
candidate-cell lookup, or k_cell_lookup / k_nn_seed + k_nn_scan + k_moments) from two rocprofv3 --pmc passes over bench.py
(FETCH_SIZE, WRITE_SIZE; kB units), per kernel.

Counters (MI355X_MICROARCH.md, HBM section): both count L2 -> fabric
requests, so Infinity-Cache hits are included (an upper bound of the HBM
bytes).  On gfx950 FETCH_SIZE reads exactly half of the bytes of a WIDE
COALESCED streaming read (16 B per lane); other access widths are
uncalibrated.  The search kernels are gathers (leaf SoA blocks, query
states, 8-byte keys), so their FETCH_SIZE is reported as read, without the
x2; k_moments streams its own 16 B / 48 B per point but gathers the
target's covariances, so it is reported raw too, with the x2 figure beside
it as the upper bound.  `bytes_per_linearize` (what bench.py reports as
roofline.traffic) is the raw sum.  Active iterations only: search
dispatches that together ran >= 20 us, or a k_moments >= MOM_NOOP_US (a no-op
iteration exits at once).

usage: python tools/pmc_traffic.py fetch.csv write.csv [out.json]
"""
import csv
import json
import sys
from collections import defaultdict

SEARCH = ("k_cell_lookup", "k_nn_seed", "k_nn_collect", "k_nn_scan")
MOM_NOOP_US = 6.0   # a k_moments that exits at once; the fused candidate-cell linearize has no search kernel


def short(name):
    for k in SEARCH + ("k_moments",):
        if k in name:
            return k
    return None


def per_iteration(path, counter):
    """[{kernel: bytes}] per active linearize, in dispatch order."""
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    out, cur, dur_s = [], defaultdict(float), 0.0
    for r in rows:
        k = short(r["Kernel_Name"])
        if k is None:
            continue
        val = float(r["Counter_Value"]) * 1024.0   # kB -> bytes
        cur[k] += val
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if k in SEARCH:
            dur_s += dur
        else:   # k_moments closes the iteration
            if dur_s >= 20.0 or dur >= MOM_NOOP_US:
                out.append(dict(cur))
            cur, dur_s = defaultdict(float), 0.0
    return out


def main():
    f = per_iteration(sys.argv[1], "FETCH_SIZE")
    w = per_iteration(sys.argv[2], "WRITE_SIZE")
    n = min(len(f), len(w))
    kernels = sorted({k for it in f[:n] + w[:n] for k in it})
    per = {}
    for k in kernels:
        fr = sum(it.get(k, 0.0) for it in f[:n]) / n
        wr = sum(it.get(k, 0.0) for it in w[:n]) / n
        per[k] = {"fetch_raw": round(fr), "write": round(wr)}
        if k == "k_moments":
            per[k]["fetch_x2_upper"] = round(2 * fr)
    raw = sum(v["fetch_raw"] + v["write"] for v in per.values())
    search_w = sum(v["write"] for k, v in per.items() if k in SEARCH)
    res = {"iterations": n, "bytes_per_linearize": raw, "per_kernel": per,
           "search_write": search_w,
           "bytes_per_linearize_upper": raw + per.get("k_moments", {}).get("fetch_raw", 0),
           "correction": "none on the gather kernels (FETCH_SIZE as read); k_moments also raw, x2 upper bound "
                         "beside it; WRITE_SIZE as read; Infinity-Cache hits included"}
    print(json.dumps(res))
    if len(sys.argv) > 3:
        json.dump(res, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
