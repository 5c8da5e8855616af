"""Summarize a rocprofv3 --kernel-trace --stats run of bench.py into markdown.

usage: python tools/profile_summary.py <rocprof dir> [prefix=run] > profiles/<name>.md

Besides rocprof's own per-kernel stats it splits every align() into its outer
iterations (k_align_init, then k_nn_search / k_moments / k_lm_step triples)
and separates ACTIVE iterations from the no-op launches of the speculative
graph chunk (an iteration after convergence exits at its first instruction:
k_nn_search < NOOP_US).  The "linearize" average (k_nn_search + k_moments of
an active iteration) is the quantity bench.py's roofline reports from HIP
events.
"""
import csv
import sys
from collections import defaultdict

NOOP_US = 8.0


def short(name):
    return name.split("(")[0].replace("void ", "").split("::")[-1]


def main():
    d = sys.argv[1]
    pre = sys.argv[2] if len(sys.argv) > 2 else "run"
    stats = list(csv.DictReader(open(f"{d}/{pre}_kernel_stats.csv")))
    print(f"# rocprofv3 kernel summary: `{d}`\n")
    print("| kernel | calls | total ms | avg us | min us | max us | % |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for r in stats:
        print(f"| {short(r['Name'])[:48]} | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.3f} | "
              f"{float(r['AverageNs'])/1e3:.1f} | {float(r['MinNs'])/1e3:.1f} | {float(r['MaxNs'])/1e3:.1f} | "
              f"{float(r['Percentage']):.1f} |")
    trace = list(csv.DictReader(open(f"{d}/{pre}_kernel_trace.csv")))
    trace.sort(key=lambda x: int(x["Start_Timestamp"]))
    seq = [(short(x["Kernel_Name"]).split("<")[0], (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3) for x in trace]
    aligns = []
    cur = None
    for n, us in seq:
        if n == "k_align_init":
            cur = []
            aligns.append(cur)
        elif cur is not None and n in ("k_nn_search", "k_moments", "k_lm_step"):
            cur.append((n, us))
        elif cur is not None and n not in ("k_nn_search", "k_moments", "k_lm_step"):
            cur = None
    per_pos = defaultdict(lambda: defaultdict(list))
    active_lin, active_search, active_mom, active_lm = [], [], [], []
    noop = []
    for a in aligns:
        it = 0
        for i in range(0, len(a) - 2, 3):
            (n0, s), (n1, m), (n2, l) = a[i], a[i + 1], a[i + 2]
            if (n0, n1, n2) != ("k_nn_search", "k_moments", "k_lm_step"):
                break
            if s < NOOP_US:
                noop.append(s + m + l)
                continue
            per_pos[it]["search"].append(s)
            per_pos[it]["moments"].append(m)
            per_pos[it]["lm"].append(l)
            active_lin.append(s + m)
            active_search.append(s)
            active_mom.append(m)
            active_lm.append(l)
            it += 1
    avg = lambda v: sum(v) / len(v) if v else float("nan")
    print(f"\n## Active outer iterations ({len(aligns)} aligns, {len(active_lin)} active iterations, "
          f"{len(noop)} no-op iterations of the speculative chunk)\n")
    print("| iteration | n | k_nn_search us | k_moments us | k_lm_step us |")
    print("|---:|---:|---:|---:|---:|")
    for it in sorted(per_pos):
        p = per_pos[it]
        print(f"| {it} | {len(p['search'])} | {avg(p['search']):.1f} | {avg(p['moments']):.1f} | {avg(p['lm']):.1f} |")
    print(f"\n- linearize (k_nn_search + k_moments) average over active iterations: **{avg(active_lin):.1f} us** "
          f"(search {avg(active_search):.1f} + moments {avg(active_mom):.1f})")
    print(f"- k_lm_step average over active iterations: {avg(active_lm):.1f} us")
    print(f"- no-op iteration (3 launches) average: {avg(noop):.1f} us")


if __name__ == "__main__":
    main()
