"""Summarize a rocprofv3 --kernel-trace --stats run of bench.py into markdown.

usage: python tools/profile_summary.py <rocprof dir> [prefix=run] > profiles/<name>.md

Besides rocprof's own per-kernel stats it splits every align() into its outer
iterations (k_align_init, then per iteration the search kernels — k_cell_lookup,
k_nn_seed + k_nn_scan, or none when the candidate-cell lookup is fused into
k_moments — k_moments, k_mom_reduce + RCCL's all-reduce (sharded) and
k_lm_step) and separates ACTIVE iterations from no-op launches (an
iteration after convergence exits at its first instruction: search kernels
< NOOP_US and k_moments < MOM_NOOP_US).  No-ops
are counted per origin: the eager profiled path (gicp_set_profiling)
launches all max_iterations iterations of an align, a graph align launches
at most one speculative chunk after the converged one.  The "linearize" average (search + k_moments of
an active iteration) is the quantity bench.py's roofline reports from HIP
events.
"""
import csv
import sys
from collections import defaultdict

NOOP_US = 20.0   # summed search kernels of an iteration that exits at once (three launches, ~4-6 us each)
MOM_NOOP_US = 6.0   # k_moments of an iteration that exits at once (~3.5-4.7 us); the fused candidate-cell
                    # linearize (k_moments<.., LOOKUP>) has no search kernel at all


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
    # k_moments<true, ...> is the LM step fused into the moment kernel (the one-kernel candidate-cell
    # iteration of a graph align since round 6): it ends its iteration like k_lm_step does
    seq = []
    for x in trace:
        full = short(x["Kernel_Name"])
        n = full.split("<")[0]
        if n == "k_moments" and full.replace(" ", "").startswith("k_moments<true"):
            n = "k_moments_fused"
        seq.append((n, (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3))
    SEARCH = ("k_cell_lookup", "k_nn_seed", "k_nn_collect", "k_nn_scan")
    LOOP = SEARCH + ("k_moments", "k_moments_fused", "k_lm_step", "k_mom_reduce")
    # a sharded align's all-reduce sits between k_mom_reduce and k_lm_step (RCCL's own kernel)
    SKIP = ("ncclDevKernel", "ncclKernel", "__amd_rocclr")
    aligns = []
    cur = None
    for n, us in seq:
        if n == "k_align_init":
            cur = []
            aligns.append(cur)
        elif cur is not None and n in LOOP:
            cur.append((n, us))
        elif cur is not None and n.startswith(SKIP):
            continue
        else:
            cur = None
    per_pos = defaultdict(lambda: defaultdict(list))
    active_lin, active_search, active_mom, active_lm = [], [], [], []
    active_lin_eager, active_fused, fused_pos = [], [], defaultdict(list)
    noop, noop_eager = [], []
    eager_aligns = 0
    for a in aligns:
        # iterations: search kernels..., k_moments, k_lm_step
        iters, it_k = [], defaultdict(float)
        for n, us in a:
            it_k[n] += us
            if n in ("k_lm_step", "k_moments_fused"):
                iters.append(it_k)
                it_k = defaultdict(float)
        # a graph align launches <= kMaxFirstChunk (8) + a few single-iteration
        # chunks; an eager profiled align launches every iteration
        eager = len(iters) > 12
        eager_aligns += eager
        it = 0
        for k in iters:
            s_us = sum(k[n] for n in SEARCH)
            if k["k_moments_fused"] > 0:
                f = k["k_moments_fused"]
                if f < MOM_NOOP_US:
                    (noop_eager if eager else noop).append(f)
                    continue
                fused_pos[it].append(f)
                active_fused.append(f)
                it += 1
                continue
            m, l = k["k_moments"], k["k_lm_step"]
            if s_us < NOOP_US and m < MOM_NOOP_US:
                (noop_eager if eager else noop).append(s_us + m + l)
                continue
            if eager:
                active_lin_eager.append(s_us + m)
            per_pos[it]["search"].append(s_us)
            per_pos[it]["seed"].append(k["k_nn_seed"])
            per_pos[it]["collect"].append(k["k_nn_collect"])
            per_pos[it]["scan"].append(k["k_nn_scan"])
            per_pos[it]["lookup"].append(k["k_cell_lookup"])
            per_pos[it]["moments"].append(m)
            per_pos[it]["reduce"].append(k["k_mom_reduce"])
            per_pos[it]["lm"].append(l)
            active_lin.append(s_us + m)
            active_search.append(s_us)
            active_mom.append(m)
            active_lm.append(l)
            it += 1
    avg = lambda v: sum(v) / len(v) if v else float("nan")
    print(f"\n## Active outer iterations ({len(aligns)} aligns, {len(active_lin)} active iterations; no-op "
          f"iterations: {len(noop)} in {len(aligns) - eager_aligns} graph aligns (speculative chunk), "
          f"{len(noop_eager)} in {eager_aligns} eager profiled aligns)\n")
    print("| iteration | n | search us (lookup + seed + scan) | k_moments us | k_mom_reduce us | k_lm_step us |")
    print("|---:|---:|---:|---:|---:|---:|")
    for it in sorted(per_pos):
        p = per_pos[it]
        print(f"| {it} | {len(p['search'])} | {avg(p['search']):.1f} ({avg(p['lookup']):.1f} + {avg(p['seed']):.1f} + {avg(p['scan']):.1f}) | "
              f"{avg(p['moments']):.1f} | {avg(p['reduce']):.1f} | {avg(p['lm']):.1f} |")
    print(f"\n- linearize (search kernels + k_moments) average over active iterations: **{avg(active_lin):.1f} us** "
          f"(search {avg(active_search):.1f} + moments {avg(active_mom):.1f})")
    print(f"- k_lm_step average over active iterations: {avg(active_lm):.1f} us")
    print(f"- no-op iteration (3 launches) average: {avg(noop + noop_eager):.1f} us")
    if active_fused:
        print(f"\n## Graph aligns: the LM step fused into the lookup moment kernel ({len(active_fused)} active "
              f"iterations)\n")
        print("| iteration | n | k_moments<true, true> us (lookup + moments + fan-in + LM step) |")
        print("|---:|---:|---:|")
        for it in sorted(fused_pos):
            print(f"| {it} | {len(fused_pos[it])} | {avg(fused_pos[it]):.1f} |")
        print(f"\n- fused iteration average: **{avg(active_fused):.1f} us**; the linearize alone is timed on the "
              f"eager profiled aligns above (unfused, as bench.py's roofline): {avg(active_lin_eager):.1f} us")


if __name__ == "__main__":
    main()
