"""CPU baseline thread sweep: the OpenMP oracle's cfg3
S2M align at 1..all affinity CPUs on this host, median of N after 2 warm-ups.

Bench/test infrastructure (imports oracle/ as the checker-side CPU baseline).
Covariances come from the oracle too, so no GPU is needed.

    python tools/cpu_thread_sweep.py [--runs 10] [--threads 8,16,32,64,128,256]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as O  # noqa: E402
import bench  # noqa: E402


def cgroup_cpu():
    for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(p) as f:
                return p + ": " + f.read().strip()
        except OSError:
            pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--threads", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    aff = len(os.sched_getaffinity(0))
    ths = [int(t) for t in a.threads.split(",") if t] or sorted({8, 16, 32, 64, 128, aff})
    prob = bench.build_problem()
    sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
    src = prob["source"]
    kc = np.concatenate([O.covariances(kf, 10, threads=aff) for kf in prob["keyframes"]])
    tcov = np.ascontiguousarray(kc[prob["subset"]])
    scov = O.covariances(src, 10, threads=aff)
    p = O.default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32,
                         transformation_epsilon=0.01)
    guess = prob["guess"].astype(np.float32)
    rows = []
    for t in ths:
        g = O.Gicp(src, sub, p, threads=t)
        g.set_covariances(0, scov)
        g.set_covariances(1, tcov)
        for _ in range(2):
            g.align(guess)
        ts = []
        for _ in range(a.runs):
            c0 = time.perf_counter()
            _, r = g.align(guess)
            ts.append(time.perf_counter() - c0)
        rows.append({"threads": t, "median_ms": round(1e3 * float(np.median(ts)), 3),
                     "min_ms": round(1e3 * min(ts), 3), "iters": r.iterations_run})
        print(json.dumps(rows[-1]), flush=True)
    out = {"host": bench.host_info(aff), "cgroup_cpu": cgroup_cpu(), "runs": a.runs, "rows": rows}
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
