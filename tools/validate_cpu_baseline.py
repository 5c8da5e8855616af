"""Container-side validation of the timed CPU baseline:
the oracle's kd-tree stages (oracle/cpu_ref.cpp, the "port" bench.py times on
the GPU box) against the reference's OWN nanoflann compiled from
/root/reference (oracle/_ref) on identical inputs — kd-tree build, k=10 self
kNN (the covariance search) and the 1-NN correspondence search, 2 warm-ups then
the median of 10, at 8 threads and 1 thread.  Writes
profiles/r03_cpu_validation.json and .md; the bar is +-25 %."""
import ctypes as C
import json
import os
import platform
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from dynamic_direct_lidar_odometry_amd import scene  # noqa: E402
from oracle import oracle as O  # noqa: E402


def med(fn, runs=10, warm=2):
    for _ in range(warm):
        fn()
    t = []
    for _ in range(runs):
        c0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - c0)
    return 1e3 * float(np.median(t))


def main():
    L, R = O.lib(), O.ref_lib()
    if R is None:
        sys.exit("oracle/_ref not built (needs /root/reference): run make -C oracle")
    prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
    src = np.ascontiguousarray(prob["source"], np.float32)
    sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]], np.float32)
    fp = lambda a: a.ctypes.data_as(C.c_void_p)
    rows = []

    def stage(name, n, port_fn, ref_fn, threads):
        os.environ["OMP_NUM_THREADS"] = str(threads)
        a, b = med(port_fn), med(ref_fn)
        rows.append({"stage": name, "points": n, "threads": threads, "port_ms": round(a, 3), "reference_ms": round(b, 3),
                     "ratio": round(a / b, 3), "within_25pct": bool(abs(a / b - 1.0) <= 0.25)})
        print(rows[-1], flush=True)

    for name, pts in (("kd-tree build", src), ("kd-tree build", sub)):
        stage(name, len(pts), lambda p=pts: L.oref_tree_free(L.oref_tree_build(fp(p), len(p))),
              lambda p=pts: R.ref_tree_free(R.ref_tree_build(fp(p), len(p))), 1)
    ts_port = L.oref_tree_build(fp(src), len(src))
    ts_ref = R.ref_tree_build(fp(src), len(src))
    tt_port = L.oref_tree_build(fp(sub), len(sub))
    tt_ref = R.ref_tree_build(fp(sub), len(sub))
    for threads in (8, 1):
        k = 10
        idx = np.zeros((len(src), k), np.int32)
        d = np.zeros((len(src), k), np.float32)
        # the reference driver runs its OpenMP loop with the process-wide thread count
        import ctypes.util
        gomp = C.CDLL(ctypes.util.find_library("gomp"))
        gomp.omp_set_num_threads(threads)
        stage("k=10 self kNN (covariances)", len(src),
              lambda: L.oref_tree_knn(ts_port, fp(src), len(src), k, fp(idx), fp(d), threads),
              lambda: R.ref_tree_knn(ts_ref, fp(src), len(src), k, fp(idx), fp(d)), threads)
        idx1 = np.zeros((len(src), 1), np.int32)
        d1 = np.zeros((len(src), 1), np.float32)
        stage("1-NN 131k -> 500k (one outer iteration's search)", len(src),
              lambda: L.oref_tree_knn(tt_port, fp(src), len(src), 1, fp(idx1), fp(d1), threads),
              lambda: R.ref_tree_knn(tt_ref, fp(src), len(src), 1, fp(idx1), fp(d1)), threads)
    cpu = None
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    out = {"host": {"cpu_model": cpu, "nproc": os.cpu_count(), "python": platform.python_version()},
           "protocol": "2 warm-ups, median of 10; identical inputs (cfg3 scan 131,072 pts, submap 500,000 pts)",
           "port": "oracle/cpu_ref.cpp (-O2 -fopenmp)", "reference": "oracle/_ref: the reference's nanoflann_impl.hpp "
           "(-O2 -fopenmp), KDTreeSingleIndexAdaptor<SO3_Adaptor<float>, ..., 3, int>, leaf 100",
           "stages": rows, "all_within_25pct": all(r["within_25pct"] for r in rows)}
    with open(os.path.join(HERE, "profiles", "r03_cpu_validation.json"), "w") as f:
        json.dump(out, f, indent=1)
    md = ["# CPU baseline validation (round 3)", "", f"Host: {cpu}, {os.cpu_count()} CPUs. {out['protocol']}.", "",
          "| stage | points | threads | port ms | reference ms | port / reference |", "|---|---:|---:|---:|---:|---:|"]
    for r in rows:
        md.append(f"| {r['stage']} | {r['points']} | {r['threads']} | {r['port_ms']} | {r['reference_ms']} | {r['ratio']} |")
    md.append("")
    md.append(f"All stages within +-25 %: {out['all_within_25pct']}")
    with open(os.path.join(HERE, "profiles", "r03_cpu_validation.md"), "w") as f:
        f.write("\n".join(md) + "\n")


if __name__ == "__main__":
    main()
