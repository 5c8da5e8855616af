"""cfg3 with the target's candidate cells on and off: build statistics, ms/scan,
linearize time per active iteration (HIP events), walk sub-groups per align.

python tools/grid_probe.py [--aligns 100]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--aligns", type=int, default=100)
    args = ap.parse_args()
    prob = bench.build_problem()
    sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
    cov = bench.keyframe_covariances(lambda: P.Context(0), prob["keyframes"])[prob["subset"]]
    kw = dict(k_correspondences=10, max_correspondence_distance=2.0, max_iterations=32, transformation_epsilon=0.01)
    guess = prob["guess"].astype(np.float32)
    out = {}
    for name, mode in (("walk", P.GRID_OFF), ("grid", P.GRID_ON)):
        c = P.Context(0)
        c.set_params(P.default_params(**kw))
        c.set_target_grid(mode)
        c.set_target(sub)
        c.set_covariances(TARGET, np.ascontiguousarray(cov))
        c.set_source(prob["source"])
        c.compute_covariances(SOURCE)
        t0 = time.perf_counter()
        pose, res = c.align(guess)
        first = time.perf_counter() - t0
        info = c.grid_info()
        for _ in range(10):
            c.align(guess)
        c.synchronize()
        t0 = time.perf_counter()
        it = 0
        dev = []
        for _ in range(args.aligns):
            _, r = c.align(guess)
            it += r.iterations_run
            dev.append(r.device_ms)
        c.synchronize()
        el = time.perf_counter() - t0
        walk = c.lookup_walk_groups()
        c.set_profiling(True)
        lin, nit = 0.0, 0
        for _ in range(5):
            _, r = c.align(guess)
            lin += r.linearize_ms
            nit += r.iterations_run
        c.set_profiling(False)
        out[name] = {"ms_per_scan": 1e3 * el / args.aligns, "iters_per_scan": it / args.aligns,
                     "device_ms_median": float(np.median(dev)),
                     "linearize_us_per_iter": 1e3 * lin / max(nit, 1), "first_align_ms": 1e3 * first,
                     "walk_groups_last_align": walk, "pose": pose.tolist(), "grid": info}
        print(name, json.dumps({k: v for k, v in out[name].items() if k != "pose"}), flush=True)
        c.close()
    same = np.array_equal(np.array(out["walk"]["pose"]), np.array(out["grid"]["pose"]))
    print("identical poses:", same, flush=True)


if __name__ == "__main__":
    main()
