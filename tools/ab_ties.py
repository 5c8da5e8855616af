"""A/B of the correspondence tie detection (nanoflann order vs Morton order)
on cfg3 (S2M LM) with the target's candidate cells (the bench's path) and
with the walk, and on cfg2 (S2S, 20 GN iterations, the walk): the same
contexts, the order switched with gicp_set_tie_order, interleaved
repetitions."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET, scene  # noqa: E402


def timed(c, g, n):
    c.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        out, res = c.align(g)
    c.synchronize()
    return (time.perf_counter() - t) / n * 1e3, res


def main():
    prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
    sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
    def cfg3_ctx(grid):
        c = P.Context(0)
        c.set_target_grid(grid)
        c.set_params(P.default_params(k_correspondences=10))
        c.set_target(sub)
        c.compute_covariances(TARGET)
        c.set_source(prob["source"])
        c.compute_covariances(SOURCE)
        c.set_params(P.default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32,
                                      transformation_epsilon=0.01))
        return c

    c = cfg3_ctx(P.GRID_ON)
    w = cfg3_ctx(P.GRID_OFF)
    g = prob["guess"].astype(np.float32)
    src, tgt, _ = scene.s2s_pair(64, 2048, 2)
    d = P.Context(0)
    d.set_target_grid(P.GRID_OFF)
    d.set_params(P.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=20,
                                  optimizer=P.GAUSS_NEWTON, fixed_iterations=20))
    d.set_target(tgt)
    d.set_source(src)
    d.compute_covariances(SOURCE)
    d.compute_covariances(TARGET)
    for ctx, gg in ((c, g), (w, g), (d, None)):
        for _ in range(5):
            ctx.align(gg)
    rows = {(k, o): [] for k in ("cfg3 cells", "cfg3 walk", "cfg2") for o in (1, 0)}
    for rep in range(7):
        for order in (1, 0):
            for ctx in (c, w, d):
                ctx.set_tie_order(bool(order))
            ms, r = timed(c, g, 200)
            rows[("cfg3 cells", order)].append(ms)
            msw, rw = timed(w, g, 100)
            rows[("cfg3 walk", order)].append(msw)
            ms2, r2 = timed(d, None, 10)
            rows[("cfg2", order)].append(ms2)
            if rep == 0:
                print(f"order {order}: cfg3 iters {r.iterations_run} ties {r.ties_resolved} (walk {rw.ties_resolved}); "
                      f"cfg2 ties {r2.ties_resolved}", flush=True)
    for k, v in rows.items():
        print(f"{k[0]} {'nanoflann' if k[1] else 'morton'}: median {np.median(v):.4f} ms  {np.round(v, 4).tolist()}",
              flush=True)
    for k in ("cfg3 cells", "cfg3 walk", "cfg2"):
        a, b = np.median(rows[(k, 1)]), np.median(rows[(k, 0)])
        print(f"{k}: tie detection +{100 * (a / b - 1):.2f} %", flush=True)


if __name__ == "__main__":
    main()
