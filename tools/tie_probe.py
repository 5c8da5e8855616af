"""Tied correspondences of the headline problem (cfg3): ties resolved per align and the align time with the
nanoflann tie order (default) and the Morton order (no resolution)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET  # noqa: E402

prob = bench.build_problem()
sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
tcov = np.ascontiguousarray(bench.keyframe_covariances(lambda: P.Context(0), prob["keyframes"])[prob["subset"]])
for order in (1, 0):
    with P.default_option(P.OPT_TIE_ORDER, order):
        c = P.Context(0)
        c.set_params(P.default_params(k_correspondences=10))
        c.set_source(prob["source"])
        c.compute_covariances(SOURCE)
        c.set_params(P.default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32,
                                      transformation_epsilon=0.01))
        c.set_target_grid(P.GRID_ON)
        c.set_target(sub)
        c.set_covariances(TARGET, tcov)
        g = prob["guess"].astype(np.float32)
        _, r = c.align(g)
        for _ in range(5):
            c.align(g)
        c.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            _, r = c.align(g)
        c.synchronize()
        el = (time.perf_counter() - t0) / 50
        print(f"tie order {order}: {1e3 * el:.4f} ms/align, iterations {r.iterations_run}, ties resolved {r.ties_resolved}")
        c.close()
