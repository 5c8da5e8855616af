"""One bench leg's GPU workload alone, for rocprofv3 runs (kernel trace / PMC
passes) that must not mix legs.  Same problems and parameters as bench.py.

    python tools/legs.py cfg3 [aligns]     # the headline: S2M 131k -> 500k, candidate cells (built first)
    python tools/legs.py cfg2 [aligns]     # S2S 131k <-> 131k, 20 fixed GN iterations
    python tools/legs.py cfg4 [aligns]     # S2M 262k -> 2M, one-rank RCCL (groups mode)
    python tools/legs.py cfg5 [frames]     # per scan: index, k=10 covariances (+ nanoflann tree), S2S align
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET, scene  # noqa: E402


def cfg2(n):
    src, tgt, _ = scene.s2s_pair(64, 2048, 2)
    c = P.Context(0)
    c.set_target_grid(P.GRID_OFF)   # as bench.py's cfg2 leg (an S2S target is aligned against once)
    c.set_params(P.default_params(k_correspondences=10, max_correspondence_distance=1.0, optimizer=P.GAUSS_NEWTON,
                                  fixed_iterations=20, max_iterations=20))
    c.set_target(tgt)
    c.set_source(src)
    c.compute_covariances(SOURCE)
    c.compute_covariances(TARGET)
    for _ in range(n):
        c.align()
    c.synchronize()


def cfg3(n):
    prob = bench.build_problem()
    sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
    tcov = np.ascontiguousarray(bench.keyframe_covariances(lambda: P.Context(0), prob["keyframes"])[prob["subset"]])
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
    for _ in range(n):
        c.align(g)
    c.synchronize()


def cfg4(n):
    from dynamic_direct_lidar_odometry_amd.shard import ShardedGicp
    prob = scene.s2m_problem(128, 2048, 8, 2000000, 4)
    sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
    kcov = bench.keyframe_covariances(lambda: P.Context(0), prob["keyframes"], k=10)
    tcov = np.ascontiguousarray(kcov[prob["subset"]])
    c = P.Context(0)
    c.set_params(P.default_params(k_correspondences=10))
    c.set_source(prob["source"])
    c.compute_covariances(SOURCE)
    scov = c.get_covariances(SOURCE)
    c.close()
    params = P.default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32,
                              transformation_epsilon=0.01)
    sh = ShardedGicp(0, 0, 1, P.comm_unique_id(), params)
    sh.ctx.set_target_grid(P.GRID_ON)   # as bench.py's sharded leg: the cells built at the first align
    sh.set_target(sub, tcov)
    sh.set_source(prob["source"], scov)
    g = prob["guess"].astype(np.float32)
    for _ in range(n):
        sh.align(g)
    sh.ctx.synchronize()
    sh.close()


def cfg5(n):
    frames = scene.loop_sequence(64, 2048, 0, n + 1, device=0)[0]
    c = P.Context(0)
    c.set_params(P.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32,
                                  transformation_epsilon=0.01))
    c.set_target(frames[0])
    c.compute_covariances(TARGET)
    t0 = time.perf_counter()
    for f in frames[1:]:
        c.set_source(f)
        c.compute_covariances(SOURCE)
        c.align()
        c.swap_source_target()
    c.synchronize()
    print(f"cfg5 serial S2S: {1e3 * (time.perf_counter() - t0) / n:.3f} ms per scan")


if __name__ == "__main__":
    leg = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    {"cfg2": cfg2, "cfg3": cfg3, "cfg4": cfg4, "cfg5": cfg5}[leg](n)
