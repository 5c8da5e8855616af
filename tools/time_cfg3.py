"""Developer timing: cfg3 S2M align ms/scan (LM, reference S2M params)."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dynamic_direct_lidar_odometry_amd as P  # noqa
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET, scene  # noqa

prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
c = P.Context(0)
c.set_params(P.default_params(k_correspondences=10))
c.set_target(sub); c.compute_covariances(TARGET)
c.set_source(prob["source"]); c.compute_covariances(SOURCE)
c.set_params(P.default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32, transformation_epsilon=0.01))
g = prob["guess"].astype(np.float32)
for _ in range(3):
    c.align(g)
c.synchronize()
t = time.perf_counter()
for _ in range(20):
    out, res = c.align(g)
c.synchronize()
ms = (time.perf_counter() - t) / 20 * 1e3
c.set_profiling(True)
_, r = c.align(g)
print(f"R0={os.environ.get('DDLO_TILE_R0','-')} split={os.environ.get('DDLO_SPLIT_EXTENT','-')}: {ms:.3f} ms/scan, iters {res.iterations_run}, linearize avg {r.linearize_ms / r.iterations_run * 1e3:.1f} us")
