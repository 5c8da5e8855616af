"""Developer probe: tied queries per cloud of the k = 10 covariance kNN on cfg 5 frames (DDLO_TIE_DEBUG=1 prints them)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa
from dynamic_direct_lidar_odometry_amd import scene, Context, default_params, SOURCE  # noqa
frames = scene.loop_sequence(64, 2048, 0, 40, device=0)[0]
c = Context(0)
c.set_params(default_params(k_correspondences=10))
for f in frames:
    c.set_source(np.ascontiguousarray(f, np.float32))
    c.compute_covariances(SOURCE)
c.synchronize()
