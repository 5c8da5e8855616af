"""Are the device covariances bit-identical to the oracle's (k = 10, PLANE)?  Ray-cast scans (tied queries
resolved in nanoflann's order, order-free inner ties kept from the Morton order) and a tied lattice."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import TARGET, scene  # noqa: E402
from oracle import oracle as O  # noqa: E402

frames = scene.loop_sequence(64, 2048, 0, 4, device=0)[0]
lat = np.stack(np.meshgrid(np.arange(24), np.arange(24), np.arange(5), indexing="ij"), -1).reshape(-1, 3)
clouds = [("scan%d" % i, f) for i, f in enumerate(frames)] + [("lattice", lat.astype(np.float32) * np.float32(0.25))]
c = P.Context(0)
c.set_params(P.default_params(k_correspondences=10))
for name, pts in clouds:
    c.set_target(pts)
    c.compute_covariances(TARGET)
    got = c.get_covariances(TARGET)
    ref = O.covariances(pts, 10, threads=16)
    d = np.abs(got - ref).max(axis=1)
    print(name, "points", len(pts), "not bit-identical", int((got != ref).any(axis=1).sum()), "max |diff|", float(d.max()))
