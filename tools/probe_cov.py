"""Developer probe: split the covariance pass (k=10, 131k points) into kNN and regularization cost."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import scene, SOURCE, TARGET

src, tgt, _ = scene.s2s_pair(64, 2048, 2)
c = P.Context(0)
for reg, name in ((P.REG_PLANE, "PLANE"), (P.REG_NONE, "NONE"), (P.REG_MIN_EIG, "MIN_EIG")):
    for k in (10, 20):
        c.set_params(P.default_params(k_correspondences=k, regularization=reg))
        c.set_source(src)
        c.compute_covariances(SOURCE); c.synchronize()
        ts = []
        for _ in range(5):
            c.set_source(src); c.synchronize()
            t = time.perf_counter(); c.compute_covariances(SOURCE); c.synchronize(); ts.append(time.perf_counter() - t)
        print(f"covariances {name} k={k}: {1e3*np.median(ts):.3f} ms")
c.set_params(P.default_params(k_correspondences=10))
c.set_target(tgt)
for k in (1, 10, 20):
    ts = []
    for _ in range(5):
        t = time.perf_counter(); c.knn_target(tgt, k) if hasattr(c, "knn_target") else None; ts.append(time.perf_counter() - t)
    print(f"knn_target self k={k}: {1e3*np.median(ts):.3f} ms (incl. D2H of results)")
