"""Debug: covariance mismatches between GPU and oracle on the cfg3 source."""
import os, sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import numpy as np
import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import scene, SOURCE, TARGET
from oracle import oracle as O
prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
src = prob["source"]
c = P.Context(0)
c.set_params(P.default_params(k_correspondences=10))
c.set_source(src); c.compute_covariances(SOURCE)
g = c.get_covariances(SOURCE)
o = O.covariances(src, 10)
bad = np.where(np.abs(g - o).max(1) > 1e-12)[0]
print("bad", bad)
c.set_target(src)
gi, gd = c.knn_target(src[bad], 10)
oi, od = O.knn(src, src[bad], 10)
for r, i in enumerate(bad):
    print(i, "gpu", gi[r], gd[r]); print(i, "orc", oi[r], od[r])
    nb = src[oi[r]].astype(np.float64); X = nb - nb.mean(0); C = X.T @ X / 10
    print("eig", np.linalg.eigvalsh(C)); print("g", g[i]); print("o", o[i])
    for reg in range(5):
        pass
np.save("gpurun_out/badcov.npy", np.stack([g[bad], o[bad]]))
