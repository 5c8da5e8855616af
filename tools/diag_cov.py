"""Diagnostics (development): covariance rows where the device differs from the oracle."""
import sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import TARGET
from oracle import oracle as O
from conftest import load_golden

np.set_printoptions(precision=17, linewidth=200)
g = load_golden("gicp_s2s.npz")
rng = np.random.default_rng(7)
lattice = rng.integers(0, 40, size=(20000, 3)).astype(np.float32)
for name, cloud, k in (("scan", g["src"], 7), ("lattice", lattice, 10)):
    for reg in (0, 3):
        ref = O.covariances(cloud, k, reg=reg)
        c = P.Context(0)
        c.set_params(P.default_params(k_correspondences=k, regularization=reg))
        c.set_target(cloud)
        c.compute_covariances(TARGET)
        got = c.get_covariances(TARGET)
        c.close()
        scale = max(np.abs(ref).max(), 1.0)
        bad = np.where(np.abs(got - ref).max(axis=1) > 1e-12 * scale)[0]
        print(name, "k", k, "reg", reg, "bad", len(bad), bad[:10])
        idx, d = O.knn(cloud, cloud[bad], k + 1)
        for j, b in enumerate(bad[:5]):
            print("  row", b, "d", d[j].tolist())
            print("   gpu", got[b])
            print("   ref", ref[b])
