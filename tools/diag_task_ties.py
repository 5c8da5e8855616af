"""Diagnostics (development): task-based kNN covariances on a tied lattice, repeated, vs the oracle."""
import os
import sys
import numpy as np
sys.path.insert(0, ".")
import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import TARGET
from oracle import oracle as O

rng = np.random.default_rng(7)
lattice = rng.integers(0, 40, size=(20000, 3)).astype(np.float32)
k = int(sys.argv[1]) if len(sys.argv) > 1 else 10
ref = O.covariances(lattice, k)
scale = max(np.abs(ref).max(), 1.0)
_, d = O.knn(lattice, lattice, k + 1)
for tasks in ("1", "0") * 5:
    os.environ["DDLO_COV_TASKS"] = tasks
    c = P.Context(0)
    c.set_params(P.default_params(k_correspondences=k))
    c.set_target(lattice)
    try:
        c.compute_covariances(TARGET)
    except P.GicpError as e:
        print("tasks", tasks, "ERROR", e)
        c.close()
        continue
    got = c.get_covariances(TARGET)
    c.close()
    bad = np.where(np.abs(got - ref).max(axis=1) > 1e-12 * scale)[0]
    print("tasks", tasks, "bad", len(bad), bad[:12].tolist())
    for b in bad[:3]:
        print("   d", d[b].tolist())
