"""Covariance timing on one 64x2048 ray-cast scan (131k points): k = 10 / 20, nanoflann tie order on / off.
Wall time of gicp_compute_covariances (includes the tree build on the aux stream and the tie resolution)."""
import sys
import time
import numpy as np
sys.path.insert(0, ".")
import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import TARGET, scene

frames = scene.loop_sequence(64, 2048, 0, 6, device=0)[0]
out = {}
for k in (10, 20):
    for exact in (True, False):
        c = P.Context(0)
        c.set_params(P.default_params(k_correspondences=k))
        c.set_tie_order(exact)
        ts = []
        for f in frames:
            c.set_target(f)
            c.synchronize()
            t0 = time.perf_counter()
            c.compute_covariances(TARGET)
            ts.append(time.perf_counter() - t0)
        c.close()
        out[f"k{k}_{'nanoflann' if exact else 'morton'}_ms"] = round(1e3 * float(np.median(ts[1:])), 4)
print(out)
# device stage times (HIP events) of the nanoflann-order pass: covariance kernel, tree build, tie resolution
c = P.Context(0)
c.set_params(P.default_params(k_correspondences=10))
c.set_profiling(True)
st = []
for f in frames:
    c.set_target(f)
    c.compute_covariances(TARGET)
    c.synchronize()
    st.append(c.stage_times())
c.close()
print({"k10_stage_ms (cov, tree, resolve)": [round(float(v), 4) for v in np.median(np.array(st[1:]), axis=0)]})
