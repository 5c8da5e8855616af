"""Developer timing: where a cfg 3 align's wall time goes on the host side.
Per align: wall time of the C-ABI call (ctypes, cached pointers), the
device span res.device_ms (event before the graph -> event after the final
chunk) and their difference (host + launch latency)."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET, scene  # noqa: E402

prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
c = P.Context(0)
c.set_target_grid(P.GRID_ON)   # the headline path (candidate cells, built at the first align)
c.set_params(P.default_params(k_correspondences=10))
c.set_target(sub)
c.compute_covariances(TARGET)
c.set_source(prob["source"])
c.compute_covariances(SOURCE)
c.set_params(P.default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32,
                              transformation_epsilon=0.01))
g = np.ascontiguousarray(prob["guess"], np.float32)
out = np.zeros((4, 4), np.float32)
res = P.GicpResult()
gp, op, rp = g.ctypes.data, out.ctypes.data, C.pointer(res)
f = c.L.gicp_align
for _ in range(10):
    f(c.h, gp, op, rp)
N = 300
wall = np.zeros(N)
dev = np.zeros(N)
for i in range(N):
    t = time.perf_counter()
    f(c.h, gp, op, rp)
    wall[i] = time.perf_counter() - t
    dev[i] = res.device_ms
t = time.perf_counter()
for i in range(N):
    f(c.h, gp, op, rp)
loop = (time.perf_counter() - t) / N
t = time.perf_counter()
for i in range(N):
    c.align(g)
loop_py = (time.perf_counter() - t) / N
wall *= 1e6
dev *= 1e3
print(f"{os.environ.get('DDLO_GICP_LIB', 'lib')} spin={os.environ.get('DDLO_SPIN_WAIT', '0')}: "
      f"call wall {np.median(wall):.1f} us (mean {wall.mean():.1f}), device span {np.median(dev):.1f} us, "
      f"host+launch {np.median(wall - dev):.1f} us; back-to-back C-ABI {loop * 1e6:.1f} us/align, "
      f"Context.align {loop_py * 1e6:.1f} us/align, iters {res.iterations_run}")
