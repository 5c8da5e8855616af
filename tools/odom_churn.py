"""The odometry chain (cfg 5, 300 frames, bench parameters) in a fresh process (argv[1] == "bare") or after
10 contexts made and destroyed (argv[1] == "churn"): does the process's stream / queue history change it?"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import types  # noqa: E402

import bench  # noqa: E402
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import odometry as OD  # noqa: E402

args = types.SimpleNamespace(batch_frames=300)
frames = bench.cfg5_frames(args, 0, 300, 0)
if sys.argv[1] == "churn":
    for _ in range(10):
        P.Context(0).close()
w = OD.Odometry(0)
for f in frames[:4]:
    w.process(f)
w.close()
o = OD.Odometry(0)
t0 = time.perf_counter()
for f in frames:
    o.process(f)
el = time.perf_counter() - t0
o.close()
print(sys.argv[1], f"{1e3 * el / len(frames):.4f} ms/frame", flush=True)
