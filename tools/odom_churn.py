"""The odometry chain (cfg 5, 300 frames, bench parameters) in a fresh process (argv[1] == "bare"), after
10 contexts made and destroyed ("churn"), after the headline leg's 20 aligns ("cfg3"), after the cfg3 problem
built but not aligned ("cfg3build"), or after 2 GiB of device memory taken and released ("alloc"): what in the
process's history changes it?"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import types  # noqa: E402

import bench  # noqa: E402
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import odometry as OD  # noqa: E402

args = types.SimpleNamespace(batch_frames=300)
frames = bench.cfg5_frames(args, 0, 300, 0)
mode = sys.argv[1]
if mode == "churn":
    for _ in range(10):
        P.Context(0).close()
elif mode in ("cfg3", "cfg3build"):
    import legs  # noqa: E402
    legs.cfg3(20 if mode == "cfg3" else 0)
elif mode == "alloc":
    import torch
    x = torch.empty(2 << 30, dtype=torch.uint8, device="cuda:0")
    x.fill_(1)
    torch.cuda.synchronize()
    del x
    torch.cuda.empty_cache()
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
