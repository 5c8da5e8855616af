"""Odometry pass order vs. host-to-device upload time: the same 1000 frames
driven four times (nanoflann, nanoflann, Morton, nanoflann tie order) with
DDLO_ODOM_TIMING=1, to tell a first-pass host-memory effect from a tie-order
effect (diagnostics, used via gpurun)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DDLO_ODOM_TIMING"] = "1"
from dynamic_direct_lidar_odometry_amd import odometry as OD, scene  # noqa: E402

frames = scene.loop_sequence(64, 2048, 0, 1000, device=0)[0]
for tag, exact in (("nanoflann#1", "1"), ("nanoflann#2", "1"), ("morton", "0"), ("nanoflann#3", "1")):
    os.environ["DDLO_TIE_EXACT"] = exact
    odo = OD.Odometry(0)
    t0 = time.perf_counter()
    for f in frames:
        odo.process(f)
    el = time.perf_counter() - t0
    print(f"{tag}: {1e3 * el / len(frames):.4f} ms/frame", flush=True)
    sys.stderr.write(f"--- {tag}\n")
    sys.stderr.flush()
    odo.close()
