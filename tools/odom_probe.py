"""cfg5's odometry chain with the S2M target's candidate cells off / auto / on:
ms per frame, keyframes, final pose (identical poses expected across modes).

python tools/odom_probe.py [--frames 400]
"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
from dynamic_direct_lidar_odometry_amd import odometry as OD  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--modes", default="0,1,2,0")
    args = ap.parse_args()
    frames = bench.cfg5_frames(args, 0, args.frames, 0)
    w = OD.Odometry(0)
    for f in frames[:4]:
        w.process(f)
    w.close()
    poses = {}
    for mode in (int(m) for m in args.modes.split(",")):
        o = OD.Odometry(0, OD.default_odom_params(s2m_target_grid=mode))
        t0 = time.perf_counter()
        kfs = 0
        for f in frames:
            r = o.process(f)
            kfs += r.keyframe_added
        el = time.perf_counter() - t0
        pose = r.pose()
        o.close()
        same = "" if mode not in poses else f" same_as_before={np.array_equal(poses[mode], pose)}"
        poses.setdefault(mode, pose)
        print(f"s2m_target_grid={mode} ms/frame {1e3 * el / len(frames):.4f} keyframes {kfs} "
              f"identical_to_off={np.array_equal(pose, poses.get(0, pose))}{same}", flush=True)


if __name__ == "__main__":
    main()
