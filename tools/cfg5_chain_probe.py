"""cfg 5 chain probe (CPU, oracle only): run oracle/odom_ref.py over frames
[first, first + count) (stride s) of the 1000-frame plaza loop and report per
frame the keyframe count, submap changes and whether a submap holds a
keyframe that the knn step did not select (a hull-driven submap).  Used to
choose the GPU parity segment of tests/test_gpu_odom_long.py.

    python tools/cfg5_chain_probe.py --first 0 --count 300 --stride 1 [--gpu]
"""
import argparse
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic_direct_lidar_odometry_amd import scene  # noqa: E402
from oracle import odom_ref as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--count", type=int, default=300)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--gpu", action="store_true", help="GPU ray caster for the frames")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--set", action="append", default=[], help="odometry parameter override name=value")
    a = ap.parse_args()
    from dynamic_direct_lidar_odometry_amd import odometry as OD
    kw = {}
    for kv in a.set:
        k, v = kv.split("=")
        kw[k] = float(v) if "." in v else int(v)
    p = OD.default_odom_params(**kw)
    ref = R.OdomRef(p, threads=a.threads)
    idx = list(range(a.first, a.first + a.count * a.stride, a.stride))
    t0 = time.time()
    hull_changes = 0
    for n, k in enumerate(idx):
        f = scene.loop_sequence(64, 2048, k, 1, gpu=a.gpu)[0][0]
        o = ref.process(f)
        extra = []
        if o["status"] == 0:
            nk = len(ref.keyframes) - o["keyframe_added"]   # the keyframes the submap was selected from
            c = ref.T_s2s[:3, 3]
            ds = [math.sqrt(sum((float(c[j]) - float(kf[0][j])) ** 2 for j in range(3))) for kf in ref.keyframes[:nk]]
            knn = []
            R.push_submap_indices(ds, p.submap_knn, list(range(nk)), knn)
            extra = sorted(set(o["submap"]) - set(knn))
            if extra and o["submap_changed"]:
                hull_changes += 1
        print(f"frame {k} st {o['status']} nk {len(ref.keyframes)} kf+ {o['keyframe_added']} chg {o['submap_changed']} "
              f"sub {o.get('submap')} hull-only {extra} cvx {len(ref.keyframe_convex)} ccv {len(ref.keyframe_concave)} "
              f"t {time.time() - t0:.1f}s", flush=True)
    print(f"hull-driven submap changes: {hull_changes}")


if __name__ == "__main__":
    main()
