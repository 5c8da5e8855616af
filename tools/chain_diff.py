"""Where do the odometry driver and oracle/odom_ref.py first part?  Runs both over the first N frames of the cfg 5
loop and prints, per frame, the largest difference of the S2S result (T_s2s_local), the S2M guess (T_s2s) and the
final pose (T), with both sides' iteration counts; then re-runs the first differing frame's S2S / S2M on each
side's own inputs to name the input that differs (scan, target covariances, submap, submap covariances, guess).
Usage: python tools/chain_diff.py [N]"""
import sys

import numpy as np

sys.path.insert(0, ".")
from dynamic_direct_lidar_odometry_amd import odometry as OD  # noqa: E402
from dynamic_direct_lidar_odometry_amd import scene  # noqa: E402
from oracle import odom_ref as R  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    frames = scene.loop_sequence(64, 2048, 0, n, device=0)[0]
    p = OD.default_odom_params()
    gpu = OD.Odometry(0, p)
    ref = R.OdomRef(p, threads=16)
    first = {}
    for i, f in enumerate(frames):
        g = gpu.process(f)
        o = ref.process(f)
        if g.status != OD.TRACKED:
            continue
        row = {}
        for name, gv, ov in (("T_s2s_local", g.T_s2s_local, o["T_s2s_local"]), ("T_s2s", g.T_s2s, o["T_s2s"]),
                             ("T", g.T, o["T"])):
            d = float(np.abs(np.array(gv, np.float64).reshape(4, 4) - np.asarray(ov, np.float64)).max())
            row[name] = d
            if d > 0 and name not in first:
                first[name] = i
        print(f"{i:4d} s2s it {g.s2s.iterations_run}/{o['s2s'].iterations_run} s2m it {g.s2m.iterations_run}/"
              f"{o['s2m'].iterations_run} kf {g.num_keyframes}/{o['num_keyframes']} chg {g.submap_changed} "
              + " ".join(f"{k} {v:.2e}" for k, v in row.items()), flush=True)
    print("first differing frame:", first, flush=True)
    gpu.close()


if __name__ == "__main__":
    main()
