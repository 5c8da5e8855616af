"""Which per-frame input of the odometry chain differs between the GPU driver and oracle/odom_ref.py?  For the
first frames of the cfg 5 loop: the preprocessed scan (crop + voxel, device vs the PCL restatement) compared as
sets of exact bit patterns, and the k = 10 covariances of the oracle's scan (device vs oracle) per point.
Usage: python tools/chain_inputs.py [frames]"""
import sys

import numpy as np

sys.path.insert(0, ".")
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import TARGET, scene  # noqa: E402
from dynamic_direct_lidar_odometry_amd import odometry as OD  # noqa: E402
from oracle import odom_ref as R  # noqa: E402
from oracle import oracle as O  # noqa: E402


def rows(a):
    a = np.ascontiguousarray(a, np.float32)
    v = a.view(np.uint32).reshape(len(a), 3)
    return {tuple(r) for r in v}


n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
frames = scene.loop_sequence(64, 2048, 0, n, device=0)[0]
p = OD.default_odom_params()
ref = R.OdomRef(p, threads=16)
ctx = P.Context(0, P.default_params(k_correspondences=10))
for i, f in enumerate(frames):
    a = ref._preprocess(f)
    g = OD.preprocess(f, p.crop_size if p.crop_use else 0.0, p.vf_scan_res if p.vf_scan_use else 0.0)
    ra, rg = rows(a), rows(g)
    print(f"frame {i}: oracle {len(a)} pts, device {len(g)} pts, only oracle {len(ra - rg)}, only device "
          f"{len(rg - ra)}", flush=True)
    if ra != rg:
        oa = np.array(sorted(ra - rg), np.uint32).view(np.float32)[:5]
        og = np.array(sorted(rg - ra), np.uint32).view(np.float32)[:5]
        print("   oracle-only e.g.", oa.tolist(), "\n   device-only e.g.", og.tolist())
    co = O.covariances(a, 10, threads=16)
    ctx.set_target(a)
    ctx.compute_covariances(TARGET)
    cg = ctx.get_covariances(TARGET)
    diff = np.any(cg.view(np.uint64) != co.view(np.uint64), axis=1)
    print(f"   covariances: {int(diff.sum())} of {len(a)} points differ (max abs {float(np.abs(cg - co).max()):.3e})",
          flush=True)
ctx.close()
