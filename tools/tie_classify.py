"""Are the queries the covariance pass flags as tied (k = 10) exact distance
ties?  GPU frames of the cfg 5 loop, the flagged queries dumped by the
library (DDLO_TIE_DEBUG + DDLO_TIE_DUMP), and every query's fp32 neighbour
distances (dist2's op order) recomputed on the host: a k-th tie (d_k = d_k+1)
or an inner tie (two equal distances among the k).

    python tools/tie_classify.py [frames]
"""
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

DUMP = os.path.abspath("gpurun_out/tie_dump.txt")
os.environ["DDLO_TIE_DEBUG"] = "1"
os.environ["DDLO_TIE_DUMP"] = DUMP
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import SOURCE, scene  # noqa: E402


def true_ties(pts, k):
    x = pts.astype(np.float64)
    _, idx = cKDTree(x).query(x, k=k + 6)
    C = pts[idx]
    dx = pts[:, None, 0] - C[..., 0]
    dy = pts[:, None, 1] - C[..., 1]
    dz = pts[:, None, 2] - C[..., 2]
    d = (dx * dx + dy * dy) + dz * dz
    d = np.sort(d, axis=1)
    kth = d[:, k - 1] == d[:, k]
    inner = np.any(d[:, 1:k] == d[:, :k - 1], axis=1)
    return kth, inner


def main():
    nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    os.makedirs("gpurun_out", exist_ok=True)
    if os.path.exists(DUMP):
        os.remove(DUMP)
    frames = scene.loop_sequence(64, 2048, 0, nfr, device=0)[0]
    cpu = scene.loop_sequence(64, 2048, 0, 1, gpu=False)[0][0]
    print("GPU frame 0 == host ray caster frame 0:", cpu.shape == frames[0].shape and bool(np.array_equal(cpu, frames[0])),
          "max diff", float(np.abs(cpu - frames[0]).max()) if cpu.shape == frames[0].shape else None)
    c = P.Context(0)
    c.set_params(P.default_params(k_correspondences=10))
    for f in frames:
        c.set_source(f)
        c.compute_covariances(SOURCE)
    c.close()
    lines = open(DUMP).read().split("\n")
    for f, line in zip(frames, lines):
        v = [int(t) for t in line.split()]
        n, k, flagged = v[0], v[1], np.array(v[2:], np.int64)
        kth, inner = true_ties(f, k)
        truth = np.nonzero(kth | inner)[0]
        u, cnt = np.unique(f, axis=0, return_counts=True)
        fl = np.zeros(n, bool)
        fl[flagged[flagged >= 0]] = True
        print(f"n {n}: flagged {len(flagged)}, true ties {len(truth)} (k-th {kth.sum()}, inner {inner.sum()}), "
              f"flagged & true {np.sum(fl & (kth | inner))}, true not flagged {np.sum(~fl & (kth | inner))}, "
              f"duplicate points {np.sum(cnt > 1)}")
        bad = np.nonzero(fl & ~(kth | inner))[0][:5]
        for q in bad:
            x = f.astype(np.float64)
            dd = np.sort(((f[q] - f) ** 2).sum(1))[:k + 2]
            print("   spurious", q, f[q], "sorted d", dd)


if __name__ == "__main__":
    main()
