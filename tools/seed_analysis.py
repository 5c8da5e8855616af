"""Developer analysis (CPU): quality of the seed kernel's Morton-window bound
on the cfg3 problem at the guess pose, against the true nearest distance
(scipy cKDTree), per 16-query sub-group; and what the probe windows
("Probe seeds") give for the slowest sub-groups.
Restates the device Morton key (search.hpp morton_key, k_bbox_final's
uniform scale) and sub-grouping (sorted source, 16 queries)."""
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic_direct_lidar_odometry_amd import scene  # noqa: E402


def spread(x):
    x = x & np.uint64(0x1fffff)
    for sh, m in ((32, 0x1f00000000ffff), (16, 0x1f0000ff0000ff), (8, 0x100f00f00f00f00f),
                  (4, 0x10c30c30c30c30c3), (2, 0x1249249249249249)):
        x = (x | (x << np.uint64(sh))) & np.uint64(m)
    return x


def quant(p):
    lo = p.min(0)
    return lo, np.float32(2097151.0) / (p.max(0) - lo).max()


def mkey(p, lo, sc):
    q = np.clip((p - lo) * sc, 0, 2097151).astype(np.uint64)
    return spread(q[:, 0]) | (spread(q[:, 1]) << np.uint64(1)) | (spread(q[:, 2]) << np.uint64(2))


prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
sub = np.concatenate(prob["keyframes"])[prob["subset"]][:, :3].astype(np.float32)
src = prob["source"][:, :3].astype(np.float32)
G = prob["guess"]
S = src[np.argsort(mkey(src, *quant(src)), kind="stable")]
tlo, tsc = quant(sub)
tk = mkey(sub, tlo, tsc)
order = np.argsort(tk, kind="stable")
T, TK = sub[order], tk[order]
Q = (S.astype(np.float64) @ G[:3, :3].T + G[:3, 3]).astype(np.float32)
d1, _ = cKDTree(T).query(Q)
lb = np.searchsorted(TK, mkey(Q, tlo, tsc))
seed = np.full(len(Q), np.inf)
seedj = np.full(len(Q), -1)
for o in range(-16, 16):   # the 32-point window around the lower bound
    jj = np.clip(lb + o, 0, len(T) - 1)
    dd = ((Q - T[jj]) ** 2).sum(1)
    b = dd < seed
    seed[b], seedj[b] = dd[b], jj[b]
seed = np.sqrt(np.minimum(seed, 4.0))
ng = len(Q) // 16
bound = np.zeros(len(Q))
for g in range(ng):   # group sharing: the other queries' candidates
    s = slice(g * 16, g * 16 + 16)
    cand = T[seedj[s][seedj[s] >= 0]]
    share = np.sqrt(((Q[s][:, None] - cand[None]) ** 2).sum(2).min(1)) if len(cand) else np.full(16, 2.0)
    bound[s] = np.minimum(seed[s], share)
gmax, nnmax = bound.reshape(-1, 16).max(1), d1.reshape(-1, 16).max(1)
for thr in (0.5, 1.0, 1.5):
    m = gmax > thr
    print(f"sub-groups with a bound above {thr} m: {m.sum()} of {ng}; of those, every true distance below {thr / 2} m: "
          f"{(nnmax[m] < thr / 2).sum()}")


def probes(g, d=0.5):
    s = slice(g * 16, g * 16 + 16)
    c, dd = Q[s][0], d * 0.70710678
    offs = np.array([[d, 0, 0], [-d, 0, 0], [0, d, 0], [0, -d, 0], [0, 0, d], [0, 0, -d], [dd, dd, 0], [-dd, -dd, 0]],
                    np.float32)
    lbp = np.searchsorted(TK, mkey((c + offs).astype(np.float32), tlo, tsc))
    cand = np.concatenate([np.clip(x - 4 + np.arange(8), 0, len(T) - 1) for x in lbp])
    return np.sqrt(((Q[s][:, None] - T[cand][None]) ** 2).sum(2).min(1))


for g in np.argsort(-(gmax - nnmax))[:8]:
    s = slice(g * 16, g * 16 + 16)
    print(f"sub-group {g}: true max {nnmax[g]:.2f} m, window bound max {gmax[g]:.2f} m, "
          f"with probes max {np.minimum(bound[s], probes(g)).max():.2f} m")
