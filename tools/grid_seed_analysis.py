"""Developer analysis (CPU): seed bounds of the correspondence search on the
cfg3 problem at the guess pose -- the device's Morton window + group sharing
(+ probes) against a per-target dense cell grid that stores one target point
per cell (empty cells dilated from their neighbours), + group sharing.
Per 16-query sub-group: the largest seed bound (what sizes the walk's union
box) against the true nearest distance.  Restates tools/seed_analysis.py's
window seed."""
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from seed_analysis import Q, T, bound, d1, probes  # noqa: E402  (runs the window analysis)

ng = len(Q) // 16
cap = 2.0


def grid_seed(cell, dil):
    lo = T.min(0) - 1e-3
    dims = np.ceil((T.max(0) - lo) / cell).astype(int) + 1
    idx = np.floor((T - lo) / cell).astype(int)
    flat = (idx[:, 0] * dims[1] + idx[:, 1]) * dims[2] + idx[:, 2]
    g = np.full(dims[0] * dims[1] * dims[2], -1, np.int64)
    g[flat] = np.arange(len(T))   # last writer wins (any point of the cell)
    g = g.reshape(dims)
    for _ in range(dil):   # empty cells take a face neighbour's point
        e = g < 0
        for ax in range(3):
            for sh in (1, -1):
                nb = np.roll(g, sh, axis=ax)
                take = e & (nb >= 0) & (g < 0)
                g[take] = nb[take]
    qi = np.floor((Q - lo) / cell).astype(int)
    inside = np.all((qi >= 0) & (qi < dims), axis=1)
    qi = np.clip(qi, 0, dims - 1)
    j = g[qi[:, 0], qi[:, 1], qi[:, 2]]
    ok = inside & (j >= 0)
    seed = np.full(len(Q), cap)
    seed[ok] = np.sqrt(((Q[ok] - T[j[ok]]) ** 2).sum(1))
    seed = np.minimum(seed, cap)
    bnd = np.zeros(len(Q))
    for k in range(ng):
        s = slice(k * 16, k * 16 + 16)
        jj = j[s][ok[s]]
        share = np.sqrt(((Q[s][:, None] - T[jj][None]) ** 2).sum(2).min(1)) if len(jj) else np.full(16, cap)
        bnd[s] = np.minimum(seed[s], share)
    return bnd, dims


def report(name, b):
    gm = b.reshape(-1, 16).max(1)
    vol = (gm ** 3).sum()
    print(f"{name:28s} group-max bound mean {gm.mean():.3f} p90 {np.percentile(gm, 90):.3f} p99 {np.percentile(gm, 99):.3f}"
          f" >1m {np.sum(gm > 1.0):5d} >1.5m {np.sum(gm > 1.5):5d}  sum(ball^3) {vol:9.1f}")


report("true NN (floor)", d1)
report("window + sharing", bound)
pb = bound.copy()
gmax = bound.reshape(-1, 16).max(1)
for k in np.nonzero(gmax > 1.0)[0]:
    s = slice(k * 16, k * 16 + 16)
    pb[s] = np.minimum(pb[s], probes(k))
report("window + sharing + probes", pb)
for cell in (0.1, 0.2, 0.3, 0.5):
    for dil in (2, 4, 8):
        b, dims = grid_seed(cell, dil)
        report(f"grid {cell} m dil {dil} ({dims.prod() / 1e6:.1f}M)", np.minimum(b, pb) if False else b)
        report(f"  grid+window+probes", np.minimum(b, pb))
