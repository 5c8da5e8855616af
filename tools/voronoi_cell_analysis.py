"""Feasibility probe for an exact per-target cell -> candidate-list structure
(S2M correspondence search amortised over the submap).

For the cfg3 problem (queries at the guess pose and at the true pose) and
leaf cell sizes s: the cell's dominators are the nearest target points of
its 8 corners and centre; D = min over dominators of the farthest-corner
distance bounds every query's nearest distance in the cell; the candidates
are the target points within box distance min(D, cap) of the cell that no
dominator beats at every corner (a point strictly beaten at all corners is
beaten on the whole box, so it is never any query's nearest point).
Prints the list-size distribution per query.
"""
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402

CORN = np.array([[i, j, k] for i in (0, 1) for j in (0, 1) for k in (0, 1)], np.float64)


def cell_lists(tree, pts, lo, s, cap):
    """lo: (m,3) cell lower corners.  Returns list sizes (m,) and the unpruned ball sizes."""
    m = len(lo)
    corners = lo[:, None, :] + s * CORN[None]            # m,8,3
    cen = lo + 0.5 * s
    qp = np.concatenate([corners.reshape(-1, 3), cen], 0)
    _, nn = tree.query(qp)
    dom = np.concatenate([nn[:8 * m].reshape(m, 8), nn[8 * m:, None]], 1)   # m,9
    h = 0.5 * s * np.sqrt(3.0)
    sizes = np.zeros(m, np.int64)
    ball = np.zeros(m, np.int64)
    for c in range(m):
        dp = pts[dom[c]]                                    # 9,3
        cc = corners[c]                                     # 8,3
        d2 = ((cc[:, None, :] - dp[None, :, :]) ** 2).sum(-1)   # 8 corners x 9 dominators
        D = np.sqrt(d2.max(0).min())
        R = min(D, cap)
        idx = tree.query_ball_point(cen[c], R + h)
        ball[c] = len(idx)
        if not idx:
            continue
        P = pts[idx]
        bd = np.maximum(np.maximum(lo[c] - P, P - (lo[c] + s)), 0.0)
        keep = (bd ** 2).sum(1) <= R * R * (1 + 1e-6)
        P = P[keep]
        pc = ((cc[None, :, :] - P[:, None, :]) ** 2).sum(-1)          # n,8
        # dominated by dominator j iff d(corner, dom_j) < d(corner, p) at every corner
        dom_all = (d2[None, :, :] < pc[:, :, None]).all(1)           # n,9
        sizes[c] = int((~dom_all.any(1)).sum())
    return sizes, ball


def main():
    prob = bench.build_problem()
    sub = np.concatenate(prob["keyframes"])[prob["subset"]].astype(np.float64)
    src = prob["source"].astype(np.float64)
    tree = cKDTree(sub)
    cap = 2.0
    rng = np.random.default_rng(0)
    for name, T in (("guess", prob["guess"]), ("true", prob["T_true"])):
        q = src @ T[:3, :3].T.astype(np.float64) + T[:3, 3]
        dq, _ = tree.query(q, distance_upper_bound=cap)
        for s in (0.05, 0.1, 0.2):
            cell = np.floor(q / s).astype(np.int64)
            uc, inv = np.unique(cell, axis=0, return_inverse=True)
            inv = inv.ravel()
            pick = rng.choice(len(uc), size=min(len(uc), 6000), replace=False)
            sizes, ball = cell_lists(tree, sub, uc[pick] * s, s, cap)
            # per-query weighting: how many queries fall in each sampled cell
            w = np.bincount(inv, minlength=len(uc))[pick]
            per_q = np.repeat(sizes, w)
            per_qb = np.repeat(ball, w)
            print(f"[{name}] s={s}: cells {len(uc)} (q/cell {len(q) / len(uc):.2f}); pruned list per query "
                  f"pct 50/90/99 {np.percentile(per_q, [50, 90, 99]).round(1)} max {per_q.max()} "
                  f"mean {per_q.mean():.1f}; ball mean {per_qb.mean():.1f}", flush=True)


if __name__ == "__main__":
    main()
