"""Feasibility probe for a per-target cell -> candidate-list structure (S2M).

For the cfg3 problem, queries at the guess pose and at the true pose; for cell
sizes s, the candidate list of the cell a query falls in is every target point
p with |p - c| <= min(d0(c) + h, cap) + h (c the centre, h the half diagonal,
d0 the centre's nearest distance): a superset of the points that can be the
nearest neighbour of any query inside the cell.  Prints the list-size
distribution over queries and the number of occupied cells.
"""
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402


def main():
    prob = bench.build_problem()
    sub = np.concatenate(prob["keyframes"])[prob["subset"]].astype(np.float64)
    src = prob["source"].astype(np.float64)
    tree = cKDTree(sub)
    cap = 2.0
    for name, T in (("guess", prob["guess"]), ("true", prob["T_true"])):
        q = src @ T[:3, :3].T.astype(np.float64) + T[:3, 3]
        dq, _ = tree.query(q, distance_upper_bound=cap)
        print(f"[{name}] NN dist pct 50/90/99/max(<cap): "
              f"{np.percentile(dq[np.isfinite(dq)], [50, 90, 99])} unmatched {np.sum(~np.isfinite(dq))}")
        for s in (0.05, 0.1, 0.2, 0.4):
            h = s * np.sqrt(3) / 2
            cell = np.floor(q / s).astype(np.int64)
            uc, inv = np.unique(cell, axis=0, return_inverse=True)
            cen = (uc + 0.5) * s
            d0, _ = tree.query(cen, distance_upper_bound=cap + h)
            r = np.minimum(d0 + h, cap) + h
            cnt = np.array([len(x) for x in tree.query_ball_point(cen, r, return_length=False)]) \
                if len(uc) < 20000 else tree.query_ball_point(cen, r, return_length=True)
            per_q = cnt[inv.ravel()]
            print(f"  s={s}: cells {len(uc)}, list per query pct 50/90/99/max "
                  f"{np.percentile(per_q, [50, 90, 99]).round(1)} {per_q.max()}, mean {per_q.mean():.1f}")


if __name__ == "__main__":
    main()
