"""Developer probe (needs `make statsprof`): cfg 2's last outer iteration after n GN iterations -- how many
16-query sub-groups still walk although verified reuse passes most queries, and what their walks cost."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET, scene  # noqa: E402

src, tgt, _ = scene.s2s_pair(64, 2048, 2)
c = P.Context(0)
c.set_target_grid(P.GRID_OFF)
c.set_params(P.default_params(k_correspondences=10))
c.set_target(tgt)
c.set_source(src)
c.compute_covariances(SOURCE)
c.compute_covariances(TARGET)
for it in (2, 5, 8, 10, 15, 20):
    c.set_params(P.default_params(k_correspondences=10, max_correspondence_distance=1.0, optimizer=P.GAUSS_NEWTON,
                                  fixed_iterations=it, max_iterations=it))
    c.debug_stats(True)
    c.align(None)
    st = c.debug_stats(True, read=True)
    walked = (st[:, 0] > 0) | ((st[:, 2] & 0xffff) > 0) | (st[:, 4] > 0)
    npass = (st[:, 6] >> 8) & 0xff
    cyc = st[:, 4].astype(np.float64)
    seed = (st[:, 1] & 0xffff).astype(np.float64) * 16
    print(f"iteration {it - 1}: sub-groups {len(st)}, walked {int(walked.sum())} ({100 * walked.mean():.1f} %), "
          f"reuse-passed queries {int(npass.sum())}; walked groups: blocks mean {st[walked, 0].mean() if walked.any() else 0:.1f}, "
          f"tasks mean {(st[walked, 2] & 0xffff).mean() if walked.any() else 0:.1f}, seed cycles mean {seed[walked].mean() if walked.any() else 0:.0f}, "
          f"walk cycles mean {cyc[walked].mean() if walked.any() else 0:.0f} max {cyc.max():.0f}", flush=True)
c.debug_stats(False)
