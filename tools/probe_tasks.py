"""Developer probe: task-search statistics of the cfg3 S2M search, per outer iteration
(per sub-group: seed cycles, hard flag, collect blocks / tasks / cycles).
Needs `make statsprof`: the production kernels carry no per-sub-group counters."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic_direct_lidar_odometry_amd import scene, Context, default_params, SOURCE, TARGET  # noqa

prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
c = Context(0)
c.set_params(default_params(k_correspondences=10))
c.set_target(sub); c.set_source(prob["source"])
c.compute_covariances(SOURCE); c.compute_covariances(TARGET)
guess = prob["guess"].astype(np.float32)
for it in (1, 2, 3):
    c.set_params(default_params(k_correspondences=10, max_correspondence_distance=2.0, max_iterations=it,
                                transformation_epsilon=1e-9))
    c.debug_stats(True)
    c.align(guess)
    st = c.debug_stats(True, read=True)
    st = st[st[:, 7] == 1]
    cyc = st[:, 4].astype(np.float64)
    seed = (st[:, 1] & 0xffff).astype(np.float64) * 16
    tasks = st[:, 2] & 0xffff
    iters = st[:, 2] >> 16
    hard = st[:, 6] & 1
    print(f"iter {it-1}: groups {len(st)} hard {hard.sum()} | blocks mean {st[:,0].mean():.1f} p99 {np.percentile(st[:,0],99):.0f} max {st[:,0].max()}"
          f" | tasks total {tasks.sum()} mean {tasks.mean():.1f} p99 {np.percentile(tasks,99):.0f} max {tasks.max()} | inline {st[:,3].sum()}")
    print(f"   seed cycles mean {seed.mean():.0f}; collect cycles mean {cyc.mean():.0f} p50 {np.percentile(cyc,50):.0f} p90 {np.percentile(cyc,90):.0f}"
          f" p99 {np.percentile(cyc,99):.0f} max {cyc.max():.0f}; hard groups' mean {cyc[hard == 1].mean() if hard.any() else 0:.0f}, walk loop iters {iters.mean():.1f}")
    w = np.argsort(-cyc)[:3]
    for t in w:
        print(f"   slowest group {t}: hard {hard[t]} blocks {st[t,0]} tasks {tasks[t]} cycles {st[t,4]}")
c.debug_stats(False)
