"""Developer probe: per-iteration distribution of the seed + walk cycles per
sub-group (statsprof build, DDLO_GICP_LIB=ab/libS.so) and a list-scheduling
estimate of the kernel's makespan: 1024 block slots (256 CUs x 4 blocks of
4 waves), blocks in dispatch order, a block's slot held until its slowest
wave ends.  Variants: the H slowest sub-groups split over P waves each."""
import heapq
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic_direct_lidar_odometry_amd import scene, Context, default_params, SOURCE, TARGET  # noqa: E402


def makespan(block_cycles, slots=1024):
    h = [0.0] * slots
    for b in block_cycles:
        t = heapq.heappop(h)
        heapq.heappush(h, t + b)
    return max(h)


prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
c = Context(0)
c.set_params(default_params(k_correspondences=10))
c.set_target(sub)
c.set_source(prob["source"])
c.compute_covariances(SOURCE)
c.compute_covariances(TARGET)
guess = prob["guess"].astype(np.float32)
prev = None
dump = {}
for it in (1, 2, 3):
    c.set_params(default_params(k_correspondences=10, max_correspondence_distance=2.0, max_iterations=it,
                                transformation_epsilon=1e-9))
    c.debug_stats(True)
    c.align(guess)
    st = c.debug_stats(True, read=True)
    ng = (prob["source"].shape[0] + 15) // 16
    st = st[:ng]
    cyc = st[:, 4].astype(np.float64)
    tasks = (st[:, 2] & 0xffff).astype(np.float64)
    q = np.percentile(cyc, [50, 90, 99, 99.9])
    blk = cyc[: ng // 4 * 4].reshape(-1, 4).max(axis=1)
    ms = makespan(blk)
    print(f"iter {it - 1}: sub-groups {ng}, cycles mean {cyc.mean():.0f} p50 {q[0]:.0f} p90 {q[1]:.0f} p99 {q[2]:.0f} "
          f"p99.9 {q[3]:.0f} max {cyc.max():.0f}; sum/4096 slots {cyc.sum() / 4096:.0f}; block-max sum/1024 "
          f"{blk.sum() / 1024:.0f}; list-schedule makespan {ms:.0f}; tasks {tasks.sum():.0f}")
    wav = makespan(cyc, 4096)
    msg = f"   per-wave dynamic fetch, index order: {wav:.0f}"
    if prev is not None:
        lpt = makespan(cyc[np.argsort(-prev, kind="stable")], 4096)
        msg += f"; heaviest-previous first: {lpt:.0f}"
    msg += f"; oracle LPT: {makespan(np.sort(cyc)[::-1], 4096):.0f}"
    print(msg)
    dump[f"cyc{it - 1}"] = cyc
    dump[f"tasks{it - 1}"] = tasks
    dump[f"blocks{it - 1}"] = st[:, 0].astype(np.float64)
    order = np.argsort(-cyc)
    for H in (16, 64, 256):
        for P in (4, 8):
            c2 = cyc.copy()
            top = order[:H]
            c2[top] = c2[top] / P + 14000   # each part re-runs the seed (~14k cycles)
            extra = np.repeat(c2[top], P - 1)
            blk2 = np.concatenate([c2[: ng // 4 * 4].reshape(-1, 4).max(axis=1),
                                   extra[: len(extra) // 4 * 4].reshape(-1, 4).max(axis=1)])
            print(f"   split top {H} x {P}: makespan {makespan(blk2):.0f}")
    if prev is not None:
        a, b = set(np.argsort(-prev)[:64]), set(order[:64])
        print(f"   top-64 overlap with the previous iteration: {len(a & b)}")
    prev = cyc
c.debug_stats(False)
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/tail_sim.npz", **dump)
