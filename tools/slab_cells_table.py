"""cfg 4 shards with the candidate cells ON: the 262k -> 2M-point S2M align cut into N shards on one
device, run one after another, each a ctx holding what its rank would hold:
  * slabs: the target inside the rank's source-balanced slab + the 2 m halo, cells built over that target only;
  * groups: the whole target (replicated), cells over all of it, the rank's 16-query groups owned.
Per rank: owned queries, target points, cells build ms / MiB, and the align's per-iteration linearize (HIP events,
profiled align) and LM step from a kernel-free estimate (the unsharded align's).  The unsharded ctx (cells on) and
a one-rank RCCL ctx's align time (the in-graph all-reduce of the 80 moments at world 1) come first.
    python tools/slab_cells_table.py [N ...]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET, scene  # noqa: E402
from dynamic_direct_lidar_odometry_amd.shard import halo_indices, owner_of, plan_slabs_by_source, transform_f32  # noqa: E402

S2M = dict(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32, transformation_epsilon=0.01)
worlds = [int(a) for a in sys.argv[1:]] or [2, 4, 8]

p = scene.s2m_problem(128, 2048, 8, 2000000, 4)
sub = np.ascontiguousarray(np.concatenate(p["keyframes"])[p["subset"]])
kc = P.Context(0, P.default_params(k_correspondences=10))
covs = []
for k in p["keyframes"]:
    kc.set_target(k)
    kc.compute_covariances(TARGET)
    covs.append(kc.get_covariances(TARGET))
tcov = np.ascontiguousarray(np.concatenate(covs)[p["subset"]])
kc.set_target(p["source"])
kc.compute_covariances(TARGET)
scov = kc.get_covariances(TARGET)
kc.close()
src = p["source"]
guess = p["guess"].astype(np.float32)
MB = 1.0 / (1 << 20)


def ctx_for(target, cov, grid=P.GRID_ON):
    c = P.Context(0, P.default_params(**S2M))
    c.set_target_grid(grid)
    c.set_target(np.ascontiguousarray(target))
    c.set_covariances(TARGET, np.ascontiguousarray(cov))
    c.set_source(src)
    c.set_covariances(SOURCE, scov)
    return c


def measure(c, reps=20):
    c.align(guess)   # builds the cells (GRID_ON: at this align)
    info = c.grid_info()
    c.set_profiling(True)
    _, r = c.align(guess)
    c.set_profiling(False)
    lin_us = r.linearize_ms / max(r.iterations_run, 1) * 1e3
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        _, r2 = c.align(guess)
        ts.append(time.perf_counter() - t0)
    return info, lin_us, float(np.median(ts)) * 1e3, r2.iterations_run


c = ctx_for(sub, tcov)
info, lin, ms, it = measure(c)
db = c.device_bytes()
c.close()
print(f"unsharded (cells on): {len(src)} queries, {len(sub)} target points, cells {info['build_ms']:.1f} ms "
      f"{info['bytes'] * MB:.0f} MiB, linearize {lin:.1f} us/iteration, align {ms:.4f} ms ({it} iterations), "
      f"ctx {db['total'] * MB:.0f} MiB", flush=True)
c = ctx_for(sub, tcov)
c.set_comm(P.comm_unique_id(), 1, 0)
info1, lin1, ms1, it1 = measure(c)
c.set_comm(None, 0, 0)
c.close()
print(f"one-rank RCCL ctx (in-graph all-reduce of 80 doubles per iteration): align {ms1:.4f} ms ({it1} iterations), "
      f"+{(ms1 - ms) / max(it1, 1) * 1e3:.1f} us per iteration over the plain ctx", flush=True)
pose = guess.astype(np.float64)
for world in worlds:
    slabs = plan_slabs_by_source(src, pose, world)
    own = owner_of(transform_f32(src, pose), slabs)
    for r, sl in enumerate(slabs):
        idx = halo_indices(sub, sl, S2M["max_correspondence_distance"])
        c = ctx_for(sub[idx], tcov[idx])
        c.set_shard(sl.axis, sl.lo, sl.hi)
        info, lin, ms, it = measure(c)
        db = c.device_bytes()
        c.close()
        print(f"slabs world {world} rank {r}: owned {int((own == r).sum())}, target {len(idx)}, cells "
              f"{info['build_ms']:.1f} ms {info['bytes'] * MB:.0f} MiB (walk {info['uses_walk']}), linearize "
              f"{lin:.1f} us/iteration, align {ms:.4f} ms, ctx {db['total'] * MB:.0f} MiB", flush=True)
    c = ctx_for(sub, tcov)
    for r in range(world):
        c.set_shard_groups(world, r)
        info, lin, ms, it = measure(c)
        print(f"groups world {world} rank {r}: owned 1/{world} of the groups, target {len(sub)}, cells "
              f"{info['build_ms']:.1f} ms {info['bytes'] * MB:.0f} MiB, linearize {lin:.1f} us/iteration, "
              f"align {ms:.4f} ms", flush=True)
    c.close()
