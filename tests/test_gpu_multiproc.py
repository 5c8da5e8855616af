"""The sharded S2M linearize across PROCESSES: each of two
spawned processes opens a Context on device 0, takes its share of the source
(interleaved 16-point groups, or a spatial slab of the source with the
target's slab + halo and its restriction of the whole submap's nanoflann
tree, cut by rank 0 and sent over gloo), runs the library's
linearize and all-reduces the library's 80 moments over gloo -- the one
collective a sharded iteration makes (nano_gicp_impl.hpp:284-339 sums
per-thread partials; here per rank).  The sums equal the unsharded
gicp_get_moments at rel 1e-10 and the matched counts exactly, with the
target's candidate cells on and off.
"""
import os
import socket

import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

S2M = dict(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32, transformation_epsilon=0.01)


def _ctx(g, grid):
    import dynamic_direct_lidar_odometry_amd as P
    from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET
    c = P.Context(0)
    c.set_params(P.default_params(**S2M))
    c.set_target_grid(grid)
    c.set_target(np.ascontiguousarray(g["sub"]))
    c.set_covariances(TARGET, np.ascontiguousarray(g["cov_sub"]))
    c.set_source(np.ascontiguousarray(g["src"]))
    c.set_covariances(SOURCE, np.ascontiguousarray(g["cov_src"]))
    return c


def _worker(rank, world, port, mode, grid, q):
    import torch
    import torch.distributed as dist
    import dynamic_direct_lidar_odometry_amd as P
    from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET
    from dynamic_direct_lidar_odometry_amd.shard import halo_indices, plan_slabs_by_source
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = load_golden("gicp_s2m.npz")
        pose = np.asarray(g["guess"], np.float64)
        if mode == "groups":
            c = _ctx(g, grid)
            c.set_shard_groups(world, rank)
        else:
            slabs = plan_slabs_by_source(g["src"], pose.astype(np.float32), world)
            s = slabs[rank]
            idx = halo_indices(g["sub"], s, S2M["max_correspondence_distance"]).astype(np.int32)
            c = P.Context(0)
            c.set_params(P.default_params(**S2M))
            c.set_target_grid(grid)
            c.set_target(np.ascontiguousarray(g["sub"][idx]))
            c.set_covariances(TARGET, np.ascontiguousarray(g["cov_sub"][idx]))
            c.set_source(np.ascontiguousarray(g["src"]))
            c.set_covariances(SOURCE, np.ascontiguousarray(g["cov_src"]))
            c.set_shard(s.axis, s.lo, s.hi)
            # the whole submap's tie order: rank 0 builds it and cuts every rank's restriction, the blobs
            # travel over gloo (ShardedGicp sends them over its RCCL communicator instead)
            objs = [None]
            if rank == 0:
                c.tie_builder_set(np.ascontiguousarray(g["sub"]))
                objs = [[c.tie_builder_export(halo_indices(g["sub"], sl, S2M["max_correspondence_distance"]))
                         for sl in slabs]]
                c.tie_builder_set(None)
            dist.broadcast_object_list(objs, src=0)
            c.set_tie_tree(objs[0][rank])
            assert c.device_bytes()["tie_builder"] == 0
        c.linearize(pose)
        m = torch.from_numpy(c.moments().copy())
        own = torch.tensor([float(c.moments()[73])], dtype=torch.float64)
        dist.all_reduce(m)
        q.put((rank, m.numpy(), float(own[0]), c.grid_info()["built"]))
        c.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["groups", "slabs"])
@pytest.mark.parametrize("grid", [0, 2])
def test_two_processes_sum_to_unsharded(mode, grid):
    import torch.multiprocessing as mp
    g = load_golden("gicp_s2m.npz")
    c = _ctx(g, grid)
    c.linearize(np.asarray(g["guess"], np.float64))
    full = c.moments().copy()
    c.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, grid, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, m, own, built = q.get(timeout=240)
        res[r] = (m, own, built)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    np.testing.assert_array_equal(res[0][0], res[1][0])      # every rank holds the same sums
    m = res[0][0]
    assert m[73] == full[73]                                  # matched counts exact
    assert res[0][1] + res[1][1] == full[73] and res[0][1] > 0 and res[1][1] > 0
    np.testing.assert_allclose(m[:73], full[:73], rtol=1e-10, atol=1e-10 * np.abs(full[:73]).max())
    if grid:
        assert res[0][2] == 1 and res[1][2] == 1


def _rccl_worker(rank, world, port, q):
    """ShardedGicp in slab mode with its own RCCL communicator: rank 0 builds the whole submap's tree and
    sends every rank its restriction over RCCL (gicp_set_tie_trees_from_root); then a sharded align."""
    import torch.distributed as dist
    import dynamic_direct_lidar_odometry_amd as P
    from dynamic_direct_lidar_odometry_amd.shard import ShardedGicp
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = load_golden("gicp_s2m.npz")
        obj = [P.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        try:
            sh = ShardedGicp(0, rank, world, obj[0], P.default_params(**S2M), mode="slabs")
        except P.GicpError as e:   # e.g. RCCL refusing two ranks on one device
            q.put((rank, "skip", str(e)))
            return
        guess = np.asarray(g["guess"], np.float32)
        sh.set_target(np.ascontiguousarray(g["sub"]), np.ascontiguousarray(g["cov_sub"]),
                      source=np.ascontiguousarray(g["src"]), guess=guess)
        db = sh.ctx.device_bytes()
        sh.set_source(np.ascontiguousarray(g["src"]), np.ascontiguousarray(g["cov_src"]))
        T, r = sh.align(guess)
        q.put((rank, "ok", (np.asarray(T), int(r.iterations_run), db["tie_tree"], db["tie_builder"], len(sh.local_index))))
        sh.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_slab_tie_trees_over_rccl():
    """Two processes, slab mode, the tie-tree blobs sent over the library's RCCL communicator: every rank
    holds a tie tree of its own points only, and the sharded align equals the unsharded one (pose 1e-6,
    same iteration count).  Skipped where RCCL will not open two ranks on one device."""
    import dynamic_direct_lidar_odometry_amd as P
    import torch.multiprocessing as mp
    g = load_golden("gicp_s2m.npz")
    c = _ctx(g, 0)
    T0, r0 = c.align(np.asarray(g["guess"], np.float32))
    c.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rccl_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            rank, kind, payload = q.get(timeout=200)
            res[rank] = (kind, payload)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    if any(k == "skip" for k, _ in res.values()):
        pytest.skip("RCCL: " + next(v for k, v in res.values() if k == "skip"))
    for rank in (0, 1):
        T, iters, tie_bytes, builder_bytes, nloc = res[rank][1]
        assert iters == r0.iterations_run
        np.testing.assert_allclose(T, T0, atol=1e-6)
        assert tie_bytes > 0 and builder_bytes == 0 and nloc <= len(g["sub"])
