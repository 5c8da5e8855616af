"""GPU parity of the spatially sharded S2M path through the C-ABI.

One GPU cannot host two RCCL ranks, so the multi-rank logic and the RCCL
plumbing are checked separately:
  * N shard contexts on one device (no communicator): their linearize
    moments add up to the unsharded moments (fp64, rel 1e-10: only the
    summation order differs), matched counts exactly, and every owned
    query's correspondence equals the unsharded one (same squared distance,
    bit-exact, and the same target point: exact ties resolve in the whole
    submap's nanoflann order through gicp_set_tie_target);
  * a one-rank RCCL communicator: the align graph with the all-reduce
    inside returns the bit-identical pose, iteration count and residuals
    of the plain align.
"""
import numpy as np
import pytest

import dynamic_direct_lidar_odometry_amd as P
from conftest import load_golden
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET
from dynamic_direct_lidar_odometry_amd.shard import ShardedGicp, halo_indices, owner_of, plan_slabs
import np_gicp as NP

pytestmark = pytest.mark.gpu

S2M = dict(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32, transformation_epsilon=0.01)


def full_ctx(g):
    c = P.Context(0)
    c.set_params(P.default_params(**S2M))
    c.set_target(g["sub"])
    c.set_source(g["src"])
    c.set_covariances(SOURCE, g["cov_src"])
    c.set_covariances(TARGET, g["cov_sub"])
    return c


@pytest.mark.parametrize("world", [2, 3, 8])
def test_shard_moments_add_up(world):
    g = load_golden("gicp_s2m.npz")
    pose = g["guess"].astype(np.float64)
    full = full_ctx(g)
    H, b, cost, nc = full.linearize(pose)
    mom = full.moments()
    fcorr, fsqd = full.correspondences()
    slabs = plan_slabs(g["sub"], world)
    own = owner_of(NP.transform_f32(pose, g["src"]), slabs)
    tot = np.zeros(80)
    ntot = 0
    for r, s in enumerate(slabs):
        idx = halo_indices(g["sub"], s, S2M["max_correspondence_distance"])
        c = P.Context(0)
        c.set_params(P.default_params(**S2M))
        c.set_target(g["sub"][idx])
        c.set_source(g["src"])
        c.set_covariances(SOURCE, g["cov_src"])
        c.set_covariances(TARGET, g["cov_sub"][idx])
        c.set_shard(s.axis, s.lo, s.hi)
        c.set_tie_target(g["sub"], idx)   # ties in the whole submap's nanoflann order
        _, _, _, n_r = c.linearize(pose)
        tot += c.moments()
        ntot += n_r
        corr, sqd = c.correspondences()
        mine = own == r
        # owned queries: the unsharded correspondence, exact (ties included)
        np.testing.assert_array_equal(sqd[mine], fsqd[mine])
        gc = np.where(corr >= 0, idx[np.maximum(corr, 0)], -1)
        np.testing.assert_array_equal(gc[mine], fcorr[mine])
        c.close()
    assert ntot == nc
    np.testing.assert_allclose(tot[:74], mom[:74], rtol=1e-10, atol=1e-10 * np.abs(mom[:74]).max())
    full.close()


def test_comm1_align_identical_to_plain():
    g = load_golden("gicp_s2m.npz")
    plain = full_ctx(g)
    out0, r0 = plain.align(g["guess"])
    res0 = plain.residuals()
    uid = P.comm_unique_id()
    sh = ShardedGicp(0, 0, 1, uid, P.default_params(**S2M), mode="slabs")
    assert sh.ctx.comm_info()[0] == 1
    sh.set_target(g["sub"], g["cov_sub"], source=g["src"], guess=g["guess"])
    assert sh.slab.lo == -np.inf and sh.slab.hi == np.inf
    sh.set_source(g["src"], g["cov_src"])
    out1, r1 = sh.align(g["guess"])
    np.testing.assert_array_equal(out1, out0)
    assert (r1.iterations_run, r1.converged, r1.lm_trials) == (r0.iterations_run, r0.converged, r0.lm_trials)
    np.testing.assert_array_equal(np.array(r1.final_hessian), np.array(r0.final_hessian))
    np.testing.assert_array_equal(sh.residuals(), res0)
    # a second align reuses the captured graphs
    out2, _ = sh.align(g["guess"])
    np.testing.assert_array_equal(out2, out0)
    print("comm graphs:", sh.ctx.comm_info())
    sh.close()
    plain.close()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_group_shards_moments_add_up(world):
    """Interleaved ownership (gicp_set_shard_groups, replicated target): the N parts' moments sum to the
    unsharded linearize, their matched counts add up, and every point is searched by exactly one part with
    the unsharded answer."""
    g = load_golden("gicp_s2m.npz")
    pose = g["guess"].astype(np.float64)
    full = full_ctx(g)
    H, b, cost, nc = full.linearize(pose)
    mom = full.moments()
    fcorr, fsqd = full.correspondences()
    tot = np.zeros(80)
    ntot = 0
    matched = np.zeros(len(g["src"]), np.int64)
    for r in range(world):
        c = full_ctx(g)
        c.set_shard_groups(world, r)
        _, _, _, n_r = c.linearize(pose)
        tot += c.moments()
        ntot += n_r
        corr, _ = c.correspondences()
        matched += corr >= 0
        np.testing.assert_array_equal(corr[corr >= 0], fcorr[corr >= 0])
        c.close()
    assert ntot == nc
    np.testing.assert_array_equal(matched, (fcorr >= 0).astype(np.int64))
    np.testing.assert_allclose(tot[:74], mom[:74], rtol=1e-10, atol=1e-10 * np.abs(mom[:74]).max())
    full.close()


def test_group_shard_comm1_align_identical_to_plain():
    g = load_golden("gicp_s2m.npz")
    plain = full_ctx(g)
    out0, r0 = plain.align(g["guess"])
    sh = ShardedGicp(0, 0, 1, P.comm_unique_id(), P.default_params(**S2M))   # default mode: groups
    sh.set_target(g["sub"], g["cov_sub"])
    sh.set_source(g["src"], g["cov_src"])
    out1, r1 = sh.align(g["guess"])
    np.testing.assert_array_equal(out1, out0)
    assert (r1.iterations_run, r1.lm_trials) == (r0.iterations_run, r0.lm_trials)
    sh.close()
    plain.close()


def test_shard_arguments_rejected():
    c = P.Context(0)
    with pytest.raises(P.GicpError):
        c.set_shard(3, 0.0, 1.0)
    with pytest.raises(P.GicpError):
        c.set_shard(0, 1.0, 1.0)
    c.set_shard(-1)
    with pytest.raises(P.GicpError):
        c.set_shard_groups(4, 4)
    with pytest.raises(P.GicpError):
        c.set_comm(b"\0" * 128, 2, 5)
    c.close()


@pytest.mark.parametrize("world", [2, 3])
def test_slab_shards_tied_target(knn_golden, world):
    """Slab shards of a target full of exact ties (the reference-nanoflann
    lattice fixture): every owned correspondence equals the unsharded one,
    which equals the reference's own 1-NN."""
    tgt = np.ascontiguousarray(knn_golden["lat_pts"])
    src = np.ascontiguousarray(knn_golden["lat_q"])
    rng = np.random.default_rng(3)
    A = rng.normal(0, 0.05, (len(tgt), 3, 3))
    tcov = NP.mat_to_sym6(A @ np.transpose(A, (0, 2, 1)) + 1e-3 * np.eye(3))
    A = rng.normal(0, 0.05, (len(src), 3, 3))
    scov = NP.mat_to_sym6(A @ np.transpose(A, (0, 2, 1)) + 1e-3 * np.eye(3))
    par = dict(S2M, k_correspondences=10)
    pose = np.eye(4)
    ref = knn_golden["lat_k1_idx"][:, 0]
    slabs = plan_slabs(tgt, world)
    own = owner_of(NP.transform_f32(pose, src), slabs)
    seen = np.zeros(len(src), bool)
    for r, s in enumerate(slabs):
        idx = halo_indices(tgt, s, par["max_correspondence_distance"])
        c = P.Context(0)
        c.set_params(P.default_params(**par))
        c.set_target(np.ascontiguousarray(tgt[idx]))
        c.set_covariances(TARGET, np.ascontiguousarray(tcov[idx]))
        c.set_source(src)
        c.set_covariances(SOURCE, np.ascontiguousarray(scov))
        c.set_shard(s.axis, s.lo, s.hi)
        c.set_tie_target(tgt, idx)
        c.linearize(pose)
        corr, _ = c.correspondences()
        mine = own == r
        gc = np.where(corr >= 0, idx[np.maximum(corr, 0)], -1)
        np.testing.assert_array_equal(gc[mine], ref[mine])
        seen |= mine
        c.close()
    assert seen.all()


def test_slab_tie_tree_blobs(knn_golden):
    """The builder / rank split of the slab tie order: one ctx holds the whole lattice and exports each
    rank's restriction; the rank ctxs (which never see the whole cloud) install the blobs and resolve
    every tie as the reference's nanoflann does.  A rank's blob holds its own points only; damaged or
    foreign blobs are rejected."""
    tgt = np.ascontiguousarray(knn_golden["lat_pts"])
    src = np.ascontiguousarray(knn_golden["lat_q"])
    par = dict(S2M, k_correspondences=10)
    ref = knn_golden["lat_k1_idx"][:, 0]
    world = 3
    slabs = plan_slabs(tgt, world)
    own = owner_of(NP.transform_f32(np.eye(4), src), slabs)
    builder = P.Context(0)
    with pytest.raises(P.GicpError):
        builder.tie_builder_export(np.arange(4))   # no whole cloud yet
    builder.tie_builder_set(tgt)
    assert builder.device_bytes()["tie_builder"] > 0
    seen = np.zeros(len(src), bool)
    for r, s in enumerate(slabs):
        idx = halo_indices(tgt, s, par["max_correspondence_distance"])
        blob = builder.tie_builder_export(idx)
        c = P.Context(0)
        c.set_params(P.default_params(**par))
        c.set_target(np.ascontiguousarray(tgt[idx]))
        c.compute_covariances(TARGET)
        with pytest.raises(P.GicpError):
            c.set_tie_tree(blob[:-16])                         # truncated
        bad = bytearray(blob)
        bad[-16:-4] = np.float32([9e9, 9e9, 9e9]).tobytes()    # a point that is not the local target's
        with pytest.raises(P.GicpError):
            c.set_tie_tree(bytes(bad))
        if r > 0:
            with pytest.raises(P.GicpError):
                c.set_tie_tree(builder.tie_builder_export(halo_indices(tgt, slabs[0], 2.0)))   # another rank's
        c.set_tie_tree(blob)
        db = c.device_bytes()
        assert db["tie_tree"] > 0 and db["tie_builder"] == 0
        c.set_source(src)
        c.compute_covariances(SOURCE)
        c.set_shard(s.axis, s.lo, s.hi)
        c.linearize(np.eye(4))
        corr, _ = c.correspondences()
        mine = own == r
        gc = np.where(corr >= 0, idx[np.maximum(corr, 0)], -1)
        np.testing.assert_array_equal(gc[mine], ref[mine])
        seen |= mine
        c.close()
    builder.tie_builder_set(None)
    assert builder.device_bytes()["tie_builder"] == 0
    builder.close()
    assert seen.all()


def test_tie_trees_from_root_one_rank(knn_golden):
    """gicp_set_tie_trees_from_root over a one-rank communicator (the root sends to nobody and installs
    its own blob); ShardedGicp's slab mode at world 1 resolves the lattice's ties exactly."""
    tgt = np.ascontiguousarray(knn_golden["lat_pts"])
    src = np.ascontiguousarray(knn_golden["lat_q"])
    c = P.Context(0)
    c.set_params(P.default_params(**dict(S2M, k_correspondences=10)))
    c.set_comm(P.comm_unique_id(), 1, 0)
    c.set_target(tgt)
    c.compute_covariances(TARGET)
    c.tie_builder_set(tgt)
    blob = c.tie_builder_export(np.arange(len(tgt)))
    c.tie_builder_set(None)
    c.set_tie_trees_from_root(0, [blob])
    assert c.device_bytes()["tie_tree"] > 0
    c.set_source(src)
    c.compute_covariances(SOURCE)
    c.set_shard(0, -np.inf, np.inf)
    c.linearize(np.eye(4))
    corr, _ = c.correspondences()
    np.testing.assert_array_equal(corr, knn_golden["lat_k1_idx"][:, 0])
    c.set_comm(None, 0, 0)
    c.close()


@pytest.mark.parametrize("op", ["swap", "clear"])
def test_tie_target_dropped_with_its_target(knn_golden, op):
    """The whole-target tie order belongs to the target it was given for:
    gicp_swap_source_target / gicp_clear_target drop it (the old index map
    would re-map a tied correspondence into the wrong cloud).  After a swap
    the ctx aligns the former target (a tied lattice) like a plain ctx; a bad
    index map is rejected at gicp_set_tie_target."""
    tgt = np.ascontiguousarray(knn_golden["lat_pts"])
    src = np.ascontiguousarray(knn_golden["lat_q"])
    par = dict(S2M, k_correspondences=10)
    idx = np.arange(len(tgt), dtype=np.int32)[: len(tgt) // 2]
    sub = np.ascontiguousarray(tgt[idx])
    c = P.Context(0)
    c.set_params(P.default_params(**par))
    c.set_target(sub)
    c.compute_covariances(TARGET)
    with pytest.raises(P.GicpError):
        c.set_tie_target(tgt, idx[::-1].copy())   # not the local points
    with pytest.raises(P.GicpError):
        bad = idx.copy()
        bad[1] = bad[0]
        c.set_tie_target(tgt, bad)                # not one-to-one
    c.set_tie_target(tgt, idx)
    c.set_source(src)
    c.compute_covariances(SOURCE)
    if op == "swap":
        c.swap_source_target()   # the lattice queries become the target, the half lattice the source
    else:
        c.clear_target()
        c.set_target(src)
        c.compute_covariances(TARGET)
        c.set_source(sub)
        c.compute_covariances(SOURCE)
    plain = P.Context(0)
    plain.set_params(P.default_params(**par))
    plain.set_target(src)
    plain.compute_covariances(TARGET)
    plain.set_source(sub)
    plain.compute_covariances(SOURCE)
    H, b, cost, nc = c.linearize(np.eye(4))
    Hp, bp, costp, ncp = plain.linearize(np.eye(4))
    np.testing.assert_array_equal(c.correspondences()[0], plain.correspondences()[0])
    np.testing.assert_array_equal(H, Hp)
    assert nc == ncp
    c.close()
    plain.close()
