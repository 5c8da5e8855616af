"""GPU parity at the bench's own workload sizes:

cfg 4  262,144-pt 128x2048 scan -> 2,000,000-pt 8-keyframe submap, S2M
       parameters (k=20, maxCorr 2 m, LM):
       * N in {2, 4, 8} interleaved-ownership shard contexts on one device
         (gicp_set_shard_groups): their linearize moments add up to the
         unsharded ones (fp64, rel 1e-10: only the summation order differs),
         the matched counts add up and every matched query has the unsharded
         correspondence;
       * the one-rank RCCL ShardedGicp align against the oracle on the full
         2M cloud: |dt| <= 1e-5 m, rotation entries <= 1e-5, same iterations.
cfg 5  64x2048 frames of the 1000-frame plaza loop (GPU ray caster):
       * a 22-frame chain through the odometry driver (cfg/ddlo.yaml
         parameters) against oracle/odom_ref.py: statuses, keyframe and submap
         decisions exact, poses within the north star's 1e-4;
       * gicp_s2s_batch against the oracle's S2S on 3 pairs (1e-4).
Both sides get the same covariances where a test feeds them (the oracle's);
the covariance kernels' own parity is in test_gpu_gicp / test_gpu_nftree.
"""
import numpy as np
import pytest

import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET, scene
from dynamic_direct_lidar_odometry_amd import odometry as OD
from dynamic_direct_lidar_odometry_amd.shard import ShardedGicp
from oracle import oracle as O
from oracle import odom_ref as R

pytestmark = pytest.mark.gpu

S2M = dict(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32, transformation_epsilon=0.01)
S2S = dict(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32, transformation_epsilon=0.01)
THREADS = 16


@pytest.fixture(scope="module")
def cfg4():
    p = scene.s2m_problem(128, 2048, 8, 2000000, 4)
    sub = np.ascontiguousarray(np.concatenate(p["keyframes"])[p["subset"]])
    tcov = np.ascontiguousarray(np.concatenate([O.covariances(k, 10, threads=THREADS) for k in p["keyframes"]])
                                [p["subset"]])
    scov = O.covariances(p["source"], 10, threads=THREADS)
    return dict(src=p["source"], sub=sub, tcov=tcov, scov=scov, guess=p["guess"].astype(np.float32))


def _ctx(g):
    c = P.Context(0)
    c.set_params(P.default_params(**S2M))
    c.set_target(g["sub"])
    c.set_covariances(TARGET, g["tcov"])
    c.set_source(g["src"])
    c.set_covariances(SOURCE, g["scov"])
    return c


@pytest.mark.parametrize("world", [2, 4, 8])
def test_cfg4_group_shards_add_up(cfg4, world):
    pose = cfg4["guess"].astype(np.float64)
    full = _ctx(cfg4)
    _, _, _, nc = full.linearize(pose)
    mom = full.moments()
    fcorr, _ = full.correspondences()
    full.close()
    tot = np.zeros(80)
    ntot = 0
    matched = np.zeros(len(cfg4["src"]), np.int64)
    for r in range(world):
        c = _ctx(cfg4)
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


@pytest.mark.parametrize("world", [2, 4, 8])
def test_cfg4_slab_shards_add_up(cfg4, world):
    """Slab mode at cfg 4 size (the spatial tiling of north_star / SURVEY.md §8(e)): N contexts on one device,
    each with its slab + 2 m halo of the 2M-point submap (slabs cut on the source at the guess) and, as its
    tie order, the whole submap's nanoflann tree restricted to its points (one builder ctx exports every
    rank's restriction; a rank never holds the whole submap).  Moments add up (rel 1e-10), matched counts
    add up, every owned correspondence equals the unsharded one exactly (ties included), and a rank's tie
    tree is O(its points).  Prints the per-rank linearize time (ranks run one after another here) and
    device bytes for DESIGN.md's slab table."""
    from dynamic_direct_lidar_odometry_amd.shard import halo_indices, owner_of, plan_slabs_by_source, transform_f32
    pose = cfg4["guess"].astype(np.float64)
    full = _ctx(cfg4)
    _, _, _, nc = full.linearize(pose)
    mom = full.moments()
    fcorr, fsqd = full.correspondences()
    full_bytes = full.device_bytes()
    full.close()
    slabs = plan_slabs_by_source(cfg4["src"], pose, world)
    builder = P.Context(0)
    builder.tie_builder_set(cfg4["sub"])
    builder_bytes = builder.device_bytes()["tie_builder"]
    own = owner_of(transform_f32(cfg4["src"], pose), slabs)
    tot = np.zeros(80)
    ntot = 0
    rows = []
    for r, sl in enumerate(slabs):
        idx = halo_indices(cfg4["sub"], sl, S2M["max_correspondence_distance"])
        c = P.Context(0)
        c.set_params(P.default_params(**S2M))
        c.set_target(np.ascontiguousarray(cfg4["sub"][idx]))
        c.set_covariances(TARGET, np.ascontiguousarray(cfg4["tcov"][idx]))
        c.set_source(cfg4["src"])
        c.set_covariances(SOURCE, cfg4["scov"])
        c.set_shard(sl.axis, sl.lo, sl.hi)
        c.set_tie_tree(builder.tie_builder_export(idx))
        db = c.device_bytes()
        assert db["tie_builder"] == 0 and db["tie_tree"] <= 40 * len(idx) + (1 << 20)
        _, _, _, n_r = c.linearize(pose)
        tot += c.moments()
        ntot += n_r
        corr, sqd = c.correspondences()
        mine = own == r
        gc = np.where(corr >= 0, idx[np.maximum(corr, 0)], -1)
        np.testing.assert_array_equal(gc[mine], fcorr[mine])
        np.testing.assert_array_equal(sqd[mine], fsqd[mine])
        c.set_profiling(True)
        _, res = c.align(cfg4["guess"])
        c.set_profiling(False)
        rows.append((r, int(mine.sum()), len(idx), res.linearize_ms / max(res.iterations_run, 1) * 1e3, db))
        c.close()
    builder.close()
    assert ntot == nc
    np.testing.assert_allclose(tot[:74], mom[:74], rtol=1e-10, atol=1e-10 * np.abs(mom[:74]).max())
    mb = 1.0 / (1 << 20)
    print(f"slab world {world}: unsharded ctx {full_bytes['total'] * mb:.1f} MiB (target {full_bytes['target'] * mb:.1f}), "
          f"rank-0 builder transient {builder_bytes * mb:.1f} MiB")
    for r, nq, nt, us, db in rows:
        print(f"slab world {world} rank {r}: owned queries {nq}, target points {nt}, linearize {us:.1f} us, "
              f"device {db['total'] * mb:.1f} MiB (target {db['target'] * mb:.1f}, tie tree {db['tie_tree'] * mb:.2f}, "
              f"scratch {db['scratch'] * mb:.1f})")


def test_cfg4_comm1_pose_vs_oracle(cfg4):
    sh = ShardedGicp(0, 0, 1, P.comm_unique_id(), P.default_params(**S2M))
    sh.set_target(cfg4["sub"], cfg4["tcov"])
    sh.set_source(cfg4["src"], cfg4["scov"])
    T, r = sh.align(cfg4["guess"])
    sh.close()
    g = O.Gicp(cfg4["src"], cfg4["sub"], O.default_params(**S2M), threads=THREADS)
    g.set_covariances(0, cfg4["scov"])
    g.set_covariances(1, cfg4["tcov"])
    To, ro = g.align(cfg4["guess"])
    assert r.iterations_run == ro.iterations_run and bool(r.converged) == bool(ro.converged)
    np.testing.assert_allclose(T[:3, 3], To[:3, 3], rtol=0, atol=1e-5)
    np.testing.assert_allclose(T[:3, :3], To[:3, :3], rtol=0, atol=1e-5)


@pytest.fixture(scope="module")
def cfg5():
    return scene.loop_sequence(64, 2048, 0, 22, device=0)[0]


def test_cfg5_odometry_chain_vs_oracle(cfg5):
    p = OD.default_odom_params()
    gpu = OD.Odometry(0, p)
    ref = R.OdomRef(p, threads=THREADS)
    tracked = 0
    for i, f in enumerate(cfg5):
        g = gpu.process(f)
        o = ref.process(f)
        assert g.status == o["status"], i
        if g.status == OD.INIT:
            continue
        assert g.scan_points == o["scan_points"], i
        assert g.keyframe_added == o["keyframe_added"], i
        if g.status != OD.TRACKED:
            continue
        tracked += 1
        assert g.num_keyframes == o["num_keyframes"], i
        assert gpu.submap().tolist() == o["submap"], i
        T = g.pose()
        np.testing.assert_allclose(T[:3, 3], o["T"][:3, 3], atol=1e-4, err_msg=f"frame {i}")
        np.testing.assert_allclose(T[:3, :3], o["T"][:3, :3], atol=1e-4, err_msg=f"frame {i}")
        assert g.s2s.iterations_run == o["s2s"].iterations_run and g.s2m.iterations_run == o["s2m"].iterations_run, i
    assert tracked >= 20
    gpu.close()


def test_cfg5_s2s_batch_vs_oracle(cfg5):
    frames = cfg5[4:8]
    poses, res = P.s2s_batch(frames, P.default_params(**S2S), device=0, nstreams=2)
    for t in range(1, 4):
        g = O.Gicp(frames[t], frames[t - 1], O.default_params(**S2S), threads=THREADS)
        To, ro = g.align(np.eye(4, dtype=np.float32))
        assert res[t].iterations_run == ro.iterations_run, t
        np.testing.assert_allclose(poses[t][:3, 3], To[:3, 3], rtol=0, atol=1e-4, err_msg=f"pair {t}")
        np.testing.assert_allclose(poses[t][:3, :3], To[:3, :3], rtol=0, atol=1e-4, err_msg=f"pair {t}")
