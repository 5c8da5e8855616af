"""GPU: nanoflann's kd-tree built on the device (nftree.hip) equals the
oracle's tree, which test_nftree_cpu.py pins to the reference's own
nanoflann; tied queries resolved through it reproduce nanoflann's answers
(covariances and kNN) bit for bit."""
import numpy as np
import pytest

import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET, scene
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _clouds():
    rng = np.random.default_rng(7)
    lat = np.stack(np.meshgrid(np.arange(30), np.arange(30), np.arange(6), indexing="ij"), -1).reshape(-1, 3)
    big_lat = np.stack(np.meshgrid(np.arange(80), np.arange(80), np.arange(12), indexing="ij"), -1).reshape(-1, 3)
    return {
        "normal40k": (rng.standard_normal((40000, 3)) * [20, 20, 3]).astype(np.float32),
        "normal500k": (rng.standard_normal((500000, 3)) * [30, 30, 3]).astype(np.float32),
        "lattice": lat.astype(np.float32),
        "lattice77k": big_lat.astype(np.float32),
        "duplicates": np.repeat((rng.standard_normal((3000, 3)) * 5).astype(np.float32), 4, axis=0),
        "leaf_only": rng.standard_normal((57, 3)).astype(np.float32),
        "one_small_node": rng.standard_normal((3000, 3)).astype(np.float32),
        "outliers": np.concatenate([(rng.standard_normal((20000, 3)) * 0.5).astype(np.float32),
                                    np.array([[1e4, 1e4, 1e4], [-5e3, 2, 3]], np.float32)]),
        "flat": np.concatenate([(rng.standard_normal((9000, 2)) * 10), np.zeros((9000, 1))], 1).astype(np.float32),
        "all_equal": np.ones((5000, 3), np.float32),
    }


@pytest.mark.parametrize("name", sorted(_clouds()))
def test_device_tree_equals_oracle_tree(name):
    pts = _clouds()[name]
    c = P.Context(0)
    c.set_target(pts)
    dev = c.nftree(TARGET)
    assert O.same_tree(dev, O.tree(pts)) is None


def test_device_tree_raycast_scan():
    src, _, _ = scene.s2s_pair(64, 2048, 2)
    c = P.Context(0)
    c.set_source(src)
    assert O.same_tree(c.nftree(SOURCE), O.tree(src)) is None


@pytest.mark.parametrize("k", [10, 20])
def test_covariance_ties_lattice(k):
    """An integer lattice: nearly every point's k-th neighbour distance is tied."""
    lat = np.stack(np.meshgrid(np.arange(24), np.arange(24), np.arange(5), indexing="ij"), -1).reshape(-1, 3)
    pts = (lat.astype(np.float32) * np.float32(0.25))
    pts = pts + (np.arange(len(pts)) % 7 == 0)[:, None].astype(np.float32) * np.float32(0.01)   # some irregularity
    c = P.Context(0)
    c.set_params(P.default_params(k_correspondences=k))
    c.set_target(pts)
    c.compute_covariances(TARGET)
    got = c.get_covariances(TARGET)
    ref = O.covariances(pts, k)
    scale = max(np.abs(ref).max(), 1.0)
    bad = np.where(np.abs(got - ref).max(axis=1) > 1e-12 * scale)[0]
    _, d = O.knn(pts, pts, k + 1)
    assert (d[:, k - 1] == d[:, k]).sum() > len(pts) // 10   # the case really is tie-heavy
    assert len(bad) == 0, f"{len(bad)} mismatches, e.g. {bad[:8]}"


def test_knn_ties_random_duplicates():
    rng = np.random.default_rng(3)
    base = (rng.standard_normal((2000, 3)) * 3).astype(np.float32)
    pts = np.concatenate([base, base[::3], base[::5]])
    q = np.concatenate([base[::7], (rng.standard_normal((500, 3)) * 3).astype(np.float32)])
    c = P.Context(0)
    c.set_target(pts)
    for k in (1, 5, 10, 20, 33):
        idx, sqd = c.knn_target(q, k)
        ri, rd = O.knn(pts, q, k)
        np.testing.assert_array_equal(sqd, rd)
        np.testing.assert_array_equal(idx, ri)


def test_register_input_source_keeps_covariances():
    """registerInputSource (nano_gicp_impl.hpp:122-130) keeps source_covs_:
    gicp_set_source(build_index=0) of a same-size cloud keeps covariance i on point i."""
    rng = np.random.default_rng(5)
    a = (rng.standard_normal((3000, 3)) * 4).astype(np.float32)
    b = (rng.standard_normal((3000, 3)) * 4).astype(np.float32)
    c = P.Context(0)
    c.set_params(P.default_params(k_correspondences=10))
    c.set_source(a)
    c.compute_covariances(SOURCE)
    cov_a = c.get_covariances(SOURCE)
    c.set_source(b, build_index=False)
    assert c.has_covariances(SOURCE)
    np.testing.assert_array_equal(c.get_covariances(SOURCE), cov_a)
    c.set_source(a[:2000], build_index=False)   # size changed: recomputed at align, as the reference
    assert not c.has_covariances(SOURCE)
    c.set_source(b)                             # setInputSource clears them (:142)
    assert not c.has_covariances(SOURCE)
