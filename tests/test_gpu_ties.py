"""Exact distance ties in the correspondences of the align itself
(update_correspondences, reference nano_gicp_impl.hpp:255 ->
nanoflann_impl.hpp:205-237,1509: of several target points at the same fp32
distance nanoflann keeps the first its walk meets).

The targets are the reference-nanoflann fixtures with exact ties
(tests/golden/knn_ref.npz, produced by the reference's own nanoflann_impl.hpp
compiled in the build container): a cloud whose every point appears twice and
an integer lattice queried at its cell centres (8 equidistant corners).  Each
copy of a duplicated point gets a DIFFERENT covariance, so a wrong choice
among tied points changes M, H and b, not only an index.

Bars: correspondences and squared distances bit-exact against the reference
goldens (1-NN of the lattice) and the oracle; H, b, cost rel 1e-11; poses
1e-6 with identical iteration and LM-trial counts.
"""
import numpy as np
import pytest

import dynamic_direct_lidar_odometry_amd as P
import np_gicp as NP
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET
from oracle import oracle as O

pytestmark = pytest.mark.gpu

PAR = dict(k_correspondences=10, max_correspondence_distance=2.0, max_iterations=32, transformation_epsilon=5e-4)


def spd_covs(n, seed, scale=0.05):
    rng = np.random.default_rng(seed)
    A = rng.normal(0, scale, (n, 3, 3))
    C = A @ np.transpose(A, (0, 2, 1)) + 1e-3 * np.eye(3)
    return np.ascontiguousarray(NP.mat_to_sym6(C))


def tied_case(knn_golden, name):
    g = knn_golden
    if name == "lattice":
        tgt, src = g["lat_pts"], g["lat_q"]
    else:
        tgt, src = g["dup_pts"], g["dup_q"]
    return (np.ascontiguousarray(tgt), np.ascontiguousarray(src), spd_covs(len(tgt), 1), spd_covs(len(src), 2))


def make_ctx(tgt, src, tcov, scov, **kw):
    c = P.Context(0)
    c.set_params(P.default_params(**{**PAR, **kw}))
    c.set_target(tgt)
    c.set_covariances(TARGET, tcov)
    c.set_source(src)
    c.set_covariances(SOURCE, scov)
    return c


def make_oracle(tgt, src, tcov, scov, **kw):
    o = O.Gicp(src, tgt, O.default_params(**{**PAR, **kw}))
    o.set_covariances(0, scov)
    o.set_covariances(1, tcov)
    return o


@pytest.mark.parametrize("name", ["lattice", "duplicates"])
def test_linearize_tied_correspondences(knn_golden, name):
    tgt, src, tcov, scov = tied_case(knn_golden, name)
    c = make_ctx(tgt, src, tcov, scov)
    o = make_oracle(tgt, src, tcov, scov)
    I = np.eye(4)
    H, b, cost, nc = c.linearize(I)
    corr, sqd = c.correspondences()
    Ho, bo, co, ocorr, osqd = o.linearize(I)
    np.testing.assert_array_equal(corr, ocorr)
    np.testing.assert_array_equal(sqd, osqd)
    # the reference's own nanoflann (compiled from /root/reference in the build container)
    ref_idx = knn_golden["lat_k1_idx"][:, 0] if name == "lattice" else knn_golden["dup_k10_idx"][:, 0]
    ref_sqd = knn_golden["lat_k1_sqd"][:, 0] if name == "lattice" else knn_golden["dup_k10_sqd"][:, 0]
    np.testing.assert_array_equal(corr, np.where(ref_sqd < PAR["max_correspondence_distance"] ** 2, ref_idx, -1))
    np.testing.assert_array_equal(sqd, ref_sqd)
    np.testing.assert_allclose(H, Ho, rtol=1e-11, atol=1e-11 * np.abs(Ho).max())
    np.testing.assert_allclose(b, bo, rtol=1e-11, atol=1e-11 * np.abs(bo).max())
    assert abs(cost - co) <= 1e-11 * abs(co)
    assert nc == int(np.sum(ocorr >= 0))
    c.close()


def test_tied_queries_are_counted_and_tree_built_once(knn_golden):
    """The first align on a tied target meets ties before the target has
    nanoflann's tree: the tree is built and the align re-run (tie_reruns 1);
    later aligns use the tree (reruns 0).  Both give the oracle's result."""
    tgt, src, tcov, scov = tied_case(knn_golden, "lattice")
    c = make_ctx(tgt, src, tcov, scov)
    o = make_oracle(tgt, src, tcov, scov)
    opose, ores = o.align()
    for k in range(2):
        pose, res = c.align()
        assert res.tie_reruns == (1 if k == 0 else 0)
        assert res.ties_resolved > 0
        assert (res.iterations_run, res.converged, res.lm_trials) == (ores.iterations_run, ores.converged, ores.lm_trials)
        np.testing.assert_allclose(pose, opose, atol=1e-6)
    c.close()


@pytest.mark.parametrize("name", ["lattice", "duplicates"])
def test_align_on_tied_target(knn_golden, name):
    """Aligns from the identity (every first-iteration search tied) and from
    small offsets: pose, iterations, LM trials and the last correspondences
    equal the oracle's."""
    tgt, src, tcov, scov = tied_case(knn_golden, name)
    c = make_ctx(tgt, src, tcov, scov)
    o = make_oracle(tgt, src, tcov, scov)
    rng = np.random.default_rng(5)
    guesses = [np.eye(4, dtype=np.float32)]
    for _ in range(2):
        G = np.eye(4, dtype=np.float32)
        G[:3, :3] = NP.so3_exp(rng.normal(0, 0.01, 3))
        G[:3, 3] = rng.normal(0, 0.05, 3)
        guesses.append(G)
    for G in guesses:
        pose, res = c.align(G)
        opose, ores = o.align(G)
        assert (res.iterations_run, res.converged, res.lm_trials, res.lm_failed) == \
            (ores.iterations_run, ores.converged, ores.lm_trials, ores.lm_failed)
        np.testing.assert_allclose(pose, opose, atol=1e-6)
        corr, sqd = c.correspondences()
        oc, osd = o.last_correspondences()
        np.testing.assert_array_equal(corr, oc)
        np.testing.assert_array_equal(sqd, osd)
    c.close()


def test_morton_tie_order_differs(knn_golden):
    """gicp_set_tie_order(0) keeps the lower Morton position: the same
    distances, and on the lattice a different point for some tied queries
    (so the tests above are sensitive to the order)."""
    tgt, src, tcov, scov = tied_case(knn_golden, "lattice")
    c = make_ctx(tgt, src, tcov, scov)
    c.set_tie_order(False)
    c.linearize(np.eye(4))
    corr, sqd = c.correspondences()
    np.testing.assert_array_equal(sqd, knn_golden["lat_k1_sqd"][:, 0])
    assert np.any(corr != knn_golden["lat_k1_idx"][:, 0])
    c.close()
