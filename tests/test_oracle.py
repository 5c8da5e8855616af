"""CPU tests of the oracle (the checker): pinned to the reference's own nanoflann
(golden vectors generated from oracle/_ref) and cross-checked against the
independent numpy restatement in tests/np_gicp.py.  No GPU needed."""
import numpy as np
import pytest

import np_gicp as NP
from oracle import oracle as O


# ---------------------------------------------------------------- kNN (pinned)
@pytest.mark.parametrize("k", [1, 10, 20])
def test_oracle_knn_matches_reference_nanoflann_golden(knn_golden, k):
    g = knn_golden
    q = g["scan_q"] if k == 1 else g["scan_q"][::4]
    idx, sqd = O.knn(g["scan_pts"], q, k)
    np.testing.assert_array_equal(idx, g[f"scan_k{k}_idx"])
    np.testing.assert_array_equal(sqd, g[f"scan_k{k}_sqd"])


@pytest.mark.parametrize("case", ["self_k10", "far_k10", "dup_k10", "lat_k1", "lat_k10"])
def test_oracle_knn_edge_goldens(knn_golden, case):
    g = knn_golden
    pts, q = {"self_k10": (g["scan_pts"][:2048], g["scan_pts"][:2048]),
              "far_k10": (g["scan_pts"], g["far_q"]),
              "dup_k10": (g["dup_pts"], g["dup_q"]),
              "lat_k1": (g["lat_pts"], g["lat_q"]),
              "lat_k10": (g["lat_pts"], g["lat_q"])}[case]
    k = int(case.split("_k")[1])
    idx, sqd = O.knn(pts, q, k)
    # the oracle restates nanoflann's traversal, so even exact ties are resolved identically
    np.testing.assert_array_equal(idx, g[f"{case}_idx"])
    np.testing.assert_array_equal(sqd, g[f"{case}_sqd"])


def test_oracle_knn_live_vs_reference_build():
    """When oracle/_ref was built here (dev container), compare on fresh random data too."""
    if O.ref_lib() is None:
        pytest.skip("oracle/_ref not built (reference absent)")
    rng = np.random.default_rng(3)
    pts = (rng.standard_normal((5000, 3)) * [10, 10, 2]).astype(np.float32)
    q = (rng.standard_normal((700, 3)) * [12, 12, 3]).astype(np.float32)
    for k in (1, 7, 20):
        a = O.knn(pts, q, k)
        b = O.ref_knn(pts, q, k)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])


def test_knn_golden_distances_are_true_minima(knn_golden):
    """Independent check of the golden itself: scipy brute force agrees on distances."""
    g = knn_golden
    from scipy.spatial import cKDTree
    d, _ = cKDTree(g["scan_pts"].astype(np.float64)).query(g["scan_q"].astype(np.float64), 1)
    np.testing.assert_allclose(np.sqrt(g["scan_k1_sqd"][:, 0].astype(np.float64)), d, rtol=1e-5, atol=1e-6)
    chosen = NP.nanoflann_sqd(g["scan_q"], g["scan_pts"][g["scan_k1_idx"][:, 0]])
    np.testing.assert_array_equal(chosen, g["scan_k1_sqd"][:, 0])


# ------------------------------------------------------------- covariances
@pytest.mark.parametrize("reg", ["NONE", "MIN_EIG", "NORMALIZED_MIN_EIG", "PLANE", "FROBENIUS"])
def test_oracle_covariances_vs_numpy(s2s_golden, reg):
    src = s2s_golden["src"]
    oc = O.covariances(src, 10, reg)
    np.testing.assert_array_equal(oc, s2s_golden[f"cov_src_{reg}"])        # regression
    nc, nidx = NP.covariances(src, 10, reg)
    oidx, _ = O.knn(src, src, 10)
    same = np.all(np.sort(nidx, 1) == np.sort(oidx, 1), axis=1)
    assert same.mean() > 0.999
    scale = np.abs(nc[same]).max()
    np.testing.assert_allclose(NP.sym6_to_mat(oc)[same], nc[same], atol=1e-9 * max(scale, 1.0), rtol=0)


# ------------------------------------------------------------- linearize / error
def _np_problem(g, max_corr=1.0):
    return NP.Problem(g["src"], g["tgt"], NP.sym6_to_mat(g["cov_src_PLANE"]), NP.sym6_to_mat(g["cov_tgt"]), max_corr)


def test_oracle_linearize_vs_numpy(s2s_golden):
    g = s2s_golden
    p = _np_problem(g)
    H, b, cost = p.linearize(np.eye(4))
    oracle = O.Gicp(g["src"], g["tgt"], O.default_params(k_correspondences=10, max_correspondence_distance=1.0))
    oracle.set_covariances(0, g["cov_src_PLANE"])
    oracle.set_covariances(1, g["cov_tgt"])
    Ho, bo, co, corr, sqd = oracle.linearize(np.eye(4))
    np.testing.assert_array_equal(corr, g["lin_corr"])
    np.testing.assert_array_equal(sqd, g["lin_sqd"])
    # the oracle's OpenMP partial sums depend on the thread count: regression at 1e-12
    np.testing.assert_allclose(Ho, g["lin_H"], rtol=1e-12, atol=1e-12 * np.abs(Ho).max())
    assert (corr == p.corr).mean() > 0.9995       # scipy fp64 tree vs fp32 nanoflann: near-ties only
    np.testing.assert_array_equal(sqd[corr == p.corr], p.sqd[corr == p.corr])
    if np.all(corr == p.corr):
        np.testing.assert_allclose(Ho, H, rtol=1e-10, atol=1e-8 * np.abs(H).max())
        np.testing.assert_allclose(bo, b, rtol=1e-10, atol=1e-8 * np.abs(b).max())
        assert abs(co - cost) <= 1e-10 * abs(cost)
    # compute_error at a different pose reuses the linearization's correspondences
    T = np.eye(4)
    T[:3, 3] = [0.01, -0.02, 0.005]
    e_np = p.compute_error(T)
    e_or = oracle.compute_error(T)
    assert abs(e_np - e_or) <= 1e-9 * abs(e_np)


def test_oracle_lm_align_vs_numpy_and_golden(s2s_golden):
    g = s2s_golden
    p = _np_problem(g)
    x, it, conv, failed = NP.align(p, None, max_iterations=32, trans_eps=5e-4)
    oracle = O.Gicp(g["src"], g["tgt"], O.default_params(k_correspondences=10, max_correspondence_distance=1.0,
                                                         max_iterations=32, transformation_epsilon=5e-4))
    oracle.set_covariances(0, g["cov_src_PLANE"])
    oracle.set_covariances(1, g["cov_tgt"])
    pose, res = oracle.align()
    np.testing.assert_allclose(pose, g["lm_pose"], atol=1e-6)
    np.testing.assert_allclose(oracle.trace(), g["lm_trace"], rtol=1e-9, atol=1e-9)
    assert res.iterations_run == int(g["lm_iters"]) == it
    assert bool(res.converged) == conv and not failed
    np.testing.assert_allclose(pose.astype(np.float64), x, atol=2e-6)
    # recovers the known rigid perturbation of the synthetic pair (16-row scan: z is weakly constrained)
    assert np.abs(pose[:2, 3] - g["T_true"][:2, 3]).max() < 0.01
    assert abs(pose[2, 3] - g["T_true"][2, 3]) < 0.05


def test_oracle_gn_fixed_vs_numpy(s2s_golden):
    g = s2s_golden
    p = _np_problem(g)
    x, it, _, _ = NP.align(p, None, max_iterations=10, lm=False, fixed_iterations=10)
    oracle = O.Gicp(g["src"], g["tgt"], O.default_params(k_correspondences=10, max_correspondence_distance=1.0,
                                                         max_iterations=10, optimizer=O.GN, fixed_iterations=10))
    oracle.set_covariances(0, g["cov_src_PLANE"])
    oracle.set_covariances(1, g["cov_tgt"])
    pose, res = oracle.align()
    assert res.iterations_run == 10 == it
    np.testing.assert_allclose(pose, g["gn_pose"], atol=1e-6)
    np.testing.assert_allclose(pose.astype(np.float64), x, atol=2e-6)


def test_oracle_s2m_golden(s2m_golden):
    g = s2m_golden
    oracle = O.Gicp(g["src"], g["sub"], O.default_params(k_correspondences=20, max_correspondence_distance=2.0,
                                                         max_iterations=32, transformation_epsilon=0.01))
    oracle.set_covariances(0, g["cov_src"])
    oracle.set_covariances(1, g["cov_sub"])
    pose, res = oracle.align(g["guess"])
    np.testing.assert_allclose(pose, g["pose"], atol=1e-6)
    assert res.iterations_run == int(g["iters"])
    p = NP.Problem(g["src"], g["sub"], NP.sym6_to_mat(g["cov_src"]), NP.sym6_to_mat(g["cov_sub"]), 2.0)
    x, it, conv, _ = NP.align(p, g["guess"], max_iterations=32, trans_eps=0.01)
    assert it == res.iterations_run
    np.testing.assert_allclose(pose.astype(np.float64), x, atol=2e-6)
    assert np.abs(pose[:3, 3] - g["T_true"][:3, 3]).max() < 0.05


# ------------------------------------------------------------- KATs
@pytest.mark.parametrize("w", [[0, 0, 0], [1e-6, 0, 0], [0.3, -0.4, 0.5], [2.0, 1.0, -1.5], [0, 0, np.pi]])
def test_so3_exp_kat(w):
    w = np.array(w, np.float64)
    R = O.so3_exp(w)
    np.testing.assert_allclose(R, NP.so3_exp(w), atol=1e-15)
    th = np.linalg.norm(w)
    # Rodrigues
    K = NP.skew(w[None])[0]
    if th > 0:
        Rr = np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K
    else:
        Rr = np.eye(3)
    np.testing.assert_allclose(R, Rr, atol=1e-12)


def test_so3_exp_small_angle_branch():
    # theta^2 = 1e-12 < 1e-10 uses the Taylor branch (so3.hpp:64-70)
    w = np.array([1e-6, 0, 0])
    R = O.so3_exp(w)
    assert abs(R[1, 2] + np.sin(1e-6)) < 1e-18 and abs(R[0, 0] - 1) < 1e-15


def test_ldlt_solve_kat():
    rng = np.random.default_rng(1)
    for _ in range(20):
        A = rng.standard_normal((6, 6))
        A = A @ A.T + 1e-3 * np.eye(6)
        b = rng.standard_normal(6)
        np.testing.assert_allclose(O.ldlt_solve6(A, b), np.linalg.solve(A, b), rtol=1e-9, atol=1e-9)
    # indefinite but non-singular (LDLT with pivoting still solves)
    A = np.diag([4.0, -2.0, 1.0, 3.0, -5.0, 2.0])
    b = np.arange(1, 7, dtype=np.float64)
    np.testing.assert_allclose(O.ldlt_solve6(A, b), b / np.diag(A), rtol=1e-14)


@pytest.mark.parametrize("reg", ["NONE", "MIN_EIG", "NORMALIZED_MIN_EIG", "PLANE", "FROBENIUS"])
def test_regularize_kat(reg):
    rng = np.random.default_rng(5)
    for _ in range(10):
        X = rng.standard_normal((3, 3)) * [1.0, 0.3, 0.01]
        C = X @ X.T
        np.testing.assert_allclose(O.regularize(C, reg), NP.regularize(C, reg), atol=1e-12)
    # PLANE on a planar neighbourhood equals I - 0.999 n n^T
    n = np.array([0.0, 0.0, 1.0])
    C = np.diag([2.0, 1.0, 0.0])
    np.testing.assert_allclose(O.regularize(C, "PLANE"), np.eye(3) - 0.999 * np.outer(n, n), atol=1e-12)
