"""Full-size parity (BASELINE.json configs 2 and 3) against the live oracle,
plus size-independent properties at the benchmark size."""
import numpy as np
import pytest

import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET, scene
from oracle import oracle as O
from parity import assert_cov_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cfg3():
    prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
    sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
    c = P.Context(0)
    c.set_params(P.default_params(k_correspondences=10))
    kcov = []
    for kf in prob["keyframes"]:
        c.set_source(kf)
        c.compute_covariances(SOURCE)
        kcov.append(c.get_covariances(SOURCE))
    c.close()
    prob["sub"] = sub
    prob["cov_sub"] = np.ascontiguousarray(np.concatenate(kcov)[prob["subset"]])
    return prob


def test_cfg3_covariances_vs_oracle(cfg3):
    c = P.Context(0)
    c.set_params(P.default_params(k_correspondences=10))
    c.set_source(cfg3["source"])
    c.compute_covariances(SOURCE)
    assert_cov_parity(cfg3["source"], 10, c.get_covariances(SOURCE), O.covariances(cfg3["source"], 10))
    kf = cfg3["keyframes"][0]
    c.set_source(kf)
    c.compute_covariances(SOURCE)
    assert_cov_parity(kf, 10, c.get_covariances(SOURCE), O.covariances(kf, 10))


@pytest.mark.parametrize("optimizer", ["LM", "GN20"])
def test_cfg3_s2m_align_vs_oracle(cfg3, optimizer):
    kw = dict(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32, transformation_epsilon=0.01)
    if optimizer == "GN20":
        kw.update(optimizer=0, fixed_iterations=20, max_iterations=20)
    scov = O.covariances(cfg3["source"], 10)
    c = P.Context(0)
    c.set_params(P.default_params(**kw))
    c.set_target(cfg3["sub"])
    c.set_covariances(TARGET, cfg3["cov_sub"])
    c.set_source(cfg3["source"])
    c.set_covariances(SOURCE, scov)
    guess = cfg3["guess"].astype(np.float32)
    pose, res = c.align(guess)
    o = O.Gicp(cfg3["source"], cfg3["sub"], O.default_params(**kw))
    o.set_covariances(0, scov)
    o.set_covariances(1, cfg3["cov_sub"])
    opose, ores = o.align(guess)
    assert res.iterations_run == ores.iterations_run
    assert res.converged == ores.converged and res.lm_trials == ores.lm_trials
    np.testing.assert_allclose(pose, opose, atol=1e-5)
    corr, sqd = c.correspondences()
    ocorr, osqd = o.last_correspondences()
    np.testing.assert_array_equal(corr, ocorr)
    np.testing.assert_array_equal(sqd, osqd)
    # recovers the ground truth (perturbation 0.36 m / 2 deg)
    assert np.abs(pose[:3, 3] - cfg3["T_true"][:3, 3]).max() < 0.03


def test_cfg2_s2s_gn20_vs_oracle():
    src, tgt, T = scene.s2s_pair(64, 2048, 2)
    kw = dict(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=20, optimizer=0,
              fixed_iterations=20)
    c = P.Context(0)
    c.set_params(P.default_params(**kw))
    c.set_target(tgt)
    c.set_source(src)
    pose, res = c.align()
    o = O.Gicp(src, tgt, O.default_params(**kw))
    o.set_covariances(0, c.get_covariances(SOURCE))
    o.set_covariances(1, c.get_covariances(TARGET))
    opose, ores = o.align()
    assert res.iterations_run == ores.iterations_run == 20
    np.testing.assert_allclose(pose, opose, atol=1e-5)
    assert np.abs(pose[:3, 3] - T[:3, 3]).max() < 0.02


def test_cfg3_property_roundtrip(cfg3):
    """Size-independent property: aligning the source moved by a known rigid
    transform back onto itself (target = source) recovers the inverse."""
    src = cfg3["source"]
    M = scene.make_pose([0.2, -0.1, 0.03], (0.01, -0.01, 0.03))
    moved = scene.transform(src, M)
    c = P.Context(0)
    c.set_params(P.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32))
    c.set_target(src)
    c.set_source(moved)
    pose, res = c.align()
    assert res.converged
    np.testing.assert_allclose(pose.astype(np.float64) @ M, np.eye(4), atol=2e-3)
