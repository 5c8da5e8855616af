"""GPU parity of the odometry driver (include/ddlo_odom.h) against the CPU
restatement of OdomNode (oracle/odom_ref.py) and of its preprocessing
filters (oracle.crop_box_negative / oracle.voxel_grid, PCL restatements).

Tolerances:
  filtered points   same count and voxel order; coordinates within 4e-6 x the
                    cloud extent (a voxel's float sum runs in input order here,
                    in libstdc++ std::sort order in the reference)
  decisions         scan status, keyframe insertions, submap keyframe sets: exact
  poses             |dt| <= 1e-4 m, rotation entries <= 1e-4 (north star)
"""
import numpy as np
import pytest

import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import odometry as OD
from dynamic_direct_lidar_odometry_amd import scene
from oracle import oracle as O
from oracle import odom_ref as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def seq():
    return scene.odometry_sequence(32, 512, 14, cfg_id=7)


@pytest.mark.parametrize("crop,leaf", [(1.0, 0.1), (0.0, 0.25), (2.0, 0.0), (0.0, 0.05)])
def test_preprocess_vs_oracle(seq, crop, leaf):
    pts = seq[0][0]
    got = OD.preprocess(pts, crop_size=crop, leaf=leaf)
    ref = pts.astype(np.float32)
    if crop > 0:
        ref = O.crop_box_negative(ref, crop)
    if leaf > 0:
        ref = O.voxel_grid(ref, leaf)
    assert got.shape == ref.shape
    if leaf > 0:
        np.testing.assert_allclose(got, ref, rtol=0, atol=4e-6 * float(np.abs(pts).max()))
    else:
        np.testing.assert_array_equal(got, ref)


def test_preprocess_edge_cases():
    assert OD.preprocess(np.zeros((0, 3), np.float32), 1.0, 0.1).shape == (0, 3)
    inside = np.random.default_rng(0).uniform(-0.5, 0.5, (100, 3)).astype(np.float32)
    assert OD.preprocess(inside, crop_size=1.0, leaf=0.1).shape == (0, 3)     # everything inside the crop box
    one = np.array([[3.0, 4.0, 5.0]], np.float32)
    np.testing.assert_array_equal(OD.preprocess(one, 1.0, 0.1), one)
    dup = np.repeat(one, 7, axis=0)
    np.testing.assert_allclose(OD.preprocess(dup, 0.0, 0.1), one, rtol=1e-7)


def _params():
    return OD.default_odom_params(adaptive=0, keyframe_thresh_dist=0.25, submap_knn=3, submap_kcv=2, submap_kcc=2)


def test_driver_vs_oracle(seq):
    frames, _ = seq
    p = _params()
    gpu = OD.Odometry(0, p)
    ref = R.OdomRef(p)
    for i, f in enumerate(frames):
        g = gpu.process(f)
        o = ref.process(f)
        assert g.status == o["status"], i
        if g.status == OD.INIT:   # initializeDDLO consumed the scan (odom.cc:641-646): nothing else is reported
            continue
        assert g.scan_points == o["scan_points"], i
        assert g.keyframe_added == o["keyframe_added"], i
        assert abs(g.spaciousness - o["spaciousness"]) <= 1e-5 * o["spaciousness"], i
        if g.status != OD.TRACKED:
            continue
        assert g.num_keyframes == o["num_keyframes"], i
        assert gpu.submap().tolist() == o["submap"], i
        assert g.submap_changed == o["submap_changed"], i
        T = g.pose()
        np.testing.assert_allclose(T[:3, 3], o["T"][:3, 3], atol=1e-4, err_msg=f"frame {i}")
        np.testing.assert_allclose(T[:3, :3], o["T"][:3, :3], atol=1e-4, err_msg=f"frame {i}")
        np.testing.assert_allclose(np.array(g.T_s2s_local).reshape(4, 4), o["T_s2s_local"], atol=1e-4)
        assert g.s2s.iterations_run == o["s2s"].iterations_run and g.s2m.iterations_run == o["s2m"].iterations_run
    for k in range(len(ref.keyframes)):
        pose7, n = gpu.keyframe(k)
        np.testing.assert_allclose(pose7[:3], ref.keyframes[k][0], atol=1e-4)
        assert n == len(ref.keyframes[k][2])
    gpu.close()


def test_driver_default_params_tracks_ground_truth(seq):
    frames, poses = seq
    gpu = OD.Odometry(0)        # cfg/ddlo.yaml parameters, adaptive keyframe threshold
    T0inv = np.linalg.inv(poses[1])   # the first scan initialises; the second is the map origin
    statuses = []
    for i, f in enumerate(frames[:9]):
        r = gpu.process(f)
        statuses.append(r.status)
        if r.status == OD.TRACKED:
            truth = T0inv @ poses[i]
            assert np.abs(r.pose()[:3, 3] - truth[:3, 3]).max() < 0.05
            assert r.keyframe_thresh_dist in (0.5, 1.0, 5.0, 10.0)
    assert statuses == [OD.INIT, OD.FIRST] + [OD.TRACKED] * 7
    # the S2M context serves the residual image of the last scan (odom.cc:804-827)
    import ctypes as C
    ctx = C.c_void_p()
    assert gpu.L.ddlo_odom_ctx(gpu.h, 1, C.byref(ctx)) == 0
    img = np.zeros((64, 64), np.float32)
    assert P.load().gicp_residual_image(ctx, -np.pi / 3, np.pi / 3, 64, 64, img.ctypes.data_as(C.c_void_p), None) == 0
    assert np.isfinite(img).all() and (img > 0).any()
    gpu.close()


def test_driver_skips_small_scans():
    gpu = OD.Odometry(0, OD.default_odom_params(min_num_points=100))
    r = gpu.process(np.random.default_rng(0).uniform(-10, 10, (50, 3)).astype(np.float32))
    assert r.status == OD.SKIPPED and r.num_keyframes == 0
    gpu.close()
