"""CPU tests of the odometry driver's boundary (include/ddlo_odom.h) and of the
oracle pieces it is checked against: the header's entry points are exported
and bound, the struct layouts match the ctypes mirror, the keyframe hulls
equal qhull's (scipy wraps the library pcl::ConvexHull uses), the oracle
VoxelGrid / CropBox restatements agree with an independent numpy
restatement, and the driver fails loudly without a GPU."""
import ctypes as C
import os
import re
import shutil
import subprocess

import numpy as np
import pytest
from scipy.spatial import ConvexHull

import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import odometry as OD
from oracle import oracle as O
from oracle import odom_ref as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ddlo_odom.h")


def declared():
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"^\s*[\w\*]+\s*\**\s*(ddlo_\w+)\s*\(", txt, flags=re.M)))


def test_odom_symbols_exported_and_bound():
    names = declared()
    assert {"ddlo_odom_create", "ddlo_odom_process", "ddlo_odom_destroy", "ddlo_preprocess"} <= set(names)
    out = subprocess.run(["nm", "-D", "--defined-only", P.lib_path()], check=True, capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    assert not [n for n in names if n not in exported]
    src = open(os.path.join(ROOT, "dynamic_direct_lidar_odometry_amd", "odometry.py")).read()
    assert not [n for n in names if f'"{n}"' not in src]


PROBE = r"""
#include <stddef.h>
#include <stdio.h>
#include "ddlo_odom.h"
#define F(T, m) printf(#T "." #m " %zu %zu\n", offsetof(T, m), sizeof(((T*)0)->m));
int main(void) {
  printf("params %zu 0\nresult %zu 0\n", sizeof(ddlo_odom_params), sizeof(ddlo_odom_result));
  F(ddlo_odom_params, s2m) F(ddlo_odom_params, min_num_points) F(ddlo_odom_params, keyframe_thresh_dist)
  F(ddlo_odom_params, submap_kcc) F(ddlo_odom_params, adaptive) F(ddlo_odom_params, crop_size)
  F(ddlo_odom_params, vf_submap_res)
  F(ddlo_odom_result, T) F(ddlo_odom_result, s2s) F(ddlo_odom_result, s2m) F(ddlo_odom_result, keyframe_added)
  F(ddlo_odom_result, submap_points) F(ddlo_odom_result, keyframe_thresh_dist)
  return 0;
}
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_odom_struct_layout(tmp_path):
    c = tmp_path / "probe.c"
    c.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    lines = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {l.split()[0]: (int(l.split()[1]), int(l.split()[2])) for l in lines if l}
    assert got["params"][0] == C.sizeof(OD.OdomParams)
    assert got["result"][0] == C.sizeof(OD.OdomResult)
    for T, tn, names in ((OD.OdomParams, "ddlo_odom_params", ["s2m", "min_num_points", "keyframe_thresh_dist", "submap_kcc", "adaptive",
                                      "crop_size", "vf_submap_res"]),
                     (OD.OdomResult, "ddlo_odom_result", ["T", "s2s", "s2m", "keyframe_added", "submap_points", "keyframe_thresh_dist"])):
        for n in names:
            assert getattr(T, n).offset == got[f"{tn}.{n}"][0], n


def test_default_odom_params_are_the_yaml():
    p = OD.default_odom_params()   # cfg/ddlo.yaml:158-204
    assert (p.s2s.k_correspondences, p.s2s.max_correspondence_distance, p.s2s.max_iterations) == (10, 1.0, 32)
    assert (p.s2m.k_correspondences, p.s2m.max_correspondence_distance, p.s2m.max_iterations) == (20, 2.0, 32)
    assert p.s2s.transformation_epsilon == p.s2m.transformation_epsilon == 0.01
    assert (p.min_num_points, p.keyframe_thresh_dist, p.keyframe_thresh_rot) == (10, 1.0, pytest.approx(0.1))
    assert (p.submap_knn, p.submap_kcv, p.submap_kcc, p.adaptive) == (10, 10, 10, 1)
    assert (p.crop_use, p.crop_size, p.vf_scan_use, p.vf_scan_res, p.vf_submap_use, p.vf_submap_res) == \
        (1, 1.0, 1, pytest.approx(0.1), 1, pytest.approx(0.1))


def test_odometry_without_gpu_fails_loudly():
    if os.environ.get("HIP_VISIBLE_DEVICES") is None and P.load().gicp_ctx_create is None:
        pytest.skip("no library")
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(P.GicpError) as e:
        OD.Odometry(0)
    assert e.value.status in (1, 5)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_convex_hull_matches_qhull(seed):
    """pcl::ConvexHull with setDimension(3) (odom.cc:87): qhull's 3-D vertex set; a flat keyframe set is qhull's
    flat-simplex error, i.e. no convex keyframes at all."""
    rng = np.random.default_rng(seed)
    solid = rng.uniform(-20, 20, (80, 3)).astype(np.float32)
    np.testing.assert_array_equal(OD.convex_hull(solid), np.sort(ConvexHull(solid).vertices))
    assert OD.convex_hull(solid).tolist() == R.convex_hull(solid)
    thin = rng.uniform(-20, 20, (60, 3)).astype(np.float32)   # a ground vehicle's keyframes: z varies by cm
    thin[:, 2] = (1.5 + rng.normal(0, 0.02, 60)).astype(np.float32)
    np.testing.assert_array_equal(OD.convex_hull(thin), np.sort(ConvexHull(thin).vertices))
    flat = thin.copy()
    flat[:, 2] = 1.5
    assert OD.convex_hull(flat).tolist() == [] == R.convex_hull(flat)
    assert OD.convex_hull(solid[:3]).tolist() == []


def test_convex_hull_of_a_trajectory():
    from dynamic_direct_lidar_odometry_amd import scene
    poses = scene.trajectory(400, 1007)
    kf = np.array([p[:3, 3] for p in poses[::10]], np.float32)
    kf[:, 2] += np.random.default_rng(4).normal(0, 0.01, len(kf)).astype(np.float32)   # estimated poses: never level
    np.testing.assert_array_equal(OD.convex_hull(kf), np.array(R.convex_hull(kf)))
    assert len(OD.convex_hull(kf)) >= 3


def _alpha_shape_cases():
    rng = np.random.default_rng(3)
    blob = (rng.standard_normal((60, 3)) * [4, 4, 2]).astype(np.float32)            # interior points
    box = rng.uniform(-10, 10, (50, 3)).astype(np.float32)
    shell = rng.standard_normal((40, 3))
    shell = (shell / np.linalg.norm(shell, axis=1, keepdims=True) * 6).astype(np.float32)
    ring = np.concatenate([shell, (rng.standard_normal((15, 3)) * 0.8).astype(np.float32)])   # hollow + core
    return {"blob": blob, "box": box, "shell_core": ring}


@pytest.mark.parametrize("name", ["blob", "box", "shell_core"])
@pytest.mark.parametrize("alpha", [0.8, 2.0, 4.0, 50.0, 1e7])
def test_concave_hull_is_qhull_alpha_shape(name, alpha):
    """pcl::ConcaveHull with setDimension(3): the boundary vertices of the alpha shape of qhull's "d QJ" 3-D
    Delaunay (oracle via scipy's qhull); interior keyframes are not on it."""
    P3 = _alpha_shape_cases()[name]
    got = OD.concave_hull(P3, alpha).tolist()
    assert got == R.concave_hull(P3, alpha)
    if alpha == 1e7:   # every tetrahedron good: the boundary is the convex hull
        assert got == OD.convex_hull(P3).tolist()


def test_concave_hull_excludes_interior_keyframes():
    rng = np.random.default_rng(11)
    g = np.stack(np.meshgrid(np.arange(6), np.arange(6), np.arange(4), indexing="ij"), -1).reshape(-1, 3)
    P3 = (g + rng.uniform(-0.05, 0.05, g.shape)).astype(np.float32)   # a jittered 6 x 6 x 4 block of keyframes
    got = set(OD.concave_hull(P3, 1.5).tolist())
    assert got == set(R.concave_hull(P3, 1.5))
    interior = {i for i, p in enumerate(g) if 0 < p[0] < 5 and 0 < p[1] < 5 and 0 < p[2] < 3}
    assert interior and not (got & interior)
    assert got                                           # the block's faces are


def test_concave_hull_of_a_straight_path_is_empty():
    """Collinear keyframes: every Delaunay triangle is a sliver of huge circumradius."""
    P3 = np.stack([np.arange(12, dtype=np.float32), np.zeros(12, np.float32), np.zeros(12, np.float32)], 1)
    P3[:, 1] = (np.arange(12) % 2) * np.float32(1e-3)
    P3[:, 2] = (np.arange(12) % 3) * np.float32(1e-3)
    assert OD.concave_hull(P3, 1.0).tolist() == []


def test_push_submap_indices_keeps_ties():
    out = []
    R.push_submap_indices([3.0, 1.0, 2.0, 1.0, 5.0], 2, [10, 11, 12, 13, 14], out)
    assert out == [11, 13]          # k-th smallest is 1.0: both ties kept (odom.cc:1207-1212)
    out = []
    R.push_submap_indices([3.0, 1.0], 5, [7, 8], out)
    assert out == [7, 8]


def numpy_voxel_grid(pts, leaf):
    """Independent restatement: lexicographic voxel index, stable sort, float64 mean -> float32."""
    inv = np.float32(1.0) / np.float32(leaf)
    mn = pts.min(0)
    minb = np.floor(mn * inv).astype(np.int64)
    maxb = np.floor(pts.max(0) * inv).astype(np.int64)
    div = maxb - minb + 1
    ijk = (np.floor(pts * inv) - minb.astype(np.float32)).astype(np.int64)
    idx = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    order = np.argsort(idx, kind="stable")
    u, start, cnt = np.unique(idx[order], return_index=True, return_counts=True)
    sums = np.add.reduceat(pts[order].astype(np.float64), start, axis=0)
    return (sums / cnt[:, None]).astype(np.float32)


@pytest.mark.parametrize("leaf", [0.1, 0.25, 1.0])
def test_oracle_voxel_grid_vs_numpy(leaf):
    from dynamic_direct_lidar_odometry_amd import scene
    pts = scene.raycast(scene.make_scene(1001), scene.make_pose([0, 0, 1.5]), 32, 512, seed=3)
    v = O.voxel_grid(pts, leaf)
    ref = numpy_voxel_grid(pts, leaf)
    assert v.shape == ref.shape
    np.testing.assert_allclose(v, ref, rtol=0, atol=4e-6 * max(1.0, float(np.abs(pts).max())))


def test_oracle_crop_box():
    rng = np.random.default_rng(5)
    pts = rng.uniform(-2, 2, (5000, 3)).astype(np.float32)
    pts[:3] = [[1.0, 0.0, 0.0], [1.0000001, 0.0, 0.0], [np.nan, 5.0, 5.0]]
    out = O.crop_box_negative(pts, 1.0)
    inside = (np.abs(pts) <= 1.0).all(axis=1)
    np.testing.assert_array_equal(out, pts[~inside & np.isfinite(pts).all(axis=1)])
    assert not (out == [1.0, 0.0, 0.0]).all(axis=1).any()       # the boundary is inside the box
