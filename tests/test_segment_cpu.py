"""CPU tests of the range-image segmentation (include/ddlo_segment.h, SURVEY.md
§8(f) rank 4).

* the boundary: every ddlo_seg_* symbol is exported and bound, the params
  struct has the layout the binding assumes, and with no GPU the device entry
  point fails loudly;
* the oracle (oracle/segment_ref.py, a literal restatement of
  detection.cpp:254-724) on hand-built cases whose answer follows from the
  reference's code by inspection ("parity unpinned" against the reference's
  own outputs: it needs ROS / OpenCV / PCL and ships no fixtures);
* the product's host labelling (ddlo_seg_label, the order-dependent BFS the
  north star keeps on the host) bit-exact against the oracle on random images
  (ties, NaN z, zero z, residuals, a window touching the image edges, so the
  column wrap is exercised) and on a ray-cast scan.
"""
import ctypes as C
import math
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import scene
from dynamic_direct_lidar_odometry_amd import segmentation as S
from oracle import segment_ref as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ddlo_segment.h")


def declared():
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"^\s*[\w\*]+\s*\**\s*(ddlo_seg\w*)\s*\(", txt, flags=re.M)))


def test_library_exports_and_binds_every_symbol():
    names = declared()
    assert len(names) == 9, names
    out = subprocess.run(["nm", "-D", "--defined-only", P.lib_path()], check=True, capture_output=True, text=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    assert not [n for n in names if n not in exported]
    src = open(os.path.join(ROOT, "dynamic_direct_lidar_odometry_amd", "segmentation.py")).read()
    for n in names:
        assert f'"{n}"' in src, n


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_params_layout_matches_ctypes(tmp_path):
    fields = [f for f, _ in S.SegParams._fields_]
    body = "".join(f'printf("{f} %zu\\n", offsetof(ddlo_seg_params, {f}));' for f in fields)
    c = tmp_path / "probe.c"
    c.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "ddlo_segment.h"\nint main(void){'
                 'printf("size %zu\\n", sizeof(ddlo_seg_params));' + body +
                 'printf("rsize %zu\\n", sizeof(ddlo_seg_result)); return 0;}')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                       check=True).stdout.splitlines())
    assert int(got["size"]) == C.sizeof(S.SegParams)
    assert int(got["rsize"]) == C.sizeof(S.SegResult)
    for f in fields:
        assert int(got[f]) == getattr(S.SegParams, f).offset, f


def test_defaults_are_the_code_defaults():
    p = S.default_seg_params()
    assert (p.rows, p.cols, p.ground_rows, p.valid_point_num, p.min_line_num, p.valid_line_num) == (128, 1024, 30, 15, 5, 5)
    assert p.theta == pytest.approx(math.pi / 3) and p.minimum_range == 10 and p.sensor_mount_angle == 10
    assert (p.win_row0, p.win_row1, p.win_col0, p.win_col1) == (156, 356, 156, 356)
    y = S.yaml_seg_params()
    assert (y.rows, y.cols, y.ground_rows, y.minimum_range, y.max_distance) == (512, 512, 150, 0, 8)


def _gpu():
    h = C.c_void_p()
    rc = S._lib().ddlo_seg_create(0, None, C.byref(h))
    if rc == 0:
        S._lib().ddlo_seg_destroy(h)
    return rc == 0


def test_no_gpu_fails_loudly():
    if _gpu():
        pytest.skip("a GPU is visible")
    with pytest.raises(P.GicpError) as e:
        S.Segmentation(0)
    assert e.value.status == 5


def test_bad_params_rejected():
    with pytest.raises(P.GicpError):
        S.label_components(S.default_seg_params(rows=4, cols=4, ground_rows=4), np.ones((4, 4)), np.ones((4, 4)),
                           np.zeros((4, 4)), 0.0)
    with pytest.raises(ValueError):
        S.label_components(S.default_seg_params(rows=4, cols=4, ground_rows=1), np.ones((3, 4)), np.ones((4, 4)),
                           np.zeros((4, 4)), 0.0)


# ---------------------------------------------------------------- oracle KATs

def small(H=12, W=16, **kw):
    base = dict(rows=H, cols=W, ang_bottom=15.0, ground_rows=3, win_row0=0, win_row1=H - 1, win_col0=0,
                win_col1=W - 1, theta=math.radians(60), valid_point_num=5, min_line_num=3, valid_line_num=3,
                min_delta_z=0.1, max_delta_z=3.0, max_distance=20.0, max_elevation=2.0, minimum_range=0.0,
                sensor_mount_angle=0.0, ground_angle_threshold=10.0)
    base.update(kw)
    return S.default_seg_params(**base)


def test_oracle_flat_wall_is_one_rejected_segment_and_a_box_is_feasible():
    p = small()
    H, W = p.rows, p.cols
    rng = np.full((H, W), 10.0, np.float32)
    z = np.tile(np.linspace(2.0, -1.0, H, dtype=np.float32)[:, None], (1, W))
    lab0 = np.zeros((H, W), np.int32)
    # uniform range: every neighbour passes the angle test -> one component
    # within maxDistance, 0.1 <= dz <= 3 and min_z below maxElevation
    lab, avg, n = R.label_components(p, rng, z, lab0, 0.0)
    assert n == 1 and (lab == 1).all()
    # far wall beyond maxDistance: rejected
    lab, _, n = R.label_components(p, rng * 3, z, lab0, 0.0)
    assert n == 0 and (lab == R.REJECTED).all()
    # an object at 5 m in front of a 30 m background: the edge fails the angle test
    rng2 = np.full((H, W), 30.0, np.float32)
    rng2[3:9, 4:9] = 5.0
    lab, _, n = R.label_components(p.replace(max_distance=20.0), rng2, z, lab0, 0.0)
    assert n == 1 and (lab[3:9, 4:9] == 1).all() and (lab[lab != 1] == R.REJECTED).all()


def test_oracle_else_if_quirk_in_min_max_z():
    """The first pushed pixel is always a new min (z < 1e6), so it never
    reaches the max branch (detection.cpp:630-633): a 3-pixel column whose
    first pushed pixel has the largest z gets max_z from the others."""
    p = small(H=6, W=3, valid_point_num=3, min_line_num=1, valid_line_num=1, min_delta_z=0.5, max_delta_z=3.0,
              win_col0=1, win_col1=1)
    H, W = 6, 3
    rng = np.full((H, W), 5.0, np.float32)
    lab0 = np.full((H, W), -1, np.int32)
    lab0[0:3, 1] = 0
    z = np.zeros((H, W), np.float32)
    z[0, 1], z[1, 1], z[2, 1] = 0.0, 1.0, 0.9     # seed (0,1); pushes (1,1) z=1.0 -> min; (2,1) 0.9 -> min
    lab, _, n = R.label_components(p, rng, z, lab0, 0.0)
    assert n == 0                                  # max_z stays -1e6: dz < 0 -> infeasible
    z[2, 1] = 1.6                                  # second push: not < min -> max = 1.6, dz = 0.6
    lab, _, n = R.label_components(p, rng, z, lab0, 0.0)
    assert n == 1 and (lab[0:3, 1] == 1).all()


def test_oracle_ground_marks_follow_the_bottom_up_overwrites():
    H, W = 5, 2
    xyz = np.zeros((H, W, 3), np.float32)
    xyz[..., 0] = 1.0
    xyz[..., 1] = np.arange(H)[::-1, None] + 1.0    # rows going away along y on flat ground (z = 0)
    xyz[1, 0, 0] = 0.0                             # x == 0: "no info" for the pairs touching row 1 of column 0
    rng, full = R.project_scan(xyz.reshape(-1, 3), np.eye(4), H, W, 0.0)
    g, lab = R.ground_removal(full, rng, 3, 0.0, 10.0)
    # column 1: tests at rows 4, 3, 2 are ground -> rows 1..4 marked
    assert g[:, 1].tolist() == [0, 1, 1, 1, 1]
    # column 0: rows 4, 3 ground; test(2) has upper row 1 with x == 0 -> -1 overwrites the 1 from test(3)
    assert g[:, 0].tolist() == [0, 0, -1, 1, 1]
    assert (lab[g == 1] == -1).all() and (lab[g != 1] == 0).all()
    assert R.ground_indices(g, 3).tolist() == [4 * W + 0, 3 * W + 0, 4 * W + 1, 3 * W + 1, 2 * W + 1]


# ------------------------------------------------- product host BFS vs oracle

def random_case(seed, H=24, W=32):
    rng_ = np.random.default_rng(seed)
    p = small(H, W, win_row0=2, win_row1=H - 1, win_col0=0, win_col1=W - 1, theta=0.6, valid_point_num=4,
              min_line_num=2, valid_line_num=2, min_delta_z=0.05, max_delta_z=5.0, max_distance=40.0,
              max_elevation=3.0)
    # piecewise-constant blobs plus noise so segments of several sizes form; some ties
    base = rng_.choice(np.array([4.0, 8.0, 15.0, 30.0], np.float32), size=(H // 4 + 1, W // 4 + 1))
    r = np.kron(base, np.ones((4, 4)))[:H, :W].astype(np.float32)
    r += rng_.normal(0, 0.05, (H, W)).astype(np.float32) * (rng_.random((H, W)) < 0.7)
    r[rng_.random((H, W)) < 0.05] = 0.0
    z = rng_.normal(0.5, 1.0, (H, W)).astype(np.float32)
    z[rng_.random((H, W)) < 0.05] = 0.0
    lab0 = np.where((r == 0) | (rng_.random((H, W)) < 0.05), -1, 0).astype(np.int32)
    res = np.where(rng_.random((H, W)) < 0.6, rng_.random((H, W)), 0).astype(np.float32)
    return p, r, z, lab0, res


@pytest.mark.parametrize("seed", range(6))
def test_host_labelling_matches_oracle_random(seed):
    p, r, z, lab0, res = random_case(seed)
    for resid in (res, None):
        lab, avg, n = S.label_components(p, r, z, lab0, 0.25, resid)
        olab, oavg, on = R.label_components(p, r, z, lab0, 0.25, resid)
        assert n == on
        assert np.array_equal(lab, olab)
        assert np.array_equal(avg, oavg)
    assert (lab == R.REJECTED).any() and n >= 1


def test_host_labelling_matches_oracle_on_a_raycast_scan():
    sc = scene.make_scene(1011, moving=True)
    pose = scene.make_pose([1.0, 0.5, scene.SENSOR_Z])
    pts = scene.raycast(sc, pose, 128, 256, 1011, organized=True)
    xyz_t = scene.transform(np.nan_to_num(pts, nan=0.0), pose).astype(np.float32)
    xyz_t[~np.isfinite(pts).all(axis=1)] = np.nan
    p = S.yaml_seg_params(rows=128, cols=256, ground_rows=40, win_row0=20, win_row1=100, win_col0=40, win_col1=200)
    T = pose.astype(np.float32)
    rng, full = R.project_scan(xyz_t, T, p.rows, p.cols, p.minimum_range)
    g, lab0 = R.ground_removal(full, rng, p.ground_rows, p.sensor_mount_angle, p.ground_angle_threshold)
    z = xyz_t[:, 2].reshape(p.rows, p.cols)
    res = np.abs(np.random.default_rng(1).normal(0, 0.1, (p.rows, p.cols))).astype(np.float32)
    lab, avg, n = S.label_components(p, rng, z, lab0, float(T[2, 3]), res)
    olab, oavg, on = R.label_components(p, rng, z, lab0, float(T[2, 3]), res)
    assert n == on and np.array_equal(lab, olab) and np.array_equal(avg, oavg)
    assert (g == 1).sum() > 1000
