"""TEST INFRASTRUCTURE ONLY — CPU restatement of DDLO's range-image
segmentation, the checker for include/ddlo_segment.h.
Only tests/ may import it; the product never does.

Follows DetectionModule (reference src/detection/detection.cpp) literally,
in the reference's own loop order:
  project_scan        projectScan         :292-329
  ground_removal      groundRemoval       :458-504 (column walk from the bottom,
                                          later writes overwrite earlier ones)
  label_components    cloudSegmentation   :519-522 + labelComponents :544-724
Float semantics: ddlo.h:35 includes <stdlib.h>, so the unqualified abs /
atan2 / sqrt calls on floats are libstdc++'s float overloads; atan2f is taken
from the C library itself (the function the reference's float overload
calls), products and sums in float32.

Parity: the reference needs ROS, OpenCV and PCL (absent here) and ships no
fixtures for this path, so it is "parity unpinned" against the reference's
own outputs; tests/test_segment_cpu.py pins the restatement's behaviour on
hand-built cases.
"""
from __future__ import annotations

import ctypes as C
import ctypes.util

import numpy as np

_libm = C.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.atan2f.restype = C.c_float
_libm.atan2f.argtypes = [C.c_float, C.c_float]
F32 = np.float32
REJECTED = 999999


def atan2f(y, x) -> np.float32:
    return F32(_libm.atan2f(float(y), float(x)))


def project_scan(xyz_t: np.ndarray, T: np.ndarray, rows: int, cols: int, minimum_range: float):
    """projectScan (:292-329): range_mat_ and full_cloud_ (NaN where no range)."""
    p = np.asarray(xyz_t, np.float32)[:, :3].reshape(rows * cols, 3)
    T = np.asarray(T, np.float32)
    x0, y0, z0 = -T[0, 3], -T[1, 3], -T[2, 3]
    finite = np.isfinite(p).all(axis=1)
    with np.errstate(invalid="ignore"):
        x = p[:, 0] + x0
        y = p[:, 1] + y0
        z = p[:, 2] + z0
        r = np.sqrt((x * x + y * y) + z * z)
        keep = finite & ~(r < F32(minimum_range))
    rng = np.where(keep, r, F32(0)).astype(np.float32)
    full = np.where(keep[:, None], p, F32(np.nan)).astype(np.float32)
    return rng.reshape(rows, cols), full.reshape(rows, cols, 3)


def ground_removal(full: np.ndarray, rng: np.ndarray, ground_rows: int, mount: float, thr: float):
    """groundRemoval (:458-504): ground_mat_ (int8) and the -1 / 0 label_mat_.
    Vectorised over columns; rows in the reference's bottom-up order."""
    H, W = rng.shape
    ground = np.zeros((H, W), np.int8)
    for ri in range(ground_rows):
        row = H - 1 - ri
        lo, up = full[row], full[row - 1]
        noinfo = (lo[:, 0] == 0) | (up[:, 0] == 0)
        with np.errstate(invalid="ignore"):
            d = up - lo
            s = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1])
            a = np.array([atan2f(dz, sv) for dz, sv in zip(d[:, 2], s)], np.float32)
            angle = ((a * F32(180)).astype(np.float64) / np.pi).astype(np.float32)
            g = np.abs(angle - F32(mount)) <= F32(thr)
        ground[row, noinfo] = -1
        hit = ~noinfo & g
        ground[row, hit] = 1
        ground[row - 1, hit] = 1
    label = np.where((ground == 1) | (rng == 0), -1, 0).astype(np.int32)
    return ground, label


def _trig(rows: int, cols: int, ang_bottom: float):
    """loadParams :82-83,108-111."""
    ang_res_x = F32(360.0 / float(F32(cols)))
    ang_res_y = F32(F32(2) * F32(ang_bottom)) / F32(rows - 1)
    sx = F32(np.sin(float(ang_res_x) / 180.0 * np.pi))
    cx = F32(np.cos(float(ang_res_x) / 180.0 * np.pi))
    sy = F32(np.sin(float(ang_res_y) / 180.0 * np.pi))
    cy = F32(np.cos(float(ang_res_y) / 180.0 * np.pi))
    return sx, cx, sy, cy


def label_components(p, rng: np.ndarray, z: np.ndarray, label: np.ndarray, sensor_z: float, residual=None):
    """cloudSegmentation seeds (:519-522) + labelComponents (:544-724).
    ``p`` has the ddlo_seg_params fields.  Returns (label, avg_residuals, segments)."""
    H, W = rng.shape
    rng = rng.astype(np.float32)
    z = np.asarray(z, np.float32).reshape(H, W)
    label = label.astype(np.int64).copy()
    res = None if residual is None else np.asarray(residual, np.float32).reshape(H, W)
    sx, cx, sy, cy = _trig(H, W, p.ang_bottom)
    theta = F32(p.theta)

    def valid(i, j):
        return p.win_row0 <= i <= p.win_row1 and p.win_col0 <= j <= p.win_col1

    label_count = 1
    avg = [0.0]
    neighbors = [(-1, 0), (0, 1), (0, -1), (1, 0)]   # neighbor_iterator_ :133-145
    for i in range(H):
        for j in range(W):
            if not (label[i, j] == 0 and valid(i, j)):
                continue
            line_flag = [False] * H
            queue = [(i, j)]
            qs = 0
            min_z, max_z, min_dist, max_dist = F32(1e6), F32(-1e6), F32(1e6), F32(-1e6)
            res_count, total = 0, F32(0)
            pushed = [(i, j)]
            while qs < len(queue):
                fy, fx = queue[qs]
                qs += 1
                label[fy, fx] = label_count
                for dy, dx in neighbors:
                    ty, tx = fy + dy, fx + dx
                    if ty < 0 or ty >= H:
                        continue
                    if not valid(ty, tx):
                        continue
                    if tx < 0:
                        tx = W - 1
                    if tx >= W:
                        tx = 0
                    if label[ty, tx] != 0:
                        continue
                    d1 = max(rng[fy, fx], rng[ty, tx])
                    d2 = min(rng[fy, fx], rng[ty, tx])
                    sa, ca = (sx, cx) if dy == 0 else (sy, cy)
                    angle = atan2f(F32(d2 * sa), F32(d1 - F32(d2 * ca)))
                    if angle > theta:
                        zz = float(z[ty, tx])
                        if zz < float(min_z) and zz != 0:
                            min_z = F32(zz)
                        elif zz > float(max_z):
                            max_z = F32(zz)
                        min_dist = min(min_dist, min(d1, d2))
                        max_dist = max(max_dist, max(d1, d2))
                        queue.append((ty, tx))
                        label[ty, tx] = label_count
                        line_flag[ty] = True
                        pushed.append((ty, tx))
                        if res is not None and res[ty, tx] > 0:
                            total = F32(total + res[ty, tx])
                            res_count += 1
            lines = sum(line_flag)
            feasible = False
            if len(pushed) >= 50 and lines >= p.min_line_num:
                feasible = True
            elif len(pushed) >= p.valid_point_num and lines >= p.valid_line_num:
                feasible = True
            if feasible:
                feasible = bool(max_dist <= F32(p.max_distance))
            if feasible:
                dz = F32(max_z - min_z)
                feasible = bool(F32(p.min_delta_z) <= dz <= F32(p.max_delta_z))
            a = 0.0
            if feasible and res is not None:
                a = float(F32(total / F32(res_count))) if res_count > 0 else 0.0
            if feasible:
                feasible = bool(F32(min_z - F32(sensor_z)) <= F32(p.max_elevation))
            if feasible:
                avg.append(a)
                label_count += 1
            else:
                for (py, px) in pushed:
                    label[py, px] = REJECTED
    return label.astype(np.int32), np.array(avg), label_count - 1


def segment(p, xyz_t: np.ndarray, T: np.ndarray, residual=None):
    """The whole DetectionModule pass ddlo_seg_process replaces: returns
    (range, ground, label, avg_residuals, segments)."""
    T = np.asarray(T, np.float32).reshape(4, 4)
    rng, full = project_scan(xyz_t, T, p.rows, p.cols, p.minimum_range)
    ground, label = ground_removal(full, rng, p.ground_rows, p.sensor_mount_angle, p.ground_angle_threshold)
    z = np.asarray(xyz_t, np.float32)[:, 2].reshape(p.rows, p.cols)
    label, avg, nseg = label_components(p, rng, z, label, float(T[2, 3]), residual)
    return rng, ground, label, avg, nseg


def ground_indices(ground: np.ndarray, ground_rows: int) -> np.ndarray:
    """getGroundIndices (:1002-1013)."""
    H, W = ground.shape
    out = [(H - 1 - ri) * W + col for col in range(W) for ri in range(ground_rows) if ground[H - 1 - ri, col] == 1]
    return np.array(out, np.int32)
