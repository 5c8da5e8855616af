"""ctypes mirror of the range-image segmentation C-ABI (include/ddlo_segment.h).

``Segmentation`` is the part of the reference's ``DetectionModule``
(``src/detection/detection.cpp``) that OdomNode::applySegmentation drives
(``odom.cc:853-857``): projectScan, projectResiduals, groundRemoval and
cloudSegmentation / labelComponents on one organized scan.  The per-pixel
passes run on the GPU, the order-dependent labelling on the host.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import GicpError, _ptr, load

__all__ = ["SegParams", "SegResult", "Segmentation", "default_seg_params", "yaml_seg_params", "label_components",
           "EXCLUDED", "UNLABELLED", "REJECTED"]

EXCLUDED, UNLABELLED, REJECTED = -1, 0, 999999


class SegParams(C.Structure):
    _fields_ = [
        ("rows", C.c_int32),
        ("cols", C.c_int32),
        ("ang_bottom", C.c_float),
        ("ground_rows", C.c_int32),
        ("ground_angle_threshold", C.c_float),
        ("minimum_range", C.c_float),
        ("sensor_mount_angle", C.c_float),
        ("theta", C.c_float),
        ("valid_point_num", C.c_int32),
        ("min_line_num", C.c_int32),
        ("valid_line_num", C.c_int32),
        ("min_delta_z", C.c_float),
        ("max_delta_z", C.c_float),
        ("max_distance", C.c_float),
        ("max_elevation", C.c_float),
        ("win_row0", C.c_int32),
        ("win_row1", C.c_int32),
        ("win_col0", C.c_int32),
        ("win_col1", C.c_int32),
    ]

    def replace(self, **kw) -> "SegParams":
        q = SegParams()
        C.pointer(q)[0] = self
        for k, v in kw.items():
            setattr(q, k, v)
        return q


class SegResult(C.Structure):
    _fields_ = [
        ("segments", C.c_int32),
        ("ground_pixels", C.c_int32),
        ("range_pixels", C.c_int32),
        ("rejected_pixels", C.c_int32),
    ]


_SIGS_DONE = False


def _lib():
    global _SIGS_DONE
    L = load()
    if not _SIGS_DONE:
        P, S, I, F = C.c_void_p, C.c_size_t, C.c_int, C.c_float
        sig = {
            "ddlo_seg_default_params": (I, [C.POINTER(SegParams)]),
            "ddlo_seg_create": (I, [I, C.POINTER(SegParams), C.POINTER(P)]),
            "ddlo_seg_destroy": (I, [P]),
            "ddlo_seg_process": (I, [P, P, S, P, P, C.POINTER(SegResult)]),
            "ddlo_seg_images": (I, [P, P, P, P]),
            "ddlo_seg_avg_residuals": (I, [P, P, S, C.POINTER(S)]),
            "ddlo_seg_ground_indices": (I, [P, P, S, C.POINTER(S)]),
            "ddlo_seg_label_indices": (I, [P, P, S, P, S, C.POINTER(S)]),
            "ddlo_seg_label": (I, [C.POINTER(SegParams), P, P, P, F, P, P, S, C.POINTER(C.c_int32)]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _SIGS_DONE = True
    return L


def _check(st):
    if st != 0:
        raise GicpError(st, load().gicp_last_error().decode())


def default_seg_params(**kw) -> SegParams:
    """DetectionModule::loadParams code defaults (detection.cpp:77-107)."""
    p = SegParams()
    _check(_lib().ddlo_seg_default_params(C.byref(p)))
    return p.replace(**kw) if kw else p


def yaml_seg_params(**kw) -> SegParams:
    """cfg/ddlo.yaml:206-225 as ROS delivers it to loadParams: the parameters
    whose code default is an int literal are read as int (roscpp rounds a
    double yaml value to the nearest integer), so minimumRange 0.3 -> 0."""
    p = default_seg_params(rows=512, cols=512, ang_bottom=90, ground_rows=150, ground_angle_threshold=80,
                           minimum_range=0, sensor_mount_angle=0, theta=0.25, valid_point_num=10, min_line_num=2,
                           valid_line_num=4, min_delta_z=0.3, max_delta_z=2.0, max_distance=8, max_elevation=8.0)
    return p.replace(**kw) if kw else p


def label_components(p: SegParams, range_img, z_img, label_img, sensor_z: float, residual=None):
    """The host labelling alone (ddlo_seg_label) over caller images; returns
    (label image, avg residuals by label, segments)."""
    rng = np.ascontiguousarray(range_img, np.float32).reshape(-1)
    z = np.ascontiguousarray(z_img, np.float32).reshape(-1)
    lab = np.ascontiguousarray(label_img, np.int32).reshape(-1).copy()
    n = p.rows * p.cols
    if rng.size != n or z.size != n or lab.size != n:
        raise ValueError("images must have rows x cols pixels")
    res = None if residual is None else np.ascontiguousarray(residual, np.float32).reshape(-1)
    if res is not None and res.size != n:
        raise ValueError("residual image must have rows x cols pixels")
    avg = np.zeros(n + 1, np.float64)
    seg = C.c_int32()
    _check(_lib().ddlo_seg_label(C.byref(p), _ptr(rng), _ptr(z), None if res is None else _ptr(res), float(sensor_z),
                                 _ptr(lab), _ptr(avg), avg.size, C.byref(seg)))
    return lab.reshape(p.rows, p.cols), avg[: seg.value + 1], seg.value


class Segmentation:
    """DetectionModule's segmentation on device ``device`` (ddlo_seg_*)."""

    def __init__(self, device: int = 0, params: SegParams | None = None):
        self.L = _lib()
        self.params = params if params is not None else default_seg_params()
        self.h = C.c_void_p()
        _check(self.L.ddlo_seg_create(device, C.byref(self.params), C.byref(self.h)))
        self.last: SegResult | None = None

    def close(self):
        if self.h:
            self.L.ddlo_seg_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, xyz_t, T, residual=None) -> SegResult:
        """xyz_t: (rows*cols, >=3) float32 organized world-frame cloud (NaN = no return)."""
        a = np.ascontiguousarray(xyz_t, np.float32)
        if a.ndim != 2 or a.shape[0] != self.params.rows * self.params.cols or a.shape[1] < 3:
            raise ValueError("xyz_t must be (rows*cols, >=3)")
        Tm = np.ascontiguousarray(T, np.float32).reshape(16)
        res = None
        if residual is not None:
            res = np.ascontiguousarray(residual, np.float32).reshape(-1)
            if res.size != a.shape[0]:
                raise ValueError("residual image must have rows x cols pixels")
        r = SegResult()
        _check(self.L.ddlo_seg_process(self.h, _ptr(a), a.shape[1] * 4, _ptr(Tm), None if res is None else _ptr(res),
                                       C.byref(r)))
        self.last = r
        return r

    def images(self):
        H, W = self.params.rows, self.params.cols
        rng = np.empty((H, W), np.float32)
        gr = np.empty((H, W), np.int8)
        lab = np.empty((H, W), np.int32)
        _check(self.L.ddlo_seg_images(self.h, _ptr(rng), _ptr(gr), _ptr(lab)))
        return rng, gr, lab

    def avg_residuals(self) -> np.ndarray:
        n = C.c_size_t()
        _check(self.L.ddlo_seg_avg_residuals(self.h, None, 0, C.byref(n)))
        out = np.zeros(n.value, np.float64)
        _check(self.L.ddlo_seg_avg_residuals(self.h, _ptr(out), out.size, C.byref(n)))
        return out

    def ground_indices(self) -> np.ndarray:
        n = C.c_size_t()
        _check(self.L.ddlo_seg_ground_indices(self.h, None, 0, C.byref(n)))
        out = np.zeros(n.value, np.int32)
        _check(self.L.ddlo_seg_ground_indices(self.h, _ptr(out), out.size, C.byref(n)))
        return out

    def label_indices(self) -> list:
        """label_indices_i_: [None] + one int32 array of row-major pixel indices per segment."""
        n = C.c_size_t()
        _check(self.L.ddlo_seg_label_indices(self.h, None, 0, None, 0, C.byref(n)))
        L = self.last.segments if self.last is not None else 0
        off = np.zeros(L + 2, np.int32)
        idx = np.zeros(max(n.value, 1), np.int32)
        _check(self.L.ddlo_seg_label_indices(self.h, _ptr(off), off.size, _ptr(idx), idx.size, C.byref(n)))
        return [None] + [idx[off[l]:off[l + 1]] for l in range(1, L + 1)]

