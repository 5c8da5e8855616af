"""ctypes mirror of the odometry driver C-ABI (include/ddlo_odom.h).

``Odometry`` is the registration half of the reference's ``OdomNode``
(``src/odometry/odom.cc``): per scan the device preprocessing (crop box +
voxel filter), the spaciousness metric and adaptive keyframe threshold, S2S
then S2M GICP with pose propagation, keyframe selection and the
k-nearest / convex-hull / concave-hull submap, all point sets on the GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import GicpError, GicpParams, GicpResult, _ptr, load

__all__ = ["OdomParams", "OdomResult", "Odometry", "default_odom_params", "preprocess", "convex_hull",
           "concave_hull", "TRACKED", "FIRST", "SKIPPED", "INIT"]

TRACKED, FIRST, SKIPPED, INIT = 0, 1, 2, 3


class OdomParams(C.Structure):
    _fields_ = [
        ("s2s", GicpParams),
        ("s2m", GicpParams),
        ("min_num_points", C.c_int32),
        ("keyframe_thresh_dist", C.c_double),
        ("keyframe_thresh_rot", C.c_double),
        ("submap_knn", C.c_int32),
        ("submap_kcv", C.c_int32),
        ("submap_kcc", C.c_int32),
        ("adaptive", C.c_int32),
        ("crop_use", C.c_int32),
        ("crop_size", C.c_double),
        ("vf_scan_use", C.c_int32),
        ("vf_scan_res", C.c_double),
        ("vf_submap_use", C.c_int32),
        ("vf_submap_res", C.c_double),
        ("skip_first_scan", C.c_int32),
        ("s2m_target_grid", C.c_int32),
    ]


class OdomResult(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("scan_points", C.c_int32),
        ("T", C.c_float * 16),
        ("T_s2s", C.c_float * 16),
        ("T_s2s_local", C.c_float * 16),
        ("s2s", GicpResult),
        ("s2m", GicpResult),
        ("keyframe_added", C.c_int32),
        ("submap_changed", C.c_int32),
        ("num_keyframes", C.c_int32),
        ("submap_keyframes", C.c_int32),
        ("submap_points", C.c_int64),
        ("spaciousness", C.c_double),
        ("keyframe_thresh_dist", C.c_double),
    ]

    def pose(self) -> np.ndarray:
        return np.array(self.T, dtype=np.float32).reshape(4, 4)


_SIGS_DONE = False


def _lib():
    global _SIGS_DONE
    L = load()
    if not _SIGS_DONE:
        P, S, I, D = C.c_void_p, C.c_size_t, C.c_int, C.c_double
        sig = {
            "ddlo_odom_default_params": (I, [C.POINTER(OdomParams)]),
            "ddlo_odom_create": (I, [I, C.POINTER(OdomParams), C.POINTER(P)]),
            "ddlo_odom_destroy": (I, [P]),
            "ddlo_odom_process": (I, [P, P, S, S, C.POINTER(OdomResult)]),
            "ddlo_odom_keyframe": (I, [P, I, P, C.POINTER(S)]),
            "ddlo_odom_submap": (I, [P, P, S, C.POINTER(S)]),
            "ddlo_odom_ctx": (I, [P, I, C.POINTER(P)]),
            "ddlo_preprocess": (I, [I, P, S, S, D, D, P, S, C.POINTER(S)]),
            "ddlo_convex_hull": (I, [P, I, P, I, C.POINTER(I)]),
            "ddlo_concave_hull": (I, [P, I, D, P, I, C.POINTER(I)]),
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


def default_odom_params(**kw) -> OdomParams:
    """cfg/ddlo.yaml defaults (odom.cc:196-252)."""
    p = OdomParams()
    _check(_lib().ddlo_odom_default_params(C.byref(p)))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _xyz(points) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(points, dtype=np.float32).reshape(-1, 3))


class Odometry:
    """OdomNode registration pipeline on one GPU."""

    def __init__(self, device: int = 0, params: OdomParams | None = None):
        self.L = _lib()
        self.h = C.c_void_p()
        _check(self.L.ddlo_odom_create(device, C.byref(params) if params is not None else None, C.byref(self.h)))

    def close(self):
        if self.h:
            self.L.ddlo_odom_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, points) -> OdomResult:
        a = _xyz(points)
        r = OdomResult()
        _check(self.L.ddlo_odom_process(self.h, _ptr(a), a.shape[0], 12, C.byref(r)))
        return r

    def keyframe(self, k: int):
        pose = (C.c_float * 7)()
        n = C.c_size_t()
        _check(self.L.ddlo_odom_keyframe(self.h, k, pose, C.byref(n)))
        return np.array(pose, dtype=np.float32), n.value

    def submap(self) -> np.ndarray:
        n = C.c_size_t()
        _check(self.L.ddlo_odom_submap(self.h, None, 0, C.byref(n)))
        out = np.zeros(max(n.value, 1), np.int32)
        _check(self.L.ddlo_odom_submap(self.h, _ptr(out), out.size, C.byref(n)))
        return out[:n.value]


def preprocess(points, crop_size: float = 0.0, leaf: float = 0.0, device: int = 0) -> np.ndarray:
    """Device crop box (points inside [-s, s]^3 removed) then voxel filter."""
    a = _xyz(points)
    out = np.zeros((max(a.shape[0], 1), 3), np.float32)
    n = C.c_size_t()
    _check(_lib().ddlo_preprocess(device, _ptr(a), a.shape[0], 12, float(crop_size), float(leaf), _ptr(out),
                                  out.shape[0], C.byref(n)))
    return out[:n.value]


def convex_hull(points) -> np.ndarray:
    a = _xyz(points)
    idx = np.zeros(max(a.shape[0], 1), np.int32)
    n = C.c_int()
    _check(_lib().ddlo_convex_hull(_ptr(a), a.shape[0], _ptr(idx), idx.shape[0], C.byref(n)))
    return idx[:n.value]


def concave_hull(points, alpha: float) -> np.ndarray:
    a = _xyz(points)
    idx = np.zeros(max(a.shape[0], 1), np.int32)
    n = C.c_int()
    _check(_lib().ddlo_concave_hull(_ptr(a), a.shape[0], float(alpha), _ptr(idx), idx.shape[0], C.byref(n)))
    return idx[:n.value]
