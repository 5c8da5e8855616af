"""ctypes wrapper of the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, as the checker / timed CPU baseline.  The product package never
imports it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None


class GicpParams(C.Structure):
    _fields_ = [
        ("k_correspondences", C.c_int32),
        ("max_iterations", C.c_int32),
        ("max_correspondence_distance", C.c_double),
        ("transformation_epsilon", C.c_double),
        ("rotation_epsilon", C.c_double),
        ("lm_init_lambda_factor", C.c_double),
        ("regularization", C.c_int32),
        ("optimizer", C.c_int32),
        ("lm_max_iterations", C.c_int32),
        ("fixed_iterations", C.c_int32),
    ]


class GicpResult(C.Structure):
    _fields_ = [
        ("converged", C.c_int32),
        ("nr_iterations", C.c_int32),
        ("iterations_run", C.c_int32),
        ("lm_failed", C.c_int32),
        ("lm_trials", C.c_int32),
        ("num_correspondences", C.c_int32),
        ("final_cost", C.c_double),
        ("final_hessian", C.c_double * 36),
        ("lm_lambda", C.c_double),
        ("device_ms", C.c_double),
        ("linearize_ms", C.c_double),
    ]


REG = {"NONE": 0, "MIN_EIG": 1, "NORMALIZED_MIN_EIG": 2, "PLANE": 3, "FROBENIUS": 4}
GN, LM = 0, 1


def default_params(**kw) -> GicpParams:
    """Reference defaults (nano_gicp_impl.hpp:58-62, lsq_registration_impl.hpp:53-60)."""
    p = GicpParams(20, 64, float(np.finfo(np.float32).max), 5e-4, 2e-3, 1e-9, REG["PLANE"], LM, 10, 0)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def as_params(p) -> GicpParams:
    """Copy any ctypes struct / object with the gicp_params fields into the oracle's type."""
    if isinstance(p, GicpParams):
        return p
    q = GicpParams()
    for name, _ in GicpParams._fields_:
        setattr(q, name, getattr(p, name))
    return q


def _fp(a):
    return a.ctypes.data_as(C.c_void_p)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle library missing: {path} (run `make -C oracle`)")
        L = C.CDLL(path)
        L.oref_tree_build.restype = C.c_void_p
        L.oref_tree_build.argtypes = [C.c_void_p, C.c_int]
        L.oref_tree_free.argtypes = [C.c_void_p]
        L.oref_tree_knn.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        L.oref_tree_export.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.oref_covariances.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]
        L.oref_gicp_create.restype = C.c_void_p
        L.oref_gicp_create.argtypes = [C.POINTER(GicpParams), C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
        L.oref_gicp_free.argtypes = [C.c_void_p]
        L.oref_gicp_set_threads.argtypes = [C.c_void_p, C.c_int]
        L.oref_gicp_set_params.argtypes = [C.c_void_p, C.POINTER(GicpParams)]
        L.oref_gicp_set_covariances.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
        L.oref_gicp_compute_covariances.argtypes = [C.c_void_p, C.c_int]
        L.oref_gicp_get_covariances.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.oref_gicp_align.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(GicpResult)]
        L.oref_gicp_linearize.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oref_gicp_compute_error.restype = C.c_double
        L.oref_gicp_compute_error.argtypes = [C.c_void_p, C.c_void_p]
        L.oref_gicp_last_correspondences.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.oref_gicp_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.oref_voxel_grid.argtypes = [C.c_void_p, C.c_int, C.c_float, C.c_void_p]
        L.oref_so3_exp.argtypes = [C.c_void_p, C.c_void_p]
        L.oref_ldlt_solve6.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.oref_regularize.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        _LIB = L
    return _LIB


def ref_lib():
    """The reference's own nanoflann (oracle/_ref); None when it was not built."""
    global _REF
    if _REF is None:
        path = os.path.join(HERE, "_ref", "libref_nanoflann.so")
        if not os.path.exists(path):
            return None
        L = C.CDLL(path)
        L.ref_tree_build.restype = C.c_void_p
        L.ref_tree_build.argtypes = [C.c_void_p, C.c_int]
        L.ref_tree_free.argtypes = [C.c_void_p]
        L.ref_tree_knn.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.ref_tree_export.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        _REF = L
    return _REF


def _xyz(a):
    return np.ascontiguousarray(a, dtype=np.float32).reshape(-1, 3)


def knn(points, queries, k, threads=0):
    """Exact k-NN with the oracle kd-tree (nanoflann restatement)."""
    L = lib()
    pts, q = _xyz(points), _xyz(queries)
    h = L.oref_tree_build(_fp(pts), len(pts))
    idx = np.zeros((len(q), k), np.int32)
    d = np.zeros((len(q), k), np.float32)
    L.oref_tree_knn(h, _fp(q), len(q), k, _fp(idx), _fp(d), threads)
    L.oref_tree_free(h)
    return idx, d


def ref_knn(points, queries, k):
    """Exact k-NN with the REFERENCE nanoflann (oracle/_ref), or None."""
    L = ref_lib()
    if L is None:
        return None
    pts, q = _xyz(points), _xyz(queries)
    h = L.ref_tree_build(_fp(pts), len(pts))
    idx = np.zeros((len(q), k), np.int32)
    d = np.zeros((len(q), k), np.float32)
    L.ref_tree_knn(h, _fp(q), len(q), k, _fp(idx), _fp(d))
    L.ref_tree_free(h)
    return idx, d


def _export(L, build, free, export, points):
    pts = _xyz(points)
    h = build(_fp(pts), len(pts))
    cap = 2 * len(pts) + 2
    vind = np.zeros(len(pts), np.int32)
    nodes = np.zeros((cap, 4), np.int32)
    div = np.zeros((cap, 2), np.float32)
    nn = export(h, _fp(vind), _fp(nodes), _fp(div), cap)
    free(h)
    assert nn > 0, "tree export failed"
    return vind, nodes[:nn], div[:nn]


def tree(points):
    """The oracle's nanoflann tree: vind, preorder nodes (c1, c2, divfeat, -1; divfeat -1 = leaf with vind
    range [c1, c2)), (divlow, divhigh)."""
    L = lib()
    return _export(L, L.oref_tree_build, L.oref_tree_free, L.oref_tree_export, points)


def ref_tree(points):
    """The REFERENCE nanoflann's tree in the same layout (oracle/_ref), or None."""
    L = ref_lib()
    if L is None:
        return None
    return _export(L, L.ref_tree_build, L.ref_tree_free, L.ref_tree_export, points)


def same_tree(a, b):
    """Two exported trees (any node numbering) describe the same nanoflann tree: walked from the roots,
    identical leaves (vind ranges), divfeat, divlow and divhigh, then identical vind.  Returns a mismatch
    description (the first differing node's depth and its leaf / subtree vind range) or None."""
    va, na, da = a
    vb, nb, db = b
    st = [(0, 0, 0)]
    seen = 0
    while st:
        x, y, depth = st.pop()
        seen += 1
        if na[x, 2] != nb[y, 2]:
            return f"depth {depth}: node kind/divfeat differs ({x} vs {y}): {na[x, 2]} vs {nb[y, 2]}"
        if na[x, 2] < 0:
            if na[x, 0] != nb[y, 0] or na[x, 1] != nb[y, 1]:
                return f"depth {depth}: leaf range differs: {na[x, :2]} vs {nb[y, :2]}"
            if not np.array_equal(va[na[x, 0]:na[x, 1]], vb[nb[y, 0]:nb[y, 1]]):
                return f"depth {depth}: leaf {na[x, :2]} holds different points"
            continue
        if not (da[x, 0] == db[y, 0] and da[x, 1] == db[y, 1]):   # +-0 are the same split
            return f"depth {depth}: divlow/divhigh differ at ({x}, {y}): {da[x]} vs {db[y]}"
        st.append((na[x, 1], nb[y, 1], depth + 1))
        st.append((na[x, 0], nb[y, 0], depth + 1))
    if seen != min(len(na), len(nb)):   # the device numbers subtrees sparsely: only the denser export is exact
        return f"node counts differ: walked {seen}, sizes {len(na)} / {len(nb)}"
    if not np.array_equal(va, vb):
        i = int(np.argmax(va != vb))
        return f"vind differs first at {i}: {va[i]} vs {vb[i]}"
    return None


def covariances(points, k, reg="PLANE", threads=0):
    L = lib()
    pts = _xyz(points)
    out = np.zeros((len(pts), 6), np.float64)
    rc = L.oref_covariances(_fp(pts), len(pts), k, REG[reg] if isinstance(reg, str) else reg, _fp(out), threads)
    if rc:
        raise ValueError(f"oref_covariances failed ({rc})")
    return out


class Gicp:
    """The oracle NanoGICP problem (source/target fixed for its lifetime)."""

    def __init__(self, source, target, params: GicpParams | None = None, threads=0):
        self.L = lib()
        self.src = _xyz(source)
        self.tgt = _xyz(target)
        self.params = as_params(params) if params is not None else default_params()
        self.h = self.L.oref_gicp_create(C.byref(self.params), _fp(self.src), len(self.src), _fp(self.tgt), len(self.tgt), threads)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oref_gicp_free(self.h)
            self.h = None

    def set_threads(self, n):
        self.L.oref_gicp_set_threads(self.h, n)

    def set_params(self, p: GicpParams):
        p = as_params(p)
        self.params = p
        self.L.oref_gicp_set_params(self.h, C.byref(p))

    def set_covariances(self, side, cov6):
        cov6 = np.ascontiguousarray(cov6, np.float64)
        self.L.oref_gicp_set_covariances(self.h, side, _fp(cov6), len(cov6), 1)

    def compute_covariances(self, side):
        self.L.oref_gicp_compute_covariances(self.h, side)

    def get_covariances(self, side):
        n = len(self.src) if side == 0 else len(self.tgt)
        out = np.zeros((n, 6), np.float64)
        self.L.oref_gicp_get_covariances(self.h, side, _fp(out))
        return out

    def align(self, guess=None):
        out = np.zeros((4, 4), np.float32)
        res = GicpResult()
        g = None if guess is None else np.ascontiguousarray(guess, np.float32)
        self.L.oref_gicp_align(self.h, None if g is None else _fp(g), _fp(out), C.byref(res))
        return out, res

    def linearize(self, pose):
        pose = np.ascontiguousarray(pose, np.float64)
        H = np.zeros((6, 6)); b = np.zeros(6); cost = np.zeros(1)
        corr = np.zeros(len(self.src), np.int32); sqd = np.zeros(len(self.src), np.float32)
        rc = self.L.oref_gicp_linearize(self.h, _fp(pose), _fp(H), _fp(b), _fp(cost), _fp(corr), _fp(sqd))
        if rc:
            raise RuntimeError(f"oref_gicp_linearize failed ({rc})")
        return H, b, float(cost[0]), corr, sqd

    def compute_error(self, pose):
        pose = np.ascontiguousarray(pose, np.float64)
        return self.L.oref_gicp_compute_error(self.h, _fp(pose))

    def last_correspondences(self):
        corr = np.zeros(len(self.src), np.int32); sqd = np.zeros(len(self.src), np.float32)
        self.L.oref_gicp_last_correspondences(self.h, _fp(corr), _fp(sqd))
        return corr, sqd

    def trace(self):
        n = self.L.oref_gicp_trace(self.h, None, 0)
        out = np.zeros((max(n, 1), 13))
        self.L.oref_gicp_trace(self.h, _fp(out), n)
        return out[:n]


def so3_exp(w):
    w = np.ascontiguousarray(w, np.float64); R = np.zeros(9)
    lib().oref_so3_exp(_fp(w), _fp(R))
    return R.reshape(3, 3)


def ldlt_solve6(A, b):
    A = np.ascontiguousarray(A, np.float64); b = np.ascontiguousarray(b, np.float64); x = np.zeros(6)
    lib().oref_ldlt_solve6(_fp(A), _fp(b), _fp(x))
    return x


def regularize(C9, reg):
    C9 = np.ascontiguousarray(C9, np.float64); out = np.zeros(9)
    lib().oref_regularize(_fp(C9), REG[reg] if isinstance(reg, str) else reg, _fp(out))
    return out.reshape(3, 3)


def voxel_grid(points, leaf):
    """pcl::VoxelGrid (oracle/cpu_ref.cpp oref_voxel_grid): centroids in voxel-index order."""
    a = _xyz(points)
    out = np.zeros((max(len(a), 1), 3), np.float32)
    m = lib().oref_voxel_grid(_fp(a), len(a), float(leaf), _fp(out))
    return a.copy() if m < 0 else out[:m]


def crop_box_negative(points, size):
    """pcl::CropBox with setNegative(true), min (-s,-s,-s), max (s,s,s) (odom.cc:114-119):
    keeps the finite points with a coordinate below -s or above s, in order."""
    a = _xyz(points)
    fin = np.isfinite(a).all(axis=1)
    out = (a < -size).any(axis=1) | (a > size).any(axis=1)
    return a[fin & out]


def residual_image(points, residuals, theta_min=-np.pi / 3, theta_max=np.pi / 3, width=512, height=512):
    """Residual image restated from odom.cc:804-827 (projection, point order:
    the last point written to a pixel wins) and detection.cpp:203-252
    (projectResiduals: intensity -> CV_32F, empty pixels 0).  x*x + z*z in
    float32 as on PointXYZI members; atan2 / sqrt in double."""
    p = np.asarray(points, np.float32).reshape(-1, 3)
    xz2 = (p[:, 0] * p[:, 0] + p[:, 2] * p[:, 2]).astype(np.float64)
    theta = np.arctan2(p[:, 0].astype(np.float64), p[:, 2].astype(np.float64))
    phi = np.arctan2(p[:, 1].astype(np.float64), np.sqrt(xz2))
    u = ((theta - theta_min) / (theta_max - theta_min) * width).astype(np.int64)   # static_cast<int>: toward 0
    v = ((phi - theta_min) / (theta_max - theta_min) * height).astype(np.int64)
    keep = (u >= 0) & (u < width) & (v >= 0) & (v < height)
    winner = np.full(width * height, -1, np.int64)
    np.maximum.at(winner, (v * width + u)[keep], np.flatnonzero(keep))
    img = np.zeros(width * height, np.float32)
    hit = winner >= 0
    img[hit] = np.asarray(residuals, np.float64)[winner[hit]].astype(np.float32)
    return img.reshape(height, width), winner.reshape(height, width)
