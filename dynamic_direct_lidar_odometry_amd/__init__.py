"""MI355X-native GICP scan-matching core (drop-in for DDLO's NanoGICP S2S/S2M path).

The product is the C-ABI library ``_lib/libddlo_gicp.so`` (HIP kernels for
gfx950 + host runtime, declared in ``include/ddlo_gicp.h``).  This module is a
thin ctypes mirror of the reference's ``nano_gicp::NanoGICP`` surface
(reference ``include/nano_gicp/nano_gicp.hpp:58-148``) used by the tests and
``bench.py``; the C++ facade for native callers is ``include/nano_gicp/nano_gicp.hpp``.

There is no CPU fallback: if the HIP library is missing or no device is
visible, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import sys

import numpy as np

__all__ = ["GicpParams", "GicpResult", "Context", "NanoGICP", "GicpError", "lib_path", "load", "s2s_batch",
           "REG_NONE", "REG_MIN_EIG", "REG_NORMALIZED_MIN_EIG", "REG_PLANE", "REG_FROBENIUS",
           "GAUSS_NEWTON", "LEVENBERG_MARQUARDT", "SOURCE", "TARGET"]

REG_NONE, REG_MIN_EIG, REG_NORMALIZED_MIN_EIG, REG_PLANE, REG_FROBENIUS = range(5)
GAUSS_NEWTON, LEVENBERG_MARQUARDT = 0, 1
SOURCE, TARGET = 0, 1
COV_MAT4D, COV_SYM6 = 0, 1

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

STATUS = {0: "GICP_OK", 1: "GICP_EINVAL", 2: "GICP_ENOTARGET", 3: "GICP_ENOSOURCE", 4: "GICP_ETOOFEW",
          5: "GICP_EHIP", 6: "GICP_ENOMEM", 7: "GICP_ESTATE", 8: "GICP_ENONFINITE", 9: "GICP_ECOMM"}


class GicpError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"{STATUS.get(status, status)}: {msg}")
        self.status = status


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

    def replace(self, **kw):
        p = GicpParams()
        C.pointer(p)[0] = self
        for k, v in kw.items():
            setattr(p, k, v)
        return p


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
        ("ties_resolved", C.c_int32),
        ("tie_reruns", C.c_int32),
    ]


class GicpGridInfo(C.Structure):
    _fields_ = [
        ("built", C.c_int32),
        ("build_ms", C.c_float),
        ("cell_size", C.c_float),
        ("bytes", C.c_int64),
        ("coarse_cells", C.c_int64),
        ("band_cells", C.c_int64),
        ("nomatch_cells", C.c_int64),
        ("overflow_cells", C.c_int64),
        ("level_cells", C.c_int64 * 4),
        ("fine_cells", C.c_int64),
        ("fallback_fine", C.c_int64),
        ("entries", C.c_int64),
        ("uses_walk", C.c_int64),
        ("build_status", C.c_int64),
        ("scratch_bytes", C.c_int64),
    ]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["level_cells"] = list(self.level_cells)
        return d


GRID_OFF, GRID_AUTO, GRID_ON = 0, 1, 2


def lib_path() -> str:
    # DDLO_GICP_LIB: an alternative in-tree build of the same library (A/B runs)
    return os.environ.get("DDLO_GICP_LIB") or os.path.join(_HERE, "_lib", "libddlo_gicp.so")


def load():
    """Load the HIP library (raises if it was not built — no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        raise RuntimeError(f"HIP library not built: {path} (run __graft_entry__.build() or `make lib`)")
    # PyTorch-ROCm ships its own libamdhip64.so.7 and librccl.so.1 under the
    # same sonames as /opt/rocm's: whichever loads first serves the whole
    # process.  Loading this library (ROCm's) first and torch afterwards (e.g.
    # torch.distributed for the shard ranks' unique id) leaves torch's other
    # bundled libraries on ROCm's runtime, and the process aborts in its exit
    # teardown.  So torch, when installed, loads first (then the library runs
    # on torch's bundled HIP runtime).  A process that never imports torch can
    # set DDLO_TORCH_FIRST=0 to skip that import: the library then binds to
    # the ROCm runtime it was linked against (its RUNPATH, /opt/rocm), as a C++
    # host does (tests/test_gpu_process.py).
    if "torch" not in sys.modules and os.environ.get("DDLO_TORCH_FIRST", "1") != "0":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = C.CDLL(path)
    P, S, I, D = C.c_void_p, C.c_size_t, C.c_int, C.c_double
    sig = {
        "gicp_abi_version": (C.c_int32, []),
        "gicp_last_error": (C.c_char_p, []),
        "gicp_default_params": (I, [C.POINTER(GicpParams)]),
        "gicp_ctx_create": (I, [I, C.POINTER(P)]),
        "gicp_ctx_destroy": (I, [P]),
        "gicp_set_params": (I, [P, C.POINTER(GicpParams)]),
        "gicp_get_params": (I, [P, C.POINTER(GicpParams)]),
        "gicp_set_source": (I, [P, P, S, S, I]),
        "gicp_set_target": (I, [P, P, S, S]),
        "gicp_clear_source": (I, [P]),
        "gicp_clear_target": (I, [P]),
        "gicp_get_size": (I, [P, I, C.POINTER(S)]),
        "gicp_compute_covariances": (I, [P, I]),
        "gicp_set_covariances": (I, [P, I, P, S, I]),
        "gicp_get_covariances": (I, [P, I, P, S, I]),
        "gicp_has_covariances": (I, [P, I, C.POINTER(I)]),
        "gicp_swap_source_target": (I, [P]),
        "gicp_share_source": (I, [P, P]),
        "gicp_align": (I, [P, P, P, C.POINTER(GicpResult)]),
        "gicp_get_residuals": (I, [P, P, S]),
        "gicp_get_correspondences": (I, [P, P, P, S]),
        "gicp_transform_source": (I, [P, P, S, S]),
        "gicp_linearize": (I, [P, P, P, P, P, P]),
        "gicp_knn_target": (I, [P, P, S, S, I, P, P]),
        "gicp_get_moments": (I, [P, P]),
        "gicp_set_profiling": (I, [P, I]),
        "gicp_debug_stats": (I, [P, I, P, S, C.POINTER(S)]),
        "gicp_get_stream": (I, [P, C.POINTER(P)]),
        "gicp_synchronize": (I, [P]),
        "gicp_set_shard": (I, [P, I, C.c_float, C.c_float]),
        "gicp_set_shard_groups": (I, [P, I, I]),
        "gicp_set_tie_target": (I, [P, P, C.c_size_t, C.c_size_t, P, C.c_size_t]),
        "gicp_get_stage_times": (I, [P, P]),
        "gicp_comm_unique_id": (I, [P, S]),
        "gicp_set_comm": (I, [P, P, S, I, I]),
        "gicp_get_comm_info": (I, [P, C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
        "gicp_s2s_batch": (I, [I, C.POINTER(GicpParams), P, P, S, I, I, P, P]),
        "gicp_residual_image": (I, [P, D, D, I, I, P, P]),
        "gicp_set_tie_order": (I, [P, I]),
        "gicp_get_tie_order": (I, [P, C.POINTER(C.c_int)]),
        "gicp_set_option": (I, [P, I, I]),
        "gicp_get_option": (I, [P, I, C.POINTER(C.c_int)]),
        "gicp_set_default_option": (I, [I, I]),
        "gicp_get_default_option": (I, [I, C.POINTER(C.c_int)]),
        "gicp_tie_builder_set": (I, [P, P, C.c_size_t, C.c_size_t]),
        "gicp_tie_builder_export": (I, [P, P, C.c_size_t, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
        "gicp_set_tie_tree": (I, [P, P, C.c_size_t]),
        "gicp_set_tie_trees_from_root": (I, [P, I, P, P]),
        "gicp_get_device_bytes": (I, [P, C.POINTER(C.c_int64), I]),
        "gicp_debug_nftree": (I, [P, I, P, P, P, S, C.POINTER(S)]),
        "gicp_debug_nfbuild": (I, [P, I, I, P, P, P, P, S]),
        "gicp_set_target_grid": (I, [P, I]),
        "gicp_get_target_grid_info": (I, [P, C.POINTER(GicpGridInfo)]),
        "gicp_get_lookup_stats": (I, [P, C.POINTER(C.c_int64)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


def default_params(**kw) -> GicpParams:
    p = GicpParams()
    load().gicp_default_params(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _xyz(points):
    a = np.asarray(points)
    if a.dtype == np.float32 and a.ndim == 2 and a.shape[1] >= 3 and a.flags.c_contiguous:
        return a, a.strides[0]
    a = np.ascontiguousarray(np.asarray(points, dtype=np.float32).reshape(-1, 3))
    return a, 12


OPT_TIE_ORDER, OPT_TIE_LAZY, OPT_TIE_PARTIAL_LEVELS, OPT_COV_TASKS, OPT_GRID_MAX_MB = 1, 2, 3, 4, 5


def set_default_option(option: int, value: int):
    """The value contexts created from now on start with (gicp_set_default_option; process-wide)."""
    L = load()
    rc = L.gicp_set_default_option(int(option), int(value))
    if rc != 0:
        raise GicpError(rc, L.gicp_last_error().decode())


def get_default_option(option: int) -> int:
    L = load()
    v = C.c_int(0)
    rc = L.gicp_get_default_option(int(option), C.byref(v))
    if rc != 0:
        raise GicpError(rc, L.gicp_last_error().decode())
    return int(v.value)


class default_option:
    """Context manager: contexts created inside the block start with option = value."""

    def __init__(self, option: int, value: int):
        self.option, self.value = option, value

    def __enter__(self):
        self.old = get_default_option(self.option)
        set_default_option(self.option, self.value)
        return self

    def __exit__(self, *a):
        set_default_option(self.option, self.old)


def comm_unique_id() -> bytes:
    """ncclGetUniqueId (128 bytes) for gicp_set_comm; make it on one rank and broadcast."""
    L = load()
    buf = (C.c_uint8 * 128)()
    rc = L.gicp_comm_unique_id(C.cast(buf, C.c_void_p), 128)
    if rc != 0:
        raise GicpError(rc, L.gicp_last_error().decode())
    return bytes(buf)


def s2s_batch(frames, params: GicpParams | None = None, device: int = 0, nstreams: int = 4):
    """Frame-parallel S2S over a scan sequence (gicp_s2s_batch; odom.cc:754-768).

    frames: list of (N_t, 3) float32 clouds in sensor frames.  Returns
    (poses (T, 4, 4) float32, results list): poses[t] aligns scan t onto scan
    t-1 (poses[0] = identity)."""
    L = load()
    p = params if params is not None else default_params()
    arrs = [np.ascontiguousarray(np.asarray(f, np.float32).reshape(-1, 3)) for f in frames]
    n = len(arrs)
    ptrs = (C.c_void_p * n)(*[a.ctypes.data for a in arrs])
    sizes = (C.c_size_t * n)(*[len(a) for a in arrs])
    out = np.zeros((n, 4, 4), np.float32)
    res = (GicpResult * n)()
    rc = L.gicp_s2s_batch(device, C.byref(p), C.cast(ptrs, C.c_void_p), C.cast(sizes, C.c_void_p), 12, n,
                          nstreams, _ptr(out), C.cast(res, C.c_void_p))
    if rc != 0:
        raise GicpError(rc, L.gicp_last_error().decode())
    return out, list(res)


class Context:
    """One gicp_ctx (one NanoGICP instance) on one HIP device."""

    def __init__(self, device: int = 0, params: GicpParams | None = None):
        self.L = load()
        h = C.c_void_p()
        self._check(self.L.gicp_ctx_create(device, C.byref(h)))
        self.h = h
        if params is not None:
            self.set_params(params)

    def _check(self, rc):
        if rc != 0:
            raise GicpError(rc, self.L.gicp_last_error().decode())
        return rc

    def close(self):
        if getattr(self, "h", None):
            self.L.gicp_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- params
    def set_params(self, p: GicpParams):
        self._check(self.L.gicp_set_params(self.h, C.byref(p)))

    def get_params(self) -> GicpParams:
        p = GicpParams()
        self._check(self.L.gicp_get_params(self.h, C.byref(p)))
        return p

    # ---- clouds
    def set_source(self, points, build_index=True):
        a, stride = _xyz(points)
        self._check(self.L.gicp_set_source(self.h, _ptr(a), len(a), stride, int(build_index)))

    def set_target(self, points):
        a, stride = _xyz(points)
        self._check(self.L.gicp_set_target(self.h, _ptr(a), len(a), stride))

    def clear_source(self):
        self._check(self.L.gicp_clear_source(self.h))

    def clear_target(self):
        self._check(self.L.gicp_clear_target(self.h))

    def size(self, side) -> int:
        n = C.c_size_t()
        self._check(self.L.gicp_get_size(self.h, side, C.byref(n)))
        return n.value

    def compute_covariances(self, side):
        self._check(self.L.gicp_compute_covariances(self.h, side))

    def set_covariances(self, side, cov):
        cov = np.ascontiguousarray(cov, np.float64)
        layout = COV_MAT4D if cov.shape[-1] == 16 or cov.shape[-2:] == (4, 4) else COV_SYM6
        n = cov.shape[0]
        self._check(self.L.gicp_set_covariances(self.h, side, _ptr(cov), n, layout))

    def get_covariances(self, side, layout=COV_SYM6):
        n = self.size(side)
        out = np.zeros((n, 16 if layout == COV_MAT4D else 6), np.float64)
        self._check(self.L.gicp_get_covariances(self.h, side, _ptr(out), n, layout))
        return out

    def has_covariances(self, side) -> bool:
        v = C.c_int()
        self._check(self.L.gicp_has_covariances(self.h, side, C.byref(v)))
        return bool(v.value)

    def swap_source_target(self):
        self._check(self.L.gicp_swap_source_target(self.h))

    def share_source_from(self, other: "Context"):
        self._check(self.L.gicp_share_source(self.h, other.h))

    # ---- registration
    def align(self, guess=None):
        # Per-context guess / pose / result buffers with their addresses taken
        # once: numpy's .ctypes accessors cost ~2-4 us per call, a few percent
        # of a cfg 3 align.  The caller gets copies.
        ab = self.__dict__.get("_abuf")
        if ab is None:
            gb, ob, rb = np.zeros((4, 4), np.float32), np.zeros((4, 4), np.float32), GicpResult()
            ab = self._abuf = (gb, ob, rb, gb.ctypes.data, ob.ctypes.data, C.pointer(rb))
        gb, ob, rb, gp, op, rp = ab
        if guess is not None:
            if type(guess) is np.ndarray and guess.shape == (4, 4):
                gb[...] = guess   # (~1.6 us less than reshape + copyto per call)
            else:
                np.copyto(gb, np.reshape(guess, (4, 4)), casting="unsafe")
        self._check(self.L.gicp_align(self.h, None if guess is None else gp, op, rp))
        return ob.copy(), GicpResult.from_buffer_copy(rb)

    def residuals(self):
        n = self.size(SOURCE)
        out = np.zeros(n, np.float64)
        self._check(self.L.gicp_get_residuals(self.h, _ptr(out), n))
        return out

    def residual_image(self, theta_min=-math.pi / 3, theta_max=math.pi / 3, width=512, height=512, with_xyz=False):
        """Residual image of the last linearization (odom.cc:804-827): (H, W)
        float32 residuals and, optionally, the (H, W, 3) winning points."""
        img = np.zeros((height, width), np.float32)
        xyz = np.zeros((height, width, 3), np.float32) if with_xyz else None
        self._check(self.L.gicp_residual_image(self.h, theta_min, theta_max, width, height, _ptr(img),
                                               None if xyz is None else _ptr(xyz)))
        return (img, xyz) if with_xyz else img

    def correspondences(self):
        n = self.size(SOURCE)
        corr = np.zeros(n, np.int32)
        sqd = np.zeros(n, np.float32)
        self._check(self.L.gicp_get_correspondences(self.h, _ptr(corr), _ptr(sqd), n))
        return corr, sqd

    def transform_source(self, out=None):
        n = self.size(SOURCE)
        if out is None:
            out = np.zeros((n, 3), np.float32)
        self._check(self.L.gicp_transform_source(self.h, _ptr(out), n, out.strides[0]))
        return out

    def linearize(self, pose):
        pose = np.ascontiguousarray(pose, np.float64)
        H = np.zeros((6, 6)); b = np.zeros(6); cost = C.c_double(); nc = C.c_int32()
        self._check(self.L.gicp_linearize(self.h, _ptr(pose), _ptr(H), _ptr(b), C.byref(cost), C.byref(nc)))
        return H, b, cost.value, nc.value

    def moments(self):
        out = np.zeros(80)
        self._check(self.L.gicp_get_moments(self.h, _ptr(out)))
        return out

    def knn_target(self, queries, k):
        q, stride = _xyz(queries)
        idx = np.zeros((len(q), k), np.int32)
        d = np.zeros((len(q), k), np.float32)
        self._check(self.L.gicp_knn_target(self.h, _ptr(q), len(q), stride, k, _ptr(idx), _ptr(d)))
        return idx, d

    def set_target_grid(self, mode=GRID_AUTO):
        """Candidate cells of the target (gicp_set_target_grid): GRID_OFF / GRID_AUTO / GRID_ON."""
        self._check(self.L.gicp_set_target_grid(self.h, int(mode)))

    def grid_info(self) -> dict:
        info = GicpGridInfo()
        self._check(self.L.gicp_get_target_grid_info(self.h, C.byref(info)))
        return info.as_dict()

    def lookup_walk_groups(self) -> int:
        """16-query sub-groups the last align left to the walk (summed over its iterations)."""
        v = C.c_int64(0)
        self._check(self.L.gicp_get_lookup_stats(self.h, C.byref(v)))
        return int(v.value)

    def set_tie_order(self, nanoflann_order=True):
        """Exact distance ties in nanoflann's traversal order (default) or by Morton position."""
        self._check(self.L.gicp_set_tie_order(self.h, 1 if nanoflann_order else 0))

    def nftree(self, side):
        """nanoflann's kd-tree of a side's cloud as built on the device: (vind, nodes (c1, c2, feat, parent),
        div (divlow, divhigh))."""
        nn = C.c_size_t(0)
        self._check(self.L.gicp_debug_nftree(self.h, side, None, None, None, 0, C.byref(nn)))
        n = self.size(side)
        vind = np.empty(n, np.int32)
        nodes = np.empty((nn.value, 4), np.int32)
        div = np.empty((nn.value, 2), np.float32)
        self._check(self.L.gicp_debug_nftree(self.h, side, _ptr(vind), _ptr(nodes), _ptr(div), nn.value, C.byref(nn)))
        return vind, nodes, div

    def nfbuild_debug(self, side, stop=-1, scratch_bytes=1 << 20):
        """A fresh device tree build stopped after `stop` big levels (development):
        (vind, info16, (err, nnodes), raw scratch bytes)."""
        n = self.size(side)
        vind = np.empty(n, np.int32)
        info = np.zeros(16, np.int64)
        st = np.zeros(2, np.int32)
        raw = np.zeros(scratch_bytes, np.uint8)
        self._check(self.L.gicp_debug_nfbuild(self.h, side, int(stop), _ptr(vind), _ptr(info), _ptr(st), _ptr(raw),
                                               raw.nbytes))
        return vind, info, st, raw

    def debug_stats(self, enable=True, read=False):
        """Per 64-query group search counters of the last linearize (development)."""
        if not read:
            self._check(self.L.gicp_debug_stats(self.h, int(enable), None, 0, None))
            return None
        n = self.size(SOURCE)  # upper bound on the number of query groups
        out = np.zeros((n, 8), np.uint32)
        nw = C.c_size_t()
        self._check(self.L.gicp_debug_stats(self.h, int(enable), _ptr(out), out.size, C.byref(nw)))
        return out

    def set_profiling(self, on=True):
        self._check(self.L.gicp_set_profiling(self.h, int(on)))

    def stage_times(self):
        """(covariance kernel, tree build, tie resolvers) device ms of the last profiled compute_covariances."""
        t = (C.c_double * 3)()
        self._check(self.L.gicp_get_stage_times(self.h, C.cast(t, C.c_void_p)))
        return float(t[0]), float(t[1]), float(t[2])

    def synchronize(self):
        self._check(self.L.gicp_synchronize(self.h))

    # ---- spatial sharding
    def set_shard(self, axis: int, lo: float = -np.inf, hi: float = np.inf):
        self._check(self.L.gicp_set_shard(self.h, int(axis), float(lo), float(hi)))

    def set_shard_groups(self, nparts: int, part: int):
        """Interleaved ownership: this ctx searches the 16-point groups = part (mod nparts)."""
        self._check(self.L.gicp_set_shard_groups(self.h, int(nparts), int(part)))

    def set_tie_target(self, points, local_index):
        """Slab shard, single process: the whole target its local target was cut from and each local
        point's index in it.  Exact ties resolve through the whole target's nanoflann tree restricted to
        the local points (the whole cloud is released before the call returns).  points=None removes it."""
        if points is None:
            self._check(self.L.gicp_set_tie_target(self.h, None, 0, 12, None, 0))
            return
        a, stride = _xyz(points)
        li = np.ascontiguousarray(local_index, np.int32)
        self._check(self.L.gicp_set_tie_target(self.h, _ptr(a), len(a), stride, _ptr(li), len(li)))

    def set_option(self, option: int, value: int):
        """gicp_set_option (OPT_TIE_ORDER, OPT_TIE_LAZY, OPT_TIE_PARTIAL_LEVELS, OPT_COV_TASKS)."""
        self._check(self.L.gicp_set_option(self.h, int(option), int(value)))

    def get_option(self, option: int) -> int:
        v = C.c_int(0)
        self._check(self.L.gicp_get_option(self.h, int(option), C.byref(v)))
        return int(v.value)

    def tie_order(self) -> bool:
        """True: exact ties in nanoflann's order (default); False: Morton order."""
        v = C.c_int(0)
        self._check(self.L.gicp_get_tie_order(self.h, C.byref(v)))
        return bool(v.value)

    def tie_builder_set(self, points):
        """Tie builder (one rank per submap): the whole submap and its nanoflann tree; None frees them."""
        if points is None:
            self._check(self.L.gicp_tie_builder_set(self.h, None, 0, 12))
            return
        a, stride = _xyz(points)
        self._check(self.L.gicp_tie_builder_set(self.h, _ptr(a), len(a), stride))

    def tie_builder_export(self, local_index) -> bytes:
        """The builder's tree restricted to the points local_index names (whole-cloud indices, one per
        local target point): the blob a slab rank installs with set_tie_tree."""
        li = np.ascontiguousarray(local_index, np.int32)
        p, n = C.c_void_p(), C.c_size_t(0)
        self._check(self.L.gicp_tie_builder_export(self.h, _ptr(li), len(li), C.byref(p), C.byref(n)))
        return C.string_at(p.value, n.value)

    def set_tie_tree(self, blob: bytes | None):
        """Slab shard: install the restriction of the whole submap's tree to this rank's target (None removes it)."""
        if not blob:
            self._check(self.L.gicp_set_tie_tree(self.h, None, 0))
            return
        self._check(self.L.gicp_set_tie_tree(self.h, blob, len(blob)))

    def set_tie_trees_from_root(self, root: int, blobs: list[bytes] | None):
        """Collective over this ctx's communicator: the root passes every rank's blob, the others None."""
        if blobs is None:
            self._check(self.L.gicp_set_tie_trees_from_root(self.h, int(root), None, None))
            return
        bufs = [C.create_string_buffer(b, len(b)) for b in blobs]
        ptrs = (C.c_void_p * len(bufs))(*[C.cast(b, C.c_void_p) for b in bufs])
        sizes = (C.c_size_t * len(bufs))(*[len(b) for b in blobs])
        self._check(self.L.gicp_set_tie_trees_from_root(self.h, int(root), ptrs, sizes))

    def device_bytes(self) -> dict:
        """Device bytes this ctx holds, by part (gicp_get_device_bytes)."""
        v = (C.c_int64 * 7)()
        self._check(self.L.gicp_get_device_bytes(self.h, v, 7))
        keys = ("total", "target", "source", "covariances", "tie_tree", "tie_builder", "scratch")
        return {k: int(x) for k, x in zip(keys, v)}

    def set_comm(self, unique_id: bytes | None, nranks: int, rank: int):
        buf = None
        if unique_id is not None:
            buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        self._check(self.L.gicp_set_comm(self.h, None if buf is None else C.cast(buf, C.c_void_p), 128,
                                         int(nranks), int(rank)))

    def comm_info(self):
        n, r, g = C.c_int(), C.c_int(), C.c_int()
        self._check(self.L.gicp_get_comm_info(self.h, C.byref(n), C.byref(r), C.byref(g)))
        return n.value, r.value, bool(g.value)

    def stream(self) -> int:
        s = C.c_void_p()
        self._check(self.L.gicp_get_stream(self.h, C.byref(s)))
        return s.value or 0


class NanoGICP:
    """Reference-shaped facade (method names of nano_gicp::NanoGICP + the PCL
    Registration calls OdomNode makes, odom.cc:92-112,518-532,745-851)."""

    def __init__(self, device=0):
        self.ctx = Context(device)
        self.params = self.ctx.get_params()
        self._src_id = None
        self._tgt_id = None
        self._final = np.eye(4, dtype=np.float32)
        self._converged = False
        self.last_result = None

    def _push(self):
        self.ctx.set_params(self.params)

    # PCL Registration setters used by OdomNode
    def setMaximumIterations(self, n): self.params.max_iterations = int(n); self._push()
    def setTransformationEpsilon(self, e): self.params.transformation_epsilon = float(e); self._push()
    def setMaxCorrespondenceDistance(self, d): self.params.max_correspondence_distance = float(d); self._push()
    def setEuclideanFitnessEpsilon(self, e): pass          # no-op for NanoGICP
    def setRANSACIterations(self, n): pass                 # no-op
    def setRANSACOutlierRejectionThreshold(self, t): pass  # no-op
    def setSearchMethodSource(self, *a): pass              # no-op (force_no_recompute)
    def setSearchMethodTarget(self, *a): pass
    def setNumThreads(self, n): pass                       # CPU-only knob
    # NanoGICP / LsqRegistration setters
    def setCorrespondenceRandomness(self, k): self.params.k_correspondences = int(k); self._push()
    def setRegularizationMethod(self, m): self.params.regularization = int(m); self._push()
    def setRotationEpsilon(self, e): self.params.rotation_epsilon = float(e); self._push()
    def setInitialLambdaFactor(self, f): self.params.lm_init_lambda_factor = float(f); self._push()

    def setInputSource(self, cloud):
        if self._src_id is not None and self._src_id == id(cloud):   # pointer identity (:135)
            return
        self.ctx.set_source(cloud, True)
        self._src_id = id(cloud)

    def registerInputSource(self, cloud):
        if self._src_id is not None and self._src_id == id(cloud):
            return
        self.ctx.set_source(cloud, False)
        self._src_id = id(cloud)

    def setInputTarget(self, cloud):
        if self._tgt_id is not None and self._tgt_id == id(cloud):
            return
        self.ctx.set_target(cloud)
        self._tgt_id = id(cloud)

    def setSourceCovariances(self, covs): self.ctx.set_covariances(SOURCE, covs)
    def setTargetCovariances(self, covs): self.ctx.set_covariances(TARGET, covs)
    def calculateSourceCovariances(self): self.ctx.compute_covariances(SOURCE); return True
    def calculateTargetCovariances(self): self.ctx.compute_covariances(TARGET); return True
    def getSourceCovariances(self): return self.ctx.get_covariances(SOURCE, COV_MAT4D).reshape(-1, 4, 4)
    def getTargetCovariances(self): return self.ctx.get_covariances(TARGET, COV_MAT4D).reshape(-1, 4, 4)

    def swapSourceAndTarget(self):
        self.ctx.swap_source_target()
        self._src_id, self._tgt_id = self._tgt_id, self._src_id

    def clearSource(self): self.ctx.clear_source(); self._src_id = None
    def clearTarget(self): self.ctx.clear_target(); self._tgt_id = None

    def shareSourceFrom(self, other: "NanoGICP"):
        """odom.cc:530 + :765 (source_kdtree_ alias + source_covs_ copy)."""
        self.ctx.share_source_from(other.ctx)
        self._src_id = other._src_id

    def align(self, guess=None):
        out, res = self.ctx.align(guess)
        self._final = out
        self._converged = bool(res.converged)
        self.last_result = res
        return self.ctx.transform_source()

    def getFinalTransformation(self): return self._final.copy()
    def hasConverged(self): return self._converged
    def getFinalHessian(self): return np.array(self.last_result.final_hessian).reshape(6, 6)
    def getResiduals(self, trans=None): return self.ctx.residuals()
