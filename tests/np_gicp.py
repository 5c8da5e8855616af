"""Independent numpy/scipy restatement of NanoGICP — TEST HELPER ONLY.

Cross-checks the C++ oracle (oracle/cpu_ref.cpp) with different code:
scipy's cKDTree for neighbours, np.linalg.svd / inv / solve for the algebra.
It follows the reference directly:
  covariances      nano_gicp_impl.hpp:385-438 (k-NN incl. self, biased /k,
                   regularization via JacobiSVD :405-436)
  correspondences  nano_gicp_impl.hpp:234-275 (fp32 query transform, fp32
                   nanoflann distance, (double)d < thr^2, M = (C_B+R C_A R^T)^-1)
  linearize        nano_gicp_impl.hpp:277-336 (J = [skew(Ta) | -I])
  compute_error    nano_gicp_impl.hpp:339-383
  LM / GN / conv.  lsq_registration_impl.hpp:95-232
  so3_exp          gicp/so3.hpp:50-124 (Sophus)
"""
from __future__ import annotations

import numpy as np
from scipy.spatial import cKDTree

REG = {"NONE": 0, "MIN_EIG": 1, "NORMALIZED_MIN_EIG": 2, "PLANE": 3, "FROBENIUS": 4}


def nanoflann_sqd(q, p):
    """fp32 ((dx^2 + dy^2) + dz^2), nanoflann L2_Simple_Adaptor (nanoflann_impl.hpp:570-592)."""
    q = q.astype(np.float32)
    p = p.astype(np.float32)
    d = q - p
    return (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]


def regularize(C, reg):
    reg = REG[reg] if isinstance(reg, str) else reg
    if reg == 0:
        return C.copy()
    if reg == 4:  # FROBENIUS (:405-412)
        Ci = np.linalg.inv(C + 1e-3 * np.eye(3))
        return np.linalg.inv(Ci / np.linalg.norm(Ci))
    U, s, Vt = np.linalg.svd(C)
    if reg == 3:
        vals = np.array([1.0, 1.0, 1e-3])
    elif reg == 1:
        vals = np.maximum(s, 1e-3)
    else:
        vals = np.maximum(s / s[0], 1e-3)
    return U @ np.diag(vals) @ Vt


def covariances(points, k, reg="PLANE"):
    """Returns (cov (n,3,3), neighbour index (n,k))."""
    pts = np.asarray(points, np.float32)
    _, idx = cKDTree(pts.astype(np.float64)).query(pts.astype(np.float64), k)
    idx = np.asarray(idx).reshape(len(pts), k)
    nb = pts[idx].astype(np.float64)                    # (n,k,3)
    mean = nb.mean(axis=1, keepdims=True)
    X = nb - mean
    C = np.einsum("nki,nkj->nij", X, X) / k
    return np.stack([regularize(c, reg) for c in C]), idx


def sym6_to_mat(c6):
    """(n,6) xx,xy,xz,yy,yz,zz -> (n,3,3)."""
    c6 = np.asarray(c6, np.float64)
    m = np.empty((len(c6), 3, 3))
    m[:, 0, 0], m[:, 0, 1], m[:, 0, 2] = c6[:, 0], c6[:, 1], c6[:, 2]
    m[:, 1, 0], m[:, 1, 1], m[:, 1, 2] = c6[:, 1], c6[:, 3], c6[:, 4]
    m[:, 2, 0], m[:, 2, 1], m[:, 2, 2] = c6[:, 2], c6[:, 4], c6[:, 5]
    return m


def mat_to_sym6(m):
    return np.stack([m[:, 0, 0], m[:, 0, 1], m[:, 0, 2], m[:, 1, 1], m[:, 1, 2], m[:, 2, 2]], axis=1)


def transform_f32(pose, pts):
    """trans_f * a in fp32 with the reference's operation order (r0 x + r1 y) + (r2 z + t)."""
    T = np.asarray(pose, np.float64).astype(np.float32)
    p = np.asarray(pts, np.float32)
    out = np.empty_like(p)
    for r in range(3):
        out[:, r] = (T[r, 0] * p[:, 0] + T[r, 1] * p[:, 1]) + (T[r, 2] * p[:, 2] + T[r, 3])
    return out


def skew(v):
    z = np.zeros(len(v))
    return np.stack([np.stack([z, -v[:, 2], v[:, 1]], -1),
                     np.stack([v[:, 2], z, -v[:, 0]], -1),
                     np.stack([-v[:, 1], v[:, 0], z], -1)], 1)


def so3_exp(w):
    """Sophus SO3::exp (so3.hpp:50-124) as a rotation matrix."""
    w = np.asarray(w, np.float64)
    th2 = float(w @ w)
    if th2 < 1e-10:
        imag = 0.5 - th2 / 48.0 + th2 * th2 / 3840.0
        real = 1.0 - th2 / 8.0 + th2 * th2 / 384.0
    else:
        th = np.sqrt(th2)
        imag = np.sin(0.5 * th) / th
        real = np.cos(0.5 * th)
    x, y, z = imag * w
    w_ = real
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w_), 2 * (x * z + y * w_)],
                     [2 * (x * y + z * w_), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w_)],
                     [2 * (x * z - y * w_), 2 * (y * z + x * w_), 1 - 2 * (x * x + y * y)]])


class Problem:
    """One NanoGICP source/target pair with fixed covariances ((n,3,3) float64)."""

    def __init__(self, src, tgt, cov_src, cov_tgt, max_corr=np.finfo(np.float32).max):
        self.src = np.asarray(src, np.float32)
        self.tgt = np.asarray(tgt, np.float32)
        self.ca = cov_src
        self.cb = cov_tgt
        self.tree = cKDTree(self.tgt.astype(np.float64))
        self.thr2 = float(max_corr) ** 2
        self.corr = None

    def update_correspondences(self, pose):
        q = transform_f32(pose, self.src)
        _, j = self.tree.query(q.astype(np.float64), 1)
        sqd = nanoflann_sqd(q, self.tgt[j])
        corr = np.where(sqd.astype(np.float64) < self.thr2, j, -1)
        R = np.asarray(pose, np.float64)[:3, :3]
        ok = corr >= 0
        M = np.zeros((len(q), 3, 3))
        RCR = self.cb[corr[ok]] + R @ self.ca[ok] @ R.T
        M[ok] = np.linalg.inv(RCR)
        self.corr, self.sqd, self.M = corr, sqd, M
        return corr, sqd

    def _errors(self, pose):
        ok = self.corr >= 0
        T = np.asarray(pose, np.float64)
        a = self.src[ok].astype(np.float64)
        ta = a @ T[:3, :3].T + T[:3, 3]
        e = self.tgt[self.corr[ok]].astype(np.float64) - ta
        return ok, ta, e

    def linearize(self, pose):
        self.update_correspondences(pose)
        ok, ta, e = self._errors(pose)
        M = self.M[ok]
        J = np.concatenate([skew(ta), -np.broadcast_to(np.eye(3), (len(ta), 3, 3))], axis=2)  # (n,3,6)
        MJ = M @ J
        H = np.einsum("nki,nkj->ij", J, MJ)
        b = np.einsum("nki,nk->i", MJ, e)
        cost = float(np.einsum("ni,nij,nj->", e, M, e))
        return H, b, cost

    def compute_error(self, pose):
        ok, _, e = self._errors(pose)
        return float(np.einsum("ni,nij,nj->", e, self.M[ok], e))


def _delta(d):
    D = np.eye(4)
    D[:3, :3] = so3_exp(d[:3])
    D[:3, 3] = d[3:]
    return D


def is_converged(D, trans_eps, rot_eps):
    return max(np.abs(D[:3, :3] - np.eye(3)).max() / rot_eps, np.abs(D[:3, 3]).max() / trans_eps) < 1


def align(prob: Problem, guess=None, max_iterations=64, trans_eps=5e-4, rot_eps=2e-3, lm=True,
          lm_max_iterations=10, lm_factor=1e-9, fixed_iterations=0):
    """LsqRegistration::computeTransformation; returns (pose, iterations_run, converged, lm_failed)."""
    x = np.eye(4) if guess is None else np.asarray(guess, np.float32).astype(np.float64)
    lam = -1.0
    converged = False
    it_run = 0
    lm_failed = False
    for _ in range(max_iterations):
        if converged and not fixed_iterations:
            break
        it_run += 1
        H, b, y0 = prob.linearize(x)
        if not lm:
            d = np.linalg.solve(H, -b)
            D = _delta(d)
            x = D @ x
        else:
            if lam < 0:
                lam = lm_factor * np.abs(np.diag(H)).max()
            nu = 2.0
            ok = False
            for _t in range(lm_max_iterations):
                d = np.linalg.solve(H + lam * np.eye(6), -b)
                D = _delta(d)
                xi = D @ x
                yi = prob.compute_error(xi)
                rho = (y0 - yi) / (d @ (lam * d - b))
                if rho < 0:
                    if is_converged(D, trans_eps, rot_eps):
                        ok = True
                        break
                    lam *= nu
                    nu *= 2
                    continue
                x = xi
                lam *= max(1.0 / 3.0, 1 - (2 * rho - 1) ** 3)
                ok = True
                break
            if not ok:
                lm_failed = True
                break
        converged = is_converged(D, trans_eps, rot_eps)
    return x, it_run, converged, lm_failed
