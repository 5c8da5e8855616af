"""CPU restatement of OdomNode's registration pipeline — TEST INFRASTRUCTURE ONLY.

The oracle for the GPU odometry driver (include/ddlo_odom.h).  It follows
reference dynamic_direct_lidar_odometry/src/odometry/odom.cc step for step
(line numbers below) on top of the oracle GICP (oracle/cpu_ref.cpp via
oracle.Gicp), the PCL VoxelGrid / CropBox restatements (oracle.voxel_grid,
oracle.crop_box_negative) and scipy's qhull (the library pcl::ConvexHull
wraps) for the convex keyframe hull.  Only tests/ import it.

Parity status: the GICP, filters and keyframe/submap logic follow the
reference; PCL itself is absent from the image, so the hull steps are
"parity unpinned".  Both use qhull through scipy, the library pcl::ConvexHull
and pcl::ConcaveHull wrap, with the dimension OdomNode sets (3, odom.cc:87-88)
and PCL 1.10's options: the convex hull is qhull's 3-D vertex set (a flat set
is qhull's "initial simplex is flat" error, i.e. an empty hull); the concave
hull is the alpha shape PCL extracts from qhull's "d QJ" 3-D Delaunay
(concave_hull.hpp performReconstruction, dim 3).
"""
from __future__ import annotations

import math

import numpy as np
from scipy.spatial import ConvexHull, Delaunay
from scipy.spatial import QhullError

from . import oracle as O

F = np.float32


def mat4_mul(A, B):
    """float Matrix4f product, ((a0 b0 + a1 b1) + a2 b2) + a3 b3 per entry (as odom.hip)."""
    A = A.astype(F)
    B = B.astype(F)
    R = np.zeros((4, 4), F)
    for r in range(4):
        for c in range(4):
            R[r, c] = ((A[r, 0] * B[0, c] + A[r, 1] * B[1, c]) + A[r, 2] * B[2, c]) + A[r, 3] * B[3, c]
    return R


def transform(points, T):
    """pcl::transformPointCloud in float: (c0 x + c1 y) + (c2 z + c3)."""
    p = points.astype(F)
    T = T.astype(F)
    out = np.empty_like(p)
    for r in range(3):
        out[:, r] = (T[r, 0] * p[:, 0] + T[r, 1] * p[:, 1]) + (T[r, 2] * p[:, 2] + T[r, 3])
    return out


def quat_from_R(T):
    """Eigen::Quaternionf(Matrix3f) + propagateS2M's normalisation (odom.cc:928-937); (x, y, z, w)."""
    m = T[:3, :3].astype(F)
    t = F(m[0, 0] + m[1, 1] + m[2, 2])
    q = [F(0)] * 4
    if t > 0:
        t = F(np.sqrt(F(t + F(1.0))))
        w = F(F(0.5) * t)
        t = F(F(0.5) / t)
        q = [F((m[2, 1] - m[1, 2]) * t), F((m[0, 2] - m[2, 0]) * t), F((m[1, 0] - m[0, 1]) * t), w]
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = F(np.sqrt(F(F(m[i, i] - m[j, j]) - m[k, k]) + F(1.0)))
        c = [F(0)] * 3
        c[i] = F(F(0.5) * t)
        t = F(F(0.5) / t)
        w = F((m[k, j] - m[j, k]) * t)
        c[j] = F((m[j, i] + m[i, j]) * t)
        c[k] = F((m[k, i] + m[i, k]) * t)
        q = [c[0], c[1], c[2], w]
    x, y, z, w = q
    norm = math.sqrt(float(F(F(F(w * w) + F(x * x)) + F(y * y)) + F(z * z)))
    return [F(x / norm), F(y / norm), F(z / norm), F(w / norm)]


def quat_mul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return [F(aw * bx + ax * bw + ay * bz - az * by), F(aw * by + ay * bw + az * bx - ax * bz),
            F(aw * bz + az * bw + ax * by - ay * bx), F(aw * bw - ax * bx - ay * by - az * bz)]


def quat_inverse(q):
    x, y, z, w = q
    n2 = F(w * w + x * x + y * y + z * z)
    return [F(-x / n2), F(-y / n2), F(-z / n2), F(w / n2)]


def convex_hull(P):
    """computeConvexHull (odom.cc:993-1028) with setDimension(3): qhull's 3-D vertex set, [] when qhull fails
    (fewer than 4 points or a flat set)."""
    if len(P) < 4:
        return []
    try:
        h = ConvexHull(np.asarray(P, np.float64))
    except QhullError:
        return []
    return sorted(int(i) for i in h.vertices)


def _tri_radius(a, b, c):
    """pcl::getCircumcircleRadius: float Vector4f norms ((x^2 + z^2) + y^2, Eigen's SSE redux), Heron in double."""
    def nrm(u, v):
        d = (v - u).astype(F)
        return float(np.sqrt(F(F(d[0] * d[0] + d[2] * d[2]) + d[1] * d[1])))
    p2p1, p3p2, p1p3 = nrm(a, b), nrm(b, c), nrm(c, a)
    s = (p2p1 + p3p2 + p1p3) / 2.0
    with np.errstate(invalid="ignore", divide="ignore"):
        area = math.sqrt(s * (s - p2p1) * (s - p3p2) * (s - p1p3)) if s * (s - p2p1) * (s - p3p2) * (s - p1p3) >= 0 else float("nan")
        return (p2p1 * p3p2 * p1p3) / (4.0 * area) if area > 0 else float("inf")


def _tet_radius(V):
    A = V[1:] - V[0]
    rhs = 0.5 * (A * A).sum(axis=1)
    try:
        x = np.linalg.solve(A, rhs)
    except np.linalg.LinAlgError:
        return float("inf")
    return float(np.sqrt((x * x).sum()))


def concave_hull(P, alpha):
    """computeConcaveHull (odom.cc:1030-1065): pcl::ConcaveHull, dimension 3, alpha = keyframe_thresh_dist_.
    qhull "d QJ" Delaunay of the demeaned points; a tetrahedron is good iff its circumradius <= alpha; a
    triangle is kept iff one side is not a good tetrahedron (outside or bad) and it has circumradius <= alpha
    (a good tetrahedron's triangles always do); the hull = the kept triangles' vertices."""
    P = np.asarray(P, np.float64)
    if len(P) < 4:
        return []
    D = P - P.mean(axis=0)
    try:
        tri = Delaunay(D, qhull_options="QJ")
    except QhullError:
        return []
    S = tri.simplices
    good = np.array([_tet_radius(D[s]) <= alpha for s in S])
    on = np.zeros(len(P), bool)
    for t, s in enumerate(S):
        for j in range(4):
            nb = tri.neighbors[t, j]
            if nb >= 0 and nb < t:
                continue   # each triangle once
            gb = nb >= 0 and good[nb]
            if good[t] and gb:
                continue
            f = np.delete(s, j)
            if good[t] or gb or _tri_radius(D[f[0]], D[f[1]], D[f[2]]) <= alpha:
                on[f] = True
    return [int(i) for i in np.nonzero(on)[0]]


def push_submap_indices(dists, k, frames, out):
    """OdomNode::pushSubmapIndices (odom.cc:1180-1213)."""
    if len(dists) == 0:
        return
    kth = sorted(dists)[min(k, len(dists)) - 1]
    for d, f in zip(dists, frames):
        if d <= kth:
            out.append(f)


class OdomRef:
    """OdomNode (registration part) on the CPU oracle."""

    def __init__(self, params, threads=0):
        self.p = params
        self.s2s = O.as_params(params.s2s)
        self.s2m = O.as_params(params.s2m)
        self.threads = threads
        self.target = None          # S2S target cloud and its covariances
        self.target_cov = None
        self.T = np.eye(4, dtype=F)
        self.T_s2s = np.eye(4, dtype=F)
        self.T_s2s_prev = np.eye(4, dtype=F)
        self.pose = np.zeros(3, F)
        self.rotq = [F(0), F(0), F(0), F(1)]
        self.keyframes = []         # (pose, q, points, cov)
        self.submap_prev = []
        self.keyframe_convex = []
        self.keyframe_concave = []
        self.median_prev = None
        self.initialized = False    # ddlo_initialized_
        self.thresh = float(params.keyframe_thresh_dist)
        self.submap = None
        # on_align(kind, inputs, T, result): called after each of the two aligns of a frame with the exact
        # inputs the oracle aligned ("s2s": source, target, target_cov, guess; "s2m": source, source_cov,
        # target, target_cov, guess), so a test can run the GPU on identical inputs
        self.on_align = None

    def _preprocess(self, pts):
        a = pts.astype(F)
        if self.p.crop_use:
            a = O.crop_box_negative(a, self.p.crop_size)
        if self.p.vf_scan_use:
            a = O.voxel_grid(a, self.p.vf_scan_res)
        return a

    def _keyframe(self, scan):
        kf = transform(scan, self.T)
        if self.p.vf_submap_use:
            kf = O.voxel_grid(kf, self.p.vf_submap_res)
        cov = O.covariances(kf, min(self.s2s.k_correspondences, len(kf)), threads=self.threads)
        self.keyframes.append((self.pose.copy(), list(self.rotq), kf, cov))

    def process(self, pts):
        out = {"status": 0, "keyframe_added": 0, "submap_changed": 0}
        if len(pts) < self.p.min_num_points:
            out["status"] = 2
            return out
        if not self.initialized:    # initializeDDLO consumes the first valid scan (odom.cc:641-646)
            self.initialized = True
            if getattr(self.p, "skip_first_scan", 1):
                out["status"] = 3
                return out
        scan = self._preprocess(pts)
        out["scan_points"] = len(scan)
        # computeSpaciousness (odom.cc:981-1001)
        d = np.sqrt((scan.astype(np.float64) ** 2).sum(axis=1)).astype(F)
        med = F(np.sort(d)[len(d) // 2])
        if self.median_prev is None:
            self.median_prev = med
        lpf = F(0.95 * float(self.median_prev) + 0.05 * float(med))
        self.median_prev = lpf
        out["spaciousness"] = float(lpf)
        if self.p.adaptive:  # setAdaptiveParams (odom.cc:1156-1178)
            if lpf > 20.0:
                self.thresh = 10.0
            elif 10.0 < lpf <= 20.0:
                self.thresh = 5.0
            elif 5.0 < lpf <= 10.0:
                self.thresh = 1.0
            elif lpf <= 5.0:
                self.thresh = 0.5
        if self.target is None:  # initializeInputTarget (odom.cc:480-516)
            self.target = scan
            self.target_cov = O.covariances(scan, self.s2s.k_correspondences, threads=self.threads)
            self._keyframe(scan)
            out["status"] = 1
            out["keyframe_added"] = 1
            return out
        # scanMatching (odom.cc:745-851)
        g = O.Gicp(scan, self.target, self.s2s, threads=self.threads)
        g.set_covariances(1, self.target_cov)
        T_S2S, r1 = g.align()
        src_cov = g.get_covariances(0)
        if self.on_align is not None:
            self.on_align("s2s", dict(source=scan, target=self.target, target_cov=self.target_cov, guess=None),
                          T_S2S, r1)
        self.T_s2s = mat4_mul(self.T_s2s_prev, T_S2S)
        self.T_s2s_prev = self.T_s2s.copy()
        self.target, self.target_cov = scan, src_cov        # swapSourceAndTarget
        changed = self._submap_keyframes()
        g2 = O.Gicp(scan, self.submap[0], self.s2m, threads=self.threads)
        g2.set_covariances(0, src_cov)
        g2.set_covariances(1, self.submap[1])
        self.T, r2 = g2.align(self.T_s2s)
        if self.on_align is not None:
            self.on_align("s2m", dict(source=scan, source_cov=src_cov, target=self.submap[0],
                                      target_cov=self.submap[1], guess=self.T_s2s.copy()), self.T, r2)
        self.T = self.T.astype(F)
        self.T_s2s_prev = self.T.copy()
        self.pose = self.T[:3, 3].copy()
        self.rotq = quat_from_R(self.T)
        # updateKeyframes (odom.cc:1067-1154)
        closest_d, closest, num_nearby = np.inf, 0, 0
        for i, k in enumerate(self.keyframes):
            dd = F(math.sqrt(sum((float(self.pose[a]) - float(k[0][a])) ** 2 for a in range(3))))
            if dd <= self.thresh * 1.5:
                num_nearby += 1
            if dd < closest_d:
                closest_d, closest = dd, i
        ck = self.keyframes[closest]
        dd = F(math.sqrt(sum((float(self.pose[a]) - float(ck[0][a])) ** 2 for a in range(3))))
        dq = quat_mul(self.rotq, quat_inverse(ck[1]))
        theta_rad = F(2.0 * math.atan2(math.sqrt(float(dq[0]) ** 2 + float(dq[1]) ** 2 + float(dq[2]) ** 2), float(dq[3])))
        theta_deg = F(float(theta_rad) * (180.0 / math.pi))
        add = False
        if abs(dd) > self.thresh or abs(theta_deg) > self.p.keyframe_thresh_rot:
            add = True
        if abs(dd) <= self.thresh:
            add = False
        if abs(dd) <= self.thresh and abs(theta_deg) > self.p.keyframe_thresh_rot and num_nearby <= 1:
            add = True
        if add:
            self._keyframe(scan)
            out["keyframe_added"] = 1
        out.update(T=self.T.copy(), T_s2s=self.T_s2s.copy(), T_s2s_local=T_S2S, s2s=r1, s2m=r2,
                   submap_changed=int(changed), num_keyframes=len(self.keyframes), submap=list(self.submap_prev),
                   keyframe_thresh_dist=self.thresh)
        return out

    def _submap_keyframes(self):
        """getSubmapKeyframes (odom.cc:1215-1315)."""
        nk = len(self.keyframes)
        c = self.T_s2s[:3, 3]
        ds = [F(math.sqrt(sum((float(c[a]) - float(k[0][a])) ** 2 for a in range(3)))) for k in self.keyframes]
        cur = []
        push_submap_indices(ds, self.p.submap_knn, list(range(nk)), cur)
        P = np.array([k[0] for k in self.keyframes], F)
        if nk >= 4:
            self.keyframe_convex = convex_hull(P)
        push_submap_indices([ds[i] for i in self.keyframe_convex], self.p.submap_kcv, self.keyframe_convex, cur)
        if nk >= 5:
            self.keyframe_concave = concave_hull(P, self.thresh)
        push_submap_indices([ds[i] for i in self.keyframe_concave], self.p.submap_kcc, self.keyframe_concave, cur)
        cur = sorted(set(cur))
        changed = cur != self.submap_prev
        if changed:
            self.submap = (np.concatenate([self.keyframes[k][2] for k in cur]),
                           np.concatenate([self.keyframes[k][3] for k in cur]))
            self.submap_prev = cur
        return changed
