"""Generate the committed golden fixtures under tests/golden/ (run in the dev
container, where /root/reference exists; the GPU box only reads the .npz).

  knn_ref.npz     exact kNN from the REFERENCE's own nanoflann
                  (nano_gicp/impl/nanoflann_impl.hpp compiled from
                  /root/reference by oracle/Makefile into oracle/_ref/):
                  k = 1 / 10 / 20 on a ray-cast scan, far queries, a
                  duplicate-point cloud and an integer lattice (exact ties).
  gicp_s2s.npz    oracle (oracle/cpu_ref.cpp) results on a 16x512 S2S pair:
                  covariances (k=10 PLANE, and the other 4 regularizations),
                  one linearization at the identity, LM align + per-iteration
                  trace, GN fixed-10 align.  The GICP half cannot be built
                  from the reference (needs Eigen/PCL): these are oracle
                  regression vectors, cross-checked in tests/test_oracle.py
                  against an independent numpy implementation ("parity
                  unpinned" for the reference's GICP arithmetic).
  gicp_s2m.npz    oracle S2M problem: 16x512 scan -> 12,000-pt submap of 3
                  keyframes (per-keyframe k=10 covariances, subset), LM align.

usage: make oracle && python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from dynamic_direct_lidar_odometry_amd import scene  # noqa: E402
from oracle import oracle as O  # noqa: E402


def knn_fixture():
    assert O.ref_lib() is not None, "oracle/_ref/libref_nanoflann.so missing: build it with `make oracle` here"
    out = {}
    src, tgt, T = scene.s2s_pair(16, 512, 1)
    q = scene.transform(src, T)
    out["scan_pts"] = tgt
    out["scan_q"] = q
    for k in (1, 10, 20):
        qq = q if k == 1 else q[::4]
        i, d = O.ref_knn(tgt, qq, k)
        out[f"scan_k{k}_idx"], out[f"scan_k{k}_sqd"] = i, d
    # self queries (covariance neighbourhoods: the point itself is returned)
    i, d = O.ref_knn(tgt[:2048], tgt[:2048], 10)
    out["self_k10_idx"], out["self_k10_sqd"] = i, d
    # far queries (outside the cloud's bounding box)
    rng = np.random.default_rng(7)
    far = (rng.standard_normal((256, 3)) * 200.0).astype(np.float32)
    i, d = O.ref_knn(tgt, far, 10)
    out["far_q"], out["far_k10_idx"], out["far_k10_sqd"] = far, i, d
    # duplicate points: every point appears twice (exact distance ties)
    base = tgt[::8]
    dup = np.concatenate([base, base[::-1]]).astype(np.float32)
    qd = scene.transform(base[::3], T)
    i, d = O.ref_knn(dup, qd, 10)
    out["dup_pts"], out["dup_q"], out["dup_k10_idx"], out["dup_k10_sqd"] = dup, qd, i, d
    # integer lattice, queries on lattice points and cell centres (many ties)
    g = np.arange(12, dtype=np.float32)
    lat = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    lat = lat[rng.permutation(len(lat))].astype(np.float32)
    ql = np.concatenate([lat[:200], lat[200:400] + 0.5]).astype(np.float32)
    for k in (1, 10):
        i, d = O.ref_knn(lat, ql, k)
        out[f"lat_k{k}_idx"], out[f"lat_k{k}_sqd"] = i, d
    out["lat_pts"], out["lat_q"] = lat, ql
    np.savez_compressed(os.path.join(HERE, "knn_ref.npz"), **out)


def s2s_fixture():
    src, tgt, T = scene.s2s_pair(16, 512, 1)
    p = O.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32,
                         transformation_epsilon=5e-4)
    out = {"src": src, "tgt": tgt, "T_true": T}
    for name, reg in O.REG.items():
        out[f"cov_src_{name}"] = O.covariances(src, 10, reg)
    out["cov_tgt"] = O.covariances(tgt, 10, "PLANE")
    g = O.Gicp(src, tgt, p)
    g.set_covariances(0, out["cov_src_PLANE"])
    g.set_covariances(1, out["cov_tgt"])
    H, b, cost, corr, sqd = g.linearize(np.eye(4))
    out.update(lin_H=H, lin_b=b, lin_cost=np.float64(cost), lin_corr=corr, lin_sqd=sqd)
    pose, res = g.align()
    out.update(lm_pose=pose, lm_iters=np.int32(res.iterations_run), lm_nr=np.int32(res.nr_iterations),
               lm_converged=np.int32(res.converged), lm_trials=np.int32(res.lm_trials),
               lm_cost=np.float64(res.final_cost), lm_hessian=np.array(res.final_hessian).reshape(6, 6),
               lm_trace=g.trace())
    corr2, sqd2 = g.last_correspondences()
    out.update(lm_last_corr=corr2, lm_last_sqd=sqd2)
    gn = O.Gicp(src, tgt, O.default_params(k_correspondences=10, max_correspondence_distance=1.0,
                                           max_iterations=10, optimizer=O.GN, fixed_iterations=10))
    gn.set_covariances(0, out["cov_src_PLANE"])
    gn.set_covariances(1, out["cov_tgt"])
    pose, res = gn.align()
    out.update(gn_pose=pose, gn_iters=np.int32(res.iterations_run), gn_trace=gn.trace())
    np.savez_compressed(os.path.join(HERE, "gicp_s2s.npz"), **out)


def s2m_fixture():
    prob = scene.s2m_problem(16, 512, 3, 12000, 7)
    sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
    kcov = np.concatenate([O.covariances(k, 10) for k in prob["keyframes"]])[prob["subset"]]
    scov = O.covariances(prob["source"], 10)
    p = O.default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32,
                         transformation_epsilon=0.01)
    g = O.Gicp(prob["source"], sub, p)
    g.set_covariances(0, scov)
    g.set_covariances(1, kcov)
    pose, res = g.align(prob["guess"].astype(np.float32))
    np.savez_compressed(os.path.join(HERE, "gicp_s2m.npz"), src=prob["source"], sub=sub, cov_src=scov, cov_sub=kcov,
                        guess=prob["guess"].astype(np.float32), T_true=prob["T_true"], pose=pose,
                        iters=np.int32(res.iterations_run), converged=np.int32(res.converged),
                        cost=np.float64(res.final_cost), trace=g.trace())


if __name__ == "__main__":
    knn_fixture()
    s2s_fixture()
    s2m_fixture()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
