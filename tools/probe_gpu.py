"""Developer probe: every stage of the HIP path vs the oracle, with timings.

Run on the GPU box:  python tools/probe_gpu.py [--big]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic_direct_lidar_odometry_amd import scene, Context, default_params, SOURCE, TARGET  # noqa: E402
from oracle import oracle as O  # noqa: E402


def rot_err(A, B):
    R = A[:3, :3].astype(np.float64).T @ B[:3, :3].astype(np.float64)
    c = np.clip((np.trace(R) - 1) / 2, -1, 1)
    return float(np.arccos(c))


def main():
    big = "--big" in sys.argv
    rows, cols = (64, 2048) if big else (64, 1024)
    src, tgt, T = scene.s2s_pair(rows, cols, 1)
    print(f"S2S pair {rows}x{cols}: src {len(src)} tgt {len(tgt)}", flush=True)
    ctx = Context(0)
    p = default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32,
                       transformation_epsilon=5e-4)
    ctx.set_params(p)
    t0 = time.time(); ctx.set_target(tgt); t1 = time.time()
    print(f"set_target {1e3*(t1-t0):.2f} ms", flush=True)
    # kNN parity
    q = scene.transform(src, T)
    for k in (1, 10):
        gi, gd = ctx.knn_target(q, k)
        oi, od = O.knn(tgt, q, k)
        print(f"knn k={k}: idx equal {np.mean(gi == oi):.6f} dist equal {np.mean(gd == od):.6f} "
              f"max|dd| {np.abs(gd - od).max():.3g}", flush=True)
    # covariances
    ctx.set_source(src)
    t0 = time.time(); ctx.compute_covariances(SOURCE); ctx.compute_covariances(TARGET); t1 = time.time()
    print(f"covariances (2 clouds) {1e3*(t1-t0):.2f} ms", flush=True)
    gc = ctx.get_covariances(SOURCE)
    oc = O.covariances(src, 10)
    print(f"cov max abs diff {np.abs(gc - oc).max():.3g}", flush=True)
    # linearize parity with identical covariances
    g = O.Gicp(src, tgt, p)
    g.set_covariances(0, oc)
    g.set_covariances(1, O.covariances(tgt, 10))
    ctx.set_covariances(SOURCE, oc)
    ctx.set_covariances(TARGET, O.covariances(tgt, 10))
    pose = np.eye(4)
    H, b, cost, nc = ctx.linearize(pose)
    Ho, bo, costo, corro, sqdo = g.linearize(pose)
    gcorr, gsqd = ctx.correspondences()
    print(f"linearize: nc {nc} vs {np.sum(corro >= 0)}; corr equal {np.mean(gcorr == corro):.6f}; "
          f"cost rel {abs(cost - costo) / abs(costo):.3g}; H rel {np.abs(H - Ho).max() / np.abs(Ho).max():.3g}; "
          f"b rel {np.abs(b - bo).max() / np.abs(bo).max():.3g}", flush=True)
    # align parity
    out, res = ctx.align()
    outo, reso = g.align()
    dt = np.abs(out[:3, 3] - outo[:3, 3]).max()
    print(f"align: gpu iters {res.iterations_run} conv {res.converged} trials {res.lm_trials} | "
          f"cpu iters {reso.iterations_run} conv {reso.converged} trials {reso.lm_trials} | "
          f"dt {dt:.3g} m drot {rot_err(out, outo):.3g} rad; device {res.device_ms:.3f} ms", flush=True)
    print(f"  vs truth dt {np.abs(out[:3, 3] - T[:3, 3]).max():.3g}", flush=True)
    # residuals parity
    r = ctx.residuals()
    corr_o, sqd_o = g.last_correspondences()
    print(f"residuals max diff {np.abs(r - np.sqrt(sqd_o.astype(np.float64))).max():.3g}", flush=True)
    # timing loop
    for _ in range(3):
        ctx.align()
    t0 = time.time(); n = 20
    for _ in range(n):
        out, res = ctx.align()
    t1 = time.time()
    print(f"align wall {1e3*(t1-t0)/n:.3f} ms/scan device {res.device_ms:.3f} ms iters {res.iterations_run}", flush=True)
    ctx.set_profiling(True)
    out, res = ctx.align()
    print(f"profiled: device {res.device_ms:.3f} ms linearize total {res.linearize_ms:.3f} ms over "
          f"{res.iterations_run} iters", flush=True)

    if big:
        prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
        sub = np.concatenate(prob["keyframes"])[prob["subset"]]
        kcov = np.concatenate([O.covariances(k, 10) for k in prob["keyframes"]])[prob["subset"]]
        c2 = Context(0)
        c2.set_params(default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32,
                                     transformation_epsilon=0.01))
        t0 = time.time(); c2.set_target(sub); t1 = time.time()
        print(f"S2M set_target 500k {1e3*(t1-t0):.2f} ms", flush=True)
        c2.set_covariances(TARGET, kcov)
        c2.set_source(prob["source"])
        c2.set_covariances(SOURCE, O.covariances(prob["source"], 10))
        for _ in range(3):
            out, res = c2.align(prob["guess"])
        t0 = time.time(); n = 20
        for _ in range(n):
            out, res = c2.align(prob["guess"])
        t1 = time.time()
        print(f"S2M align {1e3*(t1-t0)/n:.3f} ms/scan, device {res.device_ms:.3f} ms, iters {res.iterations_run}, "
              f"conv {res.converged}, nc {res.num_correspondences}", flush=True)
        print(f"  vs truth dt {np.abs(out[:3, 3] - prob['T_true'][:3, 3]).max():.3g} rot {rot_err(out, prob['T_true']):.3g}")
        c2.set_profiling(True)
        out, res = c2.align(prob["guess"])
        print(f"  profiled linearize {res.linearize_ms:.3f} ms over {res.iterations_run} iters", flush=True)
        p2 = c2.get_params().replace(fixed_iterations=20, optimizer=0)
        c2.set_params(p2)
        c2.set_profiling(False)
        for _ in range(2):
            c2.align(prob["guess"])
        t0 = time.time()
        for _ in range(n):
            out, res = c2.align(prob["guess"])
        t1 = time.time()
        print(f"S2M GN fixed 20: {1e3*(t1-t0)/n:.3f} ms/scan ({20*n/(t1-t0):.1f} iters/s), device {res.device_ms:.3f} ms", flush=True)
        c2.set_profiling(True)
        out, res = c2.align(prob["guess"])
        print(f"  profiled linearize {res.linearize_ms:.3f} ms / 20 = {res.linearize_ms/20*1e3:.1f} us per launch", flush=True)
        t0 = time.time(); c2.compute_covariances(TARGET); t1 = time.time()
        print(f"  covariances 500k k=20: {1e3*(t1-t0):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
