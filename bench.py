"""Benchmark of the GICP hot path on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], SURVEY.md §8(d) cfg 3): S2M GICP of a
131,072-point 64x2048 scan against a 500,000-point fused submap of 4
keyframes (target covariances per keyframe, k=10 PLANE, as
odom.cc:1147-1149,1302-1310), reference S2M parameters (ddlo.yaml:196-201:
maxCorr 2.0 m, maxIterations 32, transformationEpsilon 0.01, LM), initial
guess = ground truth perturbed by t=(0.30,-0.20,0.05) m, yaw 2 deg,
roll/pitch 0.5 deg.  Synthetic data (scene.py ray-caster, no datasets).

One step = one align() (NanoGICP::computeTransformation), index build and
covariances excluded (SURVEY.md §8(d) "ms/scan").  value = outer GICP
iterations per second over the whole job (all ranks); ms_per_step = ms/scan.

Multi-GPU (torchrun, one process per GPU): the headline runs an independent
replica per GPU (weak scaling, no data-path collective); torch.distributed is
used for the barrier and max-time / sum-work only.  Extra legs in the same
JSON line: s2s_gn (cfg 2, 20 fixed GN iterations), sharded_s2m (cfg 4,
spatial shards + one RCCL all-reduce per iteration), batched_s2s (cfg 5
frame-parallel S2S) and odometry (cfg 5 S2M chain through the ddlo_odom
driver, one independent chain per rank's frame segment).

Roofline: the linearize step (k_nn_seed + k_nn_collect + k_nn_scan +
k_moments, launched back to back per outer iteration) timed with HIP events
on the library's stream inside this process; algorithmic bytes per launch =
76 * N_s (SURVEY.md §8(d) B_lin), peak HBM 8 TB/s (MI355X_MICROARCH.md);
traffic = HBM-side bytes per launch from the committed rocprofv3 --pmc
passes (profiles/r06_traffic.json).  cpu_baseline = the C++/OpenMP
oracle (oracle/cpu_ref.cpp, a restatement of the reference algorithm, "port")
timed on this host on the same problem.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "GICP iters/sec + ms/scan, 131k-pt source → 500k-pt submap; pose Δ vs CPU ref"
HBM_PEAK_GBS = 8000.0
# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this same workload
# (tools/pmc_traffic.sh -> tools/pmc_traffic.py), committed per round
TRAFFIC_JSON = os.environ.get("DDLO_TRAFFIC_JSON", os.path.join(HERE, "profiles", "r06_traffic.json"))


def pmc_traffic():
    """Measured HBM-side bytes per linearize launch (FETCH_SIZE + WRITE_SIZE as read:
    the search kernels are gathers, outside the x2 calibration of MI355X_MICROARCH.md),
    or None when no PMC pass is on file."""
    try:
        with open(TRAFFIC_JSON) as f:
            d = json.load(f)
        return int(d["bytes_per_linearize"]), os.path.relpath(TRAFFIC_JSON, HERE)
    except (OSError, KeyError, ValueError):
        return None, None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_problem():
    from dynamic_direct_lidar_odometry_amd import scene
    prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
    return prob


def keyframe_covariances(ctx_factory, keyframes, k=10):
    """Per-keyframe covariances on the GPU (odom.cc:1147-1149), concatenated (:1302-1310)."""
    from dynamic_direct_lidar_odometry_amd import SOURCE, default_params
    covs = []
    c = ctx_factory()
    c.set_params(default_params(k_correspondences=k))
    for kf in keyframes:
        c.set_source(kf)
        c.compute_covariances(SOURCE)
        covs.append(c.get_covariances(SOURCE))
    c.close()
    return np.concatenate(covs)


def reduce_over_ranks(dist, elapsed, iters, device):
    """Job time = MAX over ranks of the timed region; work = SUM of iterations
    (replicas: every rank aligns its own scan stream)."""
    if dist is None:
        return float(elapsed), float(iters)
    import torch
    t = torch.tensor([elapsed, float(iters)], dtype=torch.float64, device=device)
    tmax = t.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    tsum = t.clone()
    dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
    return float(tmax[0]), float(tsum[1])


def host_info(threads):
    """CPU model (/proc/cpuinfo, as lscpu's "Model name") and core counts of this host."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    quota = None   # the job's CPU share (cgroup v2 cpu.max: quota period)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "omp_threads": threads}


def varied_guesses(prob):
    """8 initial guesses around the cfg3 ground truth: the SURVEY perturbation scaled and rotated."""
    from dynamic_direct_lidar_odometry_amd import scene
    out = []
    T = prob["T_true"]
    for i, (sc, yaw) in enumerate([(1.0, 0), (0.5, 30), (1.5, 60), (0.25, 90), (1.2, 140), (0.75, 200),
                                   (1.0, 250), (0.4, 310)]):
        a = math.radians(yaw)
        t = np.array([0.30 * math.cos(a) - (-0.20) * math.sin(a), 0.30 * math.sin(a) + (-0.20) * math.cos(a), 0.05])
        P = scene.make_pose(sc * t, (math.radians(0.5 * sc), math.radians(-0.5 * sc if i % 2 else 0.5 * sc),
                                     math.radians(2.0 * sc * (1 if i % 3 else -1))))
        out.append((T @ P).astype(np.float32))
    return out


def roofline_block(bytes_per_launch, launch_s, kernel, unit_bytes):
    """roofline dict for a kernel (group): SURVEY.md §8(d) algorithmic bytes per launch / average launch time."""
    ach = bytes_per_launch / launch_s / 1e9 if launch_s > 0 else 0.0
    return {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 6), "kernel": kernel, "avg_launch_us": round(launch_s * 1e6, 2),
            "algorithmic_bytes_per_launch": int(bytes_per_launch), "bytes_rule": unit_bytes}


def lin_kernel_label(ctx):
    g = ctx.grid_info()
    if g["built"] and not g["uses_walk"]:
        return "linearize = k_moments with the fused candidate-cell lookup (one kernel per outer iteration)"
    if g["built"]:
        return "linearize = k_cell_lookup + k_nn_seed (walk of the unlisted sub-groups) + k_moments (per outer iteration)"
    return "linearize = k_nn_seed + k_nn_scan + k_moments (per outer iteration)"


def lin_roofline(ctx, guess, n_owned, reps=5):
    """Linearize roofline of a ctx's align (HIP events on the library stream, gicp_set_profiling)."""
    ctx.set_profiling(True)
    ms, launches = 0.0, 0
    for _ in range(reps):
        _, r = ctx.align(guess)
        ms += r.linearize_ms
        launches += r.iterations_run
    ctx.set_profiling(False)
    ctx.synchronize()
    return roofline_block(76.0 * n_owned, ms * 1e-3 / max(launches, 1), lin_kernel_label(ctx),
                          "B_lin = 76 B x owned source points")


def cfg3_walk_leg(ctx, guess, args, result):
    """The headline's aligns with the target's candidate cells off: the seed + walk + scan search."""
    from dynamic_direct_lidar_odometry_amd import GRID_OFF, GRID_ON
    ctx.set_target_grid(GRID_OFF)
    for _ in range(3):
        ctx.align(guess)
    ctx.synchronize()
    t_w = time.perf_counter()
    nw = max(20, args.steps // 4)
    for _ in range(nw):
        ctx.align(guess)
    ctx.synchronize()
    walk_ms = 1e3 * (time.perf_counter() - t_w) / nw
    ctx.set_profiling(True)
    wl_ms, wl_n = 0.0, 0
    for _ in range(5):
        _, r = ctx.align(guess)
        wl_ms += r.linearize_ms
        wl_n += r.iterations_run
    ctx.set_profiling(False)
    ctx.set_target_grid(GRID_ON)
    result["cfg3_walk"] = {"ms_per_scan": round(walk_ms, 4), "linearize_us": round(1e3 * wl_ms / max(wl_n, 1), 2),
                           "note": "candidate cells off (gicp_set_target_grid 0): the seed + walk + scan search"}


def rot_err(A, B):
    """Rotation angle between A and B: 2*asin(|RA - RB|_F / sqrt(8)) (well conditioned at 0)."""
    f = float(np.linalg.norm(A[:3, :3].astype(np.float64) - B[:3, :3].astype(np.float64)))
    return 2.0 * math.asin(min(1.0, f / math.sqrt(8.0)))


def sharded_leg(dist, rank, world, local_rank, args):
    """BASELINE.json configs[3] / SURVEY.md §8(e): 262,144-pt 128x2048 scan vs
    a 2,000,000-pt 8-keyframe submap, spatially sharded over the job's GPUs
    (slab + 2 m halo per rank, one RCCL all-reduce of the 80 moment doubles
    per outer iteration inside the align graph).  With one GPU it is the same
    code path with a one-rank communicator.  Reported next to the replica
    metric; strong scaling (fixed problem), so compare across n_gpus."""
    import dynamic_direct_lidar_odometry_amd as P
    from dynamic_direct_lidar_odometry_amd import scene, SOURCE
    from dynamic_direct_lidar_odometry_amd.shard import ShardedGicp

    t0 = time.time()
    prob = scene.s2m_problem(128, 2048, 8, 2000000, 4)
    sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
    src = prob["source"]
    kcov = keyframe_covariances(lambda: P.Context(local_rank), prob["keyframes"], k=10)
    tcov = np.ascontiguousarray(kcov[prob["subset"]])
    c = P.Context(local_rank)
    c.set_params(P.default_params(k_correspondences=10))
    c.set_source(src)
    c.compute_covariances(SOURCE)
    scov = c.get_covariances(SOURCE)
    c.close()
    params = P.default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32,
                              transformation_epsilon=0.01)
    # unique id from rank 0, broadcast over the job's process group
    uid = P.comm_unique_id() if rank == 0 else bytes(128)
    if dist is not None:
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]
    guess = prob["guess"].astype(np.float32)
    sh = ShardedGicp(local_rank, rank, world, uid, params, mode=args.shard_mode)
    sh.ctx.set_target_grid(P.GRID_ON)   # each rank's target's candidate cells, built at the first align
    t_st = time.perf_counter()
    slab = sh.set_target(sub, tcov, source=src, guess=guess)
    set_target_ms = 1e3 * (time.perf_counter() - t_st)
    sh.set_source(src, scov)
    log(f"[rank {rank}] sharded setup {time.time() - t0:.1f}s: src {len(src)} tgt {len(sub)} "
        f"local {len(sh.local_index)} mode {args.shard_mode}" +
        (f" slab axis {slab.axis} [{slab.lo:.2f}, {slab.hi:.2f})" if slab is not None else ""))
    sh.ctx.synchronize()
    t_b = time.perf_counter()
    out, res = sh.align(guess)   # builds the cells (once per target, outside ms/scan)
    first_align_ms = 1e3 * (time.perf_counter() - t_b)
    grid = sh.ctx.grid_info()
    for _ in range(2):
        out, res = sh.align(guess)
    sh.ctx.synchronize()
    if dist is not None:
        dist.barrier()
    t_start = time.perf_counter()
    iters = 0
    for _ in range(args.sharded_steps):
        out, res = sh.align(guess)
        iters += res.iterations_run
    sh.ctx.synchronize()
    elapsed = time.perf_counter() - t_start
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
    local_pts = len(sh.local_index)
    graphs = sh.ctx.comm_info()[2]
    # per-rank linearize roofline (eager profiled aligns: the all-reduce sits outside the timed kernels)
    roof = lin_roofline(sh.ctx, guess, len(src) / world, reps=3)
    dev_bytes = sh.ctx.device_bytes()
    sh.close()
    out_leg = {"workload": "cfg4 S2M: 262,144-pt 128x2048 scan -> 2,000,000-pt 8-keyframe submap, LM, maxCorr 2.0 m",
               "n_gpus": world, "ms_per_scan": round(1e3 * elapsed / args.sharded_steps, 4),
               "shard_mode": (f"groups: target replicated, rank r owns the source's 16-point groups = r mod {world}"
                              if args.shard_mode == "groups" else
                              "slabs: spatial slabs cut on the owned source at the guess, 2 m target halo"),
               "iters_per_s": round(iters / elapsed, 2), "iterations_per_scan": res.iterations_run,
               "converged": bool(res.converged), "target_points_per_rank_max": None,
               "collective": "RCCL all-reduce, 80 fp64 per outer iteration" + (" (in graph)" if graphs else " (eager)"),
               "scaling": "strong", "roofline_rank0": roof,
               "target_grid_rank0": {"built": grid["built"], "build_ms": round(grid["build_ms"], 3),
                                     "bytes": grid["bytes"], "first_align_ms": round(first_align_ms, 3)},
               "set_target_ms_rank0": round(set_target_ms, 2),
               "device_mib_rank0": {k: round(v / 2**20, 2) for k, v in dev_bytes.items()}}
    if dist is not None:
        import torch
        t = torch.tensor([local_pts], dtype=torch.int64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        local_pts = int(t[0])
    out_leg["target_points_per_rank_max"] = local_pts
    if rank == 0:
        # pose parity of the sharded result against the unsharded align on one GPU
        c = P.Context(local_rank)
        c.set_params(params)
        c.set_target(sub)
        c.set_covariances(1, tcov)
        c.set_source(src)
        c.set_covariances(0, scov)
        ref, _ = c.align(guess)
        c.close()
        out_leg["pose_delta_vs_1gpu"] = {"trans_m": float(np.abs(out[:3, 3] - ref[:3, 3]).max()),
                                         "rot_rad": rot_err(out, ref)}
        if not args.no_cpu:
            # the OpenMP oracle on the same cfg4 align, at the cfg3 sweep's fastest thread count
            from oracle import oracle as O
            nthr = getattr(args, "cpu_best_threads", 16)
            g = O.Gicp(src, sub, O.as_params(params), threads=nthr)
            g.set_covariances(0, scov)
            g.set_covariances(1, tcov)
            g.align(guess)
            times = []
            oo = None
            for _ in range(3):
                c0 = time.perf_counter()
                oo, _ = g.align(guess)
                times.append(time.perf_counter() - c0)
            cms = 1e3 * float(np.median(times))
            out_leg["cpu_oracle"] = {"ms_per_scan": round(cms, 3), "threads": nthr, "kind": "port",
                                     "sample": "median of 3 full cfg4 aligns after 1 warm-up, oracle/cpu_ref.cpp",
                                     "speedup_gpu_vs_cpu": round(cms / out_leg["ms_per_scan"], 2),
                                     "pose_delta_vs_cpu": {"trans_m": float(np.abs(out[:3, 3] - oo[:3, 3]).max()),
                                                           "rot_rad": rot_err(out, oo)}}
    return out_leg


_CFG5 = {}


def cfg5_frames(args, first, end, device):
    """Frames [first, end) of cfg 5's 1000-frame loop (scene.loop_sequence: GPU ray caster, test/bench
    infrastructure), cached for the legs that share them."""
    from dynamic_direct_lidar_odometry_amd import scene
    for (a, b), fr in _CFG5.items():
        if a <= first and end <= b:
            return fr[first - a:end - a]
    t0 = time.time()
    _CFG5.clear()
    fr = scene.loop_sequence(64, 2048, first, end - first, device=device)[0]
    # the first DMA read of a fresh host page is slow (~0.1 ms more per 1.5 MB frame in the pageable H2D
    # copy, tools/batch_order.py): upload every frame once here so that both tie-order passes of a leg, and
    # every leg, see the same host-page state (else the first pass over the frames pays it alone)
    import dynamic_direct_lidar_odometry_amd as P
    c = P.Context(device)
    for f in fr:
        c.set_source(f)   # H2D + index build of the frame, nothing else
    c.close()
    _CFG5[(first, end)] = fr
    log(f"cfg5 frames {first}..{end - 1}: {time.time() - t0:.1f}s")
    return _CFG5[(first, end)]


def batched_leg(dist, rank, world, local_rank, args):
    """BASELINE.json configs[4] / SURVEY.md §8(e) cfg 5: frame-parallel S2S
    over a 64x2048 scan sequence (moving pedestrians), the frames split into
    one contiguous range per rank (no collective; every pair needs only its
    two scans) and, inside a rank, into `--batch-streams` chained chunks on
    their own HIP streams (gicp_s2s_batch).  Each pair pays the real per-scan
    cost: H2D upload, index build, k=10 covariances and the align."""
    import dynamic_direct_lidar_odometry_amd as P
    t0 = time.time()
    npairs = args.batch_frames - 1
    a = npairs * rank // world
    b = npairs * (rank + 1) // world
    mine = cfg5_frames(args, a, b + 1, local_rank)
    params = P.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32,
                              transformation_epsilon=0.01)   # ddlo.yaml:187-192 (S2S)
    log(f"[rank {rank}] batch setup {time.time() - t0:.1f}s: pairs {a}..{b}")
    P.s2s_batch(mine[:min(len(mine), 2 * args.batch_streams + 1)], params, device=local_rank,
                nstreams=args.batch_streams)   # warmup (allocations, graphs)
    if dist is not None:
        dist.barrier()
    c0 = time.perf_counter()
    poses, res = P.s2s_batch(mine, params, device=local_rank, nstreams=args.batch_streams)
    elapsed = time.perf_counter() - c0
    iters = sum(r.iterations_run for r in res[1:])
    elapsed, iters_total = reduce_over_ranks(dist, elapsed, iters, f"cuda:{local_rank}")
    # the same pairs with ties in the device's Morton order (gicp_set_tie_order(0): no nanoflann tree)
    with tie_order_env("0"):
        if dist is not None:
            dist.barrier()
        c0 = time.perf_counter()
        P.s2s_batch(mine, params, device=local_rank, nstreams=args.batch_streams)
        el_m = time.perf_counter() - c0
    el_m, _ = reduce_over_ranks(dist, el_m, 0, f"cuda:{local_rank}")
    stages = cfg5_stage_rooflines(mine, params, local_rank) if rank == 0 else None
    return {"cfg5_stages_rank0": stages,
            "workload": f"cfg5 frame-parallel S2S: {npairs} pairs of {args.batch_frames} unique 64x2048 scans "
                        f"(closed plaza loop, moving pedestrians), k=10, maxCorr 1.0 m",
            "n_gpus": world, "streams_per_gpu": args.batch_streams, "pairs": npairs,
            "pairs_per_s": round(npairs / elapsed, 2), "ms_per_pair": round(1e3 * elapsed / npairs, 4),
            "iters_per_s": round(iters_total / elapsed, 2), "tie_order": "nanoflann (exact)",
            "ms_per_pair_morton_tie_order": round(1e3 * el_m / npairs, 4),
            "per_pair_work": "H2D + index build + covariances (+ nanoflann's tree for the tie order) + align",
            "collective": "none (frames split by rank)"}


def cfg5_stage_rooflines(frames, params, device, nframes=24):
    """The per-scan stages of the cfg5 S2S leg, device-timed (HIP events) on one ctx over consecutive frames:
    k=10 covariances (B_cov = 36 B x N), nanoflann's tree (tie order; B_idx = 32 B x N, SURVEY.md §8(d)'s
    index-build figure), the S2S align's linearize (B_lin = 76 B x N_s)."""
    import dynamic_direct_lidar_odometry_amd as P
    from dynamic_direct_lidar_odometry_amd import SOURCE
    c = P.Context(device)
    c.set_params(params)
    cov_s = tree_s = res_s = lin_s = 0.0
    n_pts = lin_launch = tree_n = 0
    fr = frames[:nframes + 1]
    c.set_target(fr[0])
    c.compute_covariances(1)
    for t in range(1, len(fr)):
        c.set_source(fr[t])
        c.set_profiling(True)
        c.compute_covariances(SOURCE)
        cm, tm, rm = c.stage_times()
        _, r = c.align()
        c.set_profiling(False)
        if t > 2:   # first frames: allocations and graph captures
            cov_s += cm * 1e-3
            res_s += rm * 1e-3
            if tm > 0:
                tree_s += tm * 1e-3
                tree_n += len(fr[t])
            n_pts += len(fr[t])
            lin_s += r.linearize_ms * 1e-3
            lin_launch += r.iterations_run
        c.swap_source_target()
    c.close()
    k = max(len(fr) - 3, 1)
    mean_n = n_pts / k
    return {"frames": k, "mean_points": round(mean_n, 1),
            "covariances": roofline_block(36.0 * mean_n, cov_s / k, "k_covariances2<10> (k-NN k=10 + PLANE)",
                                          "B_cov = 36 B x N"),
            "nanoflann_tree": roofline_block(32.0 * tree_n / k, tree_s / k,
                                             "nanoflann tree build (k_nf_* graph, aux stream)",
                                             "B_idx = 32 B x N (index-build figure)"),
            "tie_resolvers_us": round(1e6 * res_s / k, 2),
            "s2s_linearize": roofline_block(76.0 * mean_n, lin_s / max(lin_launch, 1),
                                            "linearize = k_nn_seed + k_nn_scan + k_moments", "B_lin = 76 B x N_s")}


def tie_order_env(v):
    """Contexts created inside the block use the given tie order ("0": Morton, no nanoflann trees)."""
    import dynamic_direct_lidar_odometry_amd as P
    return P.default_option(P.OPT_TIE_ORDER, int(v))


def s2s_gn_leg(local_rank, args):
    """BASELINE.json configs[1] / SURVEY.md §8(d) cfg 2: S2S GICP of two
    64x2048 (131,072-pt) scans, 20 fixed Gauss-Newton outer iterations
    (optimizer GN, fixed_iterations 20, convergence off), k=10 covariances
    resident.  One step = one align of 20 iterations."""
    import dynamic_direct_lidar_odometry_amd as P
    from dynamic_direct_lidar_odometry_amd import scene, SOURCE, TARGET
    src, tgt, _ = scene.s2s_pair(64, 2048, 2)
    c = P.Context(local_rank)
    c.set_params(P.default_params(k_correspondences=10, max_correspondence_distance=1.0, optimizer=P.GAUSS_NEWTON,
                                  fixed_iterations=20, max_iterations=20))
    # S2S targets are used once (OdomNode swaps every scan, odom.cc:768): the
    # walk, as in the pipeline (AUTO would build cells at this loop's 2nd align)
    c.set_target_grid(P.GRID_OFF)
    c.set_target(tgt)
    c.set_source(src)
    c.compute_covariances(SOURCE)
    c.compute_covariances(TARGET)
    for _ in range(2):
        c.align()
    c.synchronize()
    t0 = time.perf_counter()
    iters = 0
    for _ in range(args.gn_steps):
        _, r = c.align()
        iters += r.iterations_run
    c.synchronize()
    el = time.perf_counter() - t0
    roof = lin_roofline(c, None, len(src), reps=2)
    c.close()
    return {"workload": f"cfg2 S2S GICP: {len(src)}-pt -> {len(tgt)}-pt 64x2048 scans, 20 fixed GN iterations, "
                        "k=10, maxCorr 1.0 m", "iters_per_s": round(iters / el, 2),
            "ms_per_align": round(1e3 * el / args.gn_steps, 4), "iterations_per_align": iters // args.gn_steps,
            "roofline": roof}


def segmentation_leg(local_rank, args):
    """range-image segmentation (include/ddlo_segment.h)
    of one 512x512 organized scan with cfg/ddlo.yaml's detection parameters:
    H2D, the fused per-pixel device pass (projection, ground, label init), the
    read-back and the host labelling.  One step = one ddlo_seg_process."""
    import math
    from dynamic_direct_lidar_odometry_amd import scene
    from dynamic_direct_lidar_odometry_amd import segmentation as SG
    sc = scene.make_scene(1005, moving=True)
    pose = scene.make_pose([0.0, 0.0, scene.SENSOR_Z], (0.0, 0.0, math.radians(20.0)))
    pts = scene.raycast(sc, pose, 512, 512, 1005, organized=True)
    bad = ~np.isfinite(pts).all(axis=1)
    xyz = scene.transform(np.nan_to_num(pts, nan=0.0), pose).astype(np.float32)
    xyz[bad] = np.nan
    T = pose.astype(np.float32)
    resid = np.abs(np.random.default_rng(0).normal(0, 0.2, (512, 512))).astype(np.float32)
    seg = SG.Segmentation(local_rank, SG.yaml_seg_params())
    for _ in range(3):
        r = seg.process(xyz, T, resid)
    t0 = time.perf_counter()
    for _ in range(args.seg_steps):
        r = seg.process(xyz, T, resid)
    el = time.perf_counter() - t0
    seg.close()
    return {"workload": "range-image segmentation, 512x512 organized scan, ddlo.yaml detection parameters "
                        "(window rows/cols 156..356)", "ms_per_frame": round(1e3 * el / args.seg_steps, 4),
            "frames_per_s": round(args.seg_steps / el, 2), "segments": r.segments, "ground_pixels": r.ground_pixels}


def odometry_leg(dist, rank, world, local_rank, args, frames=None):
    """BASELINE.json configs[4], the S2M half (SURVEY.md §8(e) cfg 5): the
    odometry driver (include/ddlo_odom.h, cfg/ddlo.yaml parameters) over the
    64x2048 scan sequence — per frame upload, crop box + voxel filter,
    spaciousness, S2S, submap selection / assembly, S2M, keyframe insertion.
    The S2M chain is sequential, so with N GPUs the sequence is cut into N
    contiguous segments, each an independent chain (its own keyframe map)."""
    from dynamic_direct_lidar_odometry_amd import odometry as OD
    a = args.batch_frames * rank // world
    b = args.batch_frames * (rank + 1) // world
    mine = frames[a:b] if frames is not None else cfg5_frames(args, a, b, local_rank)
    warm = OD.Odometry(local_rank)
    for f in mine[:4]:
        warm.process(f)
    warm.close()
    odo = OD.Odometry(local_rank)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    kfs, tracked, s2m_it, pts, max_sub, changes = 0, 0, 0, 0, 0, 0
    for f in mine:
        r = odo.process(f)
        kfs += r.keyframe_added
        tracked += r.status == OD.TRACKED
        s2m_it += r.s2m.iterations_run
        pts += r.scan_points
        max_sub = max(max_sub, int(r.submap_points))
        changes += r.submap_changed
    el = time.perf_counter() - t0
    nk = r.num_keyframes
    sub_pts = int(r.submap_points)
    odo.close()
    el, nframes = reduce_over_ranks(dist, el, len(mine), f"cuda:{local_rank}")
    with tie_order_env("0"):   # the same chain with ties in Morton order (no nanoflann trees)
        odo = OD.Odometry(local_rank)
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        for f in mine:
            odo.process(f)
        el_m = time.perf_counter() - t0
        odo.close()
    el_m, _ = reduce_over_ranks(dist, el_m, 0, f"cuda:{local_rank}")
    return {"workload": f"cfg5 S2M chain: odometry driver over {args.batch_frames} unique 64x2048 frames "
                        "(closed plaza loop: 22 x 12 m ellipse at 1.5 m/s, ~1.4 laps, 3 cm range noise, moving pedestrians), "
                        "ddlo.yaml parameters "
                        "(crop 1 m, voxel 0.1 m, S2S k=10 / S2M k=20, adaptive keyframes, knn/kcv/kcc 10)",
            "n_gpus": world, "frames": int(nframes), "frames_per_s": round(nframes / el, 2),
            "ms_per_frame": round(1e3 * el / nframes, 4), "tie_order": "nanoflann (exact)",
            "ms_per_frame_morton_tie_order": round(1e3 * el_m / nframes, 4),
            "per_frame_work": "H2D + crop + voxel + metrics + S2S (index, covariances, align) + submap + S2M + keyframes",
            "rank0": {"keyframes": nk, "last_submap_points": sub_pts, "max_submap_points": max_sub,
                      "submap_changes": changes, "tracked": tracked,
                      "mean_scan_points": round(pts / max(len(mine), 1), 1),
                      "mean_s2m_iterations": round(s2m_it / max(tracked, 1), 2)},
            "segments": f"{world} independent chains (contiguous frame ranges)"}


def main():
    # Native libraries (RCCL's version banner) print to fd 1; the contract is
    # ONE JSON line on stdout, so route fd 1 to stderr and keep the real
    # stdout for the result line only.
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--cpu-runs", type=int, default=10, help="oracle align runs for cpu_baseline (median)")
    ap.add_argument("--cpu-warmup", type=int, default=2, help="untimed oracle aligns before them")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-sharded", action="store_true", help="skip the spatially sharded cfg4 leg")
    ap.add_argument("--sharded-steps", type=int, default=10)
    ap.add_argument("--shard-mode", choices=["groups", "slabs"], default="groups",
                    help="cfg4 ownership: interleaved source groups (replicated target) or source-balanced slabs")
    ap.add_argument("--no-batch", action="store_true", help="skip the frame-parallel S2S cfg5 leg")
    ap.add_argument("--batch-frames", type=int, default=1000, help="cfg 5 sequence length (unique frames)")
    ap.add_argument("--batch-streams", type=int, default=3,
                    help="frame-parallel S2S workers (one ctx each); inside this process 3 measured best (0.47 ms/pair "
                         "against 0.60 at 4 or 6; a fresh process prefers 4, DESIGN.md §5)")
    ap.add_argument("--no-gn", action="store_true", help="skip the cfg2 S2S 20-GN-iteration leg")
    ap.add_argument("--gn-steps", type=int, default=10)
    ap.add_argument("--no-odom", action="store_true", help="skip the cfg5 odometry-driver (S2M chain) leg")
    ap.add_argument("--no-seg", action="store_true", help="skip the range-image segmentation leg")
    ap.add_argument("--no-walk", action="store_true",
                    help="skip the cfg3 comparison with the candidate cells off (counter / trace runs of the headline)")
    ap.add_argument("--seg-steps", type=int, default=50)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as td
        torch.cuda.set_device(local_rank)
        td.init_process_group(backend="nccl")
        dist = td

    from dynamic_direct_lidar_odometry_amd import Context, default_params, SOURCE, TARGET, GRID_ON, GRID_OFF

    t0 = time.time()
    prob = build_problem()
    sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
    src = prob["source"]
    kcov_all = keyframe_covariances(lambda: Context(local_rank), prob["keyframes"], k=10)
    tcov = np.ascontiguousarray(kcov_all[prob["subset"]])
    params = default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32,
                            transformation_epsilon=0.01)
    ctx = Context(local_rank)
    # source covariances as the pipeline makes them: by the S2S instance, k=10
    # (odom.cc:765 copies them into S2M; ddlo.yaml:188)
    ctx.set_params(default_params(k_correspondences=10))
    ctx.set_source(src)
    ctx.compute_covariances(SOURCE)
    scov = ctx.get_covariances(SOURCE)
    ctx.set_params(params)
    ctx.set_target_grid(GRID_ON)   # the submap's candidate cells, built at the first align
    ctx.set_target(sub)
    ctx.set_covariances(TARGET, tcov)
    guess = prob["guess"].astype(np.float32)
    log(f"[rank {rank}] setup {time.time() - t0:.1f}s: src {len(src)} tgt {len(sub)}")
    # the per-target build (once per setInputTarget; like the index, outside ms/scan): the first align
    ctx.synchronize()
    t_b = time.perf_counter()
    ctx.align(guess)
    first_align_ms = 1e3 * (time.perf_counter() - t_b)
    grid_info = ctx.grid_info()

    # warmup
    for _ in range(args.warmup):
        out, res = ctx.align(guess)
    ctx.synchronize()

    # timed region: K aligns, barrier + sync on both sides, max over ranks
    if dist:
        dist.barrier()
    ctx.synchronize()
    t_start = time.perf_counter()
    iters = 0
    for _ in range(args.steps):
        out, res = ctx.align(guess)
        iters += res.iterations_run
    ctx.synchronize()
    t_end = time.perf_counter()
    elapsed, iters_total = reduce_over_ranks(dist, t_end - t_start, iters, f"cuda:{local_rank}")
    steps_total = args.steps * world
    value = iters_total / elapsed
    ms_per_step = 1e3 * elapsed / args.steps

    # roofline: linearize launches timed with HIP events on the library stream
    ctx.set_profiling(True)
    lin_ms, lin_launches = 0.0, 0
    for _ in range(max(3, min(args.steps, 10))):
        _, r = ctx.align(guess)
        lin_ms += r.linearize_ms
        lin_launches += r.iterations_run
    ctx.set_profiling(False)
    ctx.synchronize()
    avg_launch_s = (lin_ms / max(lin_launches, 1)) * 1e-3
    bytes_per_launch = 76.0 * len(src)   # SURVEY.md §8(d) B_lin = 76 * N_s
    traffic, traffic_src = pmc_traffic()
    achieved_gbs = bytes_per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GICP iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 search / f64 normal equations",
        "data": "synthetic (ray-cast plaza, scene.py; no datasets)",
        "config": {"workload": "cfg3 S2M GICP: 131,072-pt 64x2048 scan -> 500,000-pt 4-keyframe submap, "
                               "LM, maxCorr 2.0 m, maxIter 32, transEps 0.01",
                   "source_points": int(len(src)), "target_points": int(len(sub)),
                   "iterations_per_scan": round(iters_total / steps_total, 3),
                   "parallelism": f"replicas x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved_gbs / HBM_PEAK_GBS, 6), "traffic": traffic,
                     "traffic_unit": "bytes per linearize launch (L2->fabric, Infinity-Cache hits included; counters as read)",
                     "traffic_source": traffic_src,
                     "kernel": lin_kernel_label(ctx),
                     "avg_launch_us": round(avg_launch_s * 1e6, 2),
                     "algorithmic_bytes_per_launch": int(bytes_per_launch)},
    }

    result["target_grid"] = {**grid_info, "first_align_ms": round(first_align_ms, 3),
                             "walk_groups_last_align": ctx.lookup_walk_groups(),
                             "note": "candidate cells of the submap, built once per target (first align, outside "
                                     "ms/scan like the index build, SURVEY.md §8(d)); the odometry leg pays them"}
    # the same aligns with the cells off (the round-4 walk), for comparison
    if not args.no_walk:
        cfg3_walk_leg(ctx, guess, args, result)

    # the launch predictor's misses in the number: cycle 8 distinct guesses
    # (the headline repeats one, so its iteration count is always predicted)
    guesses = varied_guesses(prob)
    for g in guesses[:2]:
        ctx.align(g)
    ctx.synchronize()
    t_v = time.perf_counter()
    v_iters = 0
    for s_i in range(max(args.steps, 16)):
        _, r = ctx.align(guesses[s_i % len(guesses)])
        v_iters += r.iterations_run
    ctx.synchronize()
    el_v = time.perf_counter() - t_v
    nv = max(args.steps, 16)
    result["cfg3_varied_guesses"] = {"guesses": len(guesses), "aligns": nv, "ms_per_scan": round(1e3 * el_v / nv, 4),
                                     "iters_per_s": round(v_iters / el_v, 2),
                                     "iterations_per_scan": round(v_iters / nv, 3),
                                     "note": "same cfg3 problem, guesses cycled so consecutive aligns converge in "
                                             "different iteration counts"}

    if rank == 0 and not args.no_cpu:
        from oracle import oracle as O
        # The reference runs num_threads_ = omp_get_max_threads() (nano_gicp_impl.hpp:52-56), i.e. every
        # host core.  A GPU box's job is cgroup-limited (cpu.max) to a share of a large host, so "all cores"
        # is not the fastest setting there: the oracle is timed at 8, 16, 32, 64, 128 threads and at the
        # affinity count, and the headline baseline is the FASTEST median (the most favourable CPU figure).
        try:
            affinity = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            affinity = os.cpu_count() or 1
        thread_set = sorted({t for t in (8, 16, 32, 64, 128) if t <= affinity} | {affinity})

        def cpu_ms_at(nthreads, runs):
            g = O.Gicp(src, sub, O.as_params(params), threads=nthreads)
            g.set_covariances(0, scov)
            g.set_covariances(1, tcov)
            for _ in range(args.cpu_warmup):
                g.align(guess)
            times = []
            oo = ro = None
            for _ in range(runs):
                c0 = time.perf_counter()
                oo, ro = g.align(guess)
                times.append(time.perf_counter() - c0)
            return 1e3 * float(np.median(times)), oo, ro

        by_threads = {}
        oout = ores = None
        for t in thread_set:
            # a throttled setting (far above the cgroup share) takes seconds per align: 3 runs are enough to
            # show it is not the fastest
            runs = args.cpu_runs if t <= 128 else min(args.cpu_runs, 3)
            ms_t, oo, ro = cpu_ms_at(t, runs)
            by_threads[t] = round(ms_t, 3)
            if oout is None:
                oout, ores = oo, ro
        best_t = min(by_threads, key=by_threads.get)
        cpu_ms = by_threads[best_t]
        args.cpu_best_threads = best_t   # the cfg4 leg's oracle timing uses the same thread count
        result["cpu_baseline"] = {"value": round(cpu_ms, 3), "unit": "ms/scan", "cores": best_t, "kind": "port",
                                  "sample": f"median of {args.cpu_runs} full S2M aligns of the same cfg3 problem after "
                                            f"{args.cpu_warmup} warm-ups ({ores.iterations_run} iters each), OpenMP "
                                            f"oracle oracle/cpu_ref.cpp at -O2; fastest of the thread sweep "
                                            f"{thread_set} ({best_t} threads)",
                                  "ms_by_threads": {str(k): v for k, v in by_threads.items()},
                                  "value_all_cores": by_threads[affinity], "threads_all_cores": affinity,
                                  "value_16_threads": by_threads.get(16), "value_8_threads": by_threads.get(8),
                                  "host": host_info(best_t),
                                  "validation": "profiles/r03_cpu_validation.json (cpu_ref search stages vs the "
                                                "reference's own nanoflann, same inputs)",
                                  "speedup_gpu_vs_cpu": round(cpu_ms / ms_per_step, 2),
                                  "speedup_gpu_vs_cpu_all_cores": round(by_threads[affinity] / ms_per_step, 2),
                                  "speedup_gpu_vs_cpu_16_threads": (round(by_threads[16] / ms_per_step, 2)
                                                                   if 16 in by_threads else None)}
        result["pose_delta_vs_cpu"] = {"trans_m": float(np.abs(out[:3, 3] - oout[:3, 3]).max()),
                                       "rot_rad": rot_err(out, oout)}
    ctx.close()
    if not args.no_sharded:
        result["sharded_s2m"] = sharded_leg(dist, rank, world, local_rank, args)
    if not args.no_gn:
        result["s2s_gn"] = s2s_gn_leg(local_rank, args)
    if not args.no_batch:
        result["batched_s2s"] = batched_leg(dist, rank, world, local_rank, args)
    if not args.no_odom:
        result["odometry"] = odometry_leg(dist, rank, world, local_rank, args)
    if not args.no_seg:
        result["segmentation"] = segmentation_leg(local_rank, args)
    if rank == 0:
        print(json.dumps(result), file=json_out, flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
