"""Per-group timeline of k_covariances2 (k = 10) on cfg 5 scans, from a -DDDLO_COV_PROF build (make covprof):
every 32-query group stores its start / end s_memrealtime stamps (100 MHz), leaves scanned and exact-tested,
splits, its hardware slot and the group's largest k-th distance.
    DDLO_GICP_LIB=.../_lib/covprof/libddlo_gicp.so python tools/cov_timeline.py [frames]
Prints the duration distribution, the kernel span, the slowest groups and how the duration follows the
leaves scanned and the k-th distance; with --voxel the voxel-filtered scans of the odometry driver."""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, ".")
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import TARGET, scene  # noqa: E402
from dynamic_direct_lidar_odometry_amd import odometry as OD  # noqa: E402

nf = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 4
voxel = "--voxel" in sys.argv
frames = scene.loop_sequence(64, 2048, 0, nf, device=0)[0]
L = P.load()
L.ddlo_dev_cov_prof.restype = C.c_int
buf = np.zeros((8192, 4), np.uint64)
buf2 = np.zeros((8192, 4), np.uint64)   # s_memtime cycles: point wait, leaf scans, box tests; leaf blocks
has2 = hasattr(L, "ddlo_dev_cov_prof2")
c = P.Context(0)
c.set_params(P.default_params(k_correspondences=10))
c.set_tie_order(False)
for fi, f in enumerate(frames):
    if voxel:
        f = OD.preprocess(f, 1.0, 0.25)
    c.set_target(f)
    c.compute_covariances(TARGET)
    c.synchronize()
    assert L.ddlo_dev_cov_prof(buf.ctypes.data_as(C.c_void_p)) == 0
    ng = (len(f) + 31) // 32
    if has2:
        assert L.ddlo_dev_cov_prof2(buf2.ctypes.data_as(C.c_void_p)) == 0
        b2 = buf2[:ng][buf[:ng, 1] != 0].astype(np.float64)
    b = buf[:ng]
    t0 = b[:, 0].astype(np.int64)
    t1 = b[:, 1].astype(np.int64)
    dur = (t1 - t0) / 100.0   # us
    scan = (b[:, 2] & 0xffffffff).astype(np.int64)
    exact = (b[:, 2] >> 32).astype(np.int64)
    kd = np.frombuffer((b[:, 3] & 0xffffffff).astype(np.uint32).tobytes(), np.float32)
    splits = ((b[:, 3] >> 32) & 0xff).astype(np.int64)
    span = (t1.max() - t0.min()) / 100.0
    start = (t0 - t0.min()) / 100.0
    print(f"frame {fi}: n {len(f)} groups {ng} kernel span {span:.1f} us; group us p50 {np.median(dur):.1f} "
          f"p90 {np.percentile(dur, 90):.1f} p99 {np.percentile(dur, 99):.1f} max {dur.max():.1f}; "
          f"last start {start.max():.1f} us; leaves scanned p50 {np.median(scan):.0f} p99 "
          f"{np.percentile(scan, 99):.0f} max {scan.max()}", flush=True)
    order = np.argsort(-dur)[:12]
    for g in order:
        print(f"   group {g:5d} start {start[g]:7.1f} dur {dur[g]:7.1f} us scanned {scan[g]:4d} exact {exact[g]:4d} "
              f"splits {splits[g]} kth {np.sqrt(max(kd[g], 0)):.3f} m")
    cc = np.corrcoef(dur, scan)[0, 1]
    fin = start + dur
    # when do groups finish: fraction of groups done by each 10% of the span
    q = [float(np.mean(fin <= span * x)) for x in (0.25, 0.5, 0.75, 0.9)]
    print(f"   corr(dur, scanned) {cc:.2f}; groups finished by 25/50/75/90 % of the span: "
          + ", ".join(f"{v:.3f}" for v in q), flush=True)
    if has2:
        cyc = b2[:, 0] + b2[:, 1] + b2[:, 2]
        sc = np.maximum(scan, 1)
        print(f"   cycles per scanned leaf (median): wait {np.median(b2[:, 0] / sc):.0f}, scan {np.median(b2[:, 1] / sc):.0f}; "
              f"box tests per block {np.median(b2[:, 2] / np.maximum(b2[:, 3], 1)):.0f} over {np.median(b2[:, 3]):.0f} blocks; "
              f"share of the three in wait / scan / box (median) {np.median(b2[:, 0] / np.maximum(cyc, 1)):.2f} / "
              f"{np.median(b2[:, 1] / np.maximum(cyc, 1)):.2f} / {np.median(b2[:, 2] / np.maximum(cyc, 1)):.2f}; "
              f"their cycles per us of the group (median) {np.median(cyc / np.maximum(dur, 1e-3)):.0f}", flush=True)
        for g in order[:4]:
            print(f"      slow group {g}: wait {b2[g, 0]:.0f} scan {b2[g, 1]:.0f} box {b2[g, 2]:.0f} cycles over "
                  f"{b2[g, 3]:.0f} blocks, {scan[g]} leaves, {dur[g]:.1f} us", flush=True)
    # per-scan-count cost: us per leaf scanned (median of groups with >= 8 leaves)
    m = scan >= 8
    if m.any():
        print(f"   us per scanned leaf (median, groups >= 8 leaves): {np.median(dur[m] / scan[m]):.3f}; "
              f"total leaves scanned {scan.sum()}", flush=True)
c.close()
