"""Wave timeline of the fused-lookup moment kernel (cfg3 headline aligns) from a -DDDLO_MOM_PROF build:
every wavefront stores six s_memrealtime stamps (100 MHz) into a device buffer (no printf), read back
after each align through ddlo_dev_mom_prof.
    DDLO_GICP_LIB=.../_lib/momprof/libddlo_gicp.so python tools/mom_timeline.py [aligns]
Phases: state (job / state loads), lookup (cell list scan), contrib (match operands + moment terms),
treduce (wavefront reduction), tail (block reduction + slab store, incl. waiting for the block)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import SOURCE, TARGET  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
prob = bench.build_problem()
sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
tcov = np.ascontiguousarray(bench.keyframe_covariances(lambda: P.Context(0), prob["keyframes"])[prob["subset"]])
c = P.Context(0)
c.set_params(P.default_params(k_correspondences=10))
c.set_source(prob["source"])
c.compute_covariances(SOURCE)
c.set_params(P.default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32,
                              transformation_epsilon=0.01))
c.set_target_grid(P.GRID_ON)
c.set_target(sub)
c.set_covariances(TARGET, tcov)
g = prob["guess"].astype(np.float32)
L = P.load()
buf = np.zeros((8, 2048, 6), np.uint64)
nw = (len(prob["source"]) + 63) // 64
launches = []
for a in range(n + 3):
    _, r = c.align(g)
    c.synchronize()
    assert L.ddlo_dev_mom_prof(buf.ctypes.data_as(C.c_void_p)) == 0
    if a >= 3:
        for it in range(r.iterations_run):
            launches.append(buf[it, :nw].astype(np.int64).copy())
c.close()
us = 1 / 100.0
names = ["state", "lookup", "contrib", "treduce", "tail"]
ends, med, p99, slowest = [], [], [], []
for t in launches:
    T0 = t[:, 0].min()
    end = (t[:, 5] - T0) * us
    ph = np.diff(t, axis=1) * us
    ends.append([np.median(end), np.percentile(end, 99), end.max()])
    med.append(np.median(ph, axis=0))
    p99.append(np.percentile(ph, 99, axis=0))
    w = np.argsort(t[:, 4] - t[:, 0])[-3:]   # longest bodies (before the block reduction)
    for x in w:
        slowest.append([x, (t[x, 4] - T0) * us, *ph[x]])
ends, med, p99 = np.array(ends), np.array(med), np.array(p99)
print(f"{len(launches)} launches x {nw} waves; medians over launches (us)")
print("  wave end: p50 %.2f  p99 %.2f  max %.2f" % tuple(np.median(ends, axis=0)))
print("  phase p50:", dict(zip(names, np.round(np.median(med, axis=0), 2))))
print("  phase p99:", dict(zip(names, np.round(np.median(p99, axis=0), 2))))
s = np.array(slowest)
print("longest wave bodies (wave, body end, state, lookup, contrib, treduce, tail):")
for x in s[np.argsort(s[:, 1])][-10:]:
    print("  %5d " % x[0] + " ".join(f"{v:7.2f}" for v in x[1:]))
ids, cnt = np.unique(s[:, 0].astype(int), return_counts=True)
print("waves among the 3 longest bodies most often:", sorted(zip(cnt, ids), reverse=True)[:10])
