"""bench.py's batched leg on its own (argv[1] == "bare") or after the
headline's setup (argv[1] == "prelude": the cfg 3 problem, its ctx and 20
aligns, kept alive), to find what slows the leg inside bench.py
(diagnostics, used via gpurun)."""
import os
import sys
import types

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402

keep = []
if sys.argv[1].startswith("prelude"):
    prob = bench.build_problem()
    sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
    kcov = bench.keyframe_covariances(lambda: P.Context(0), prob["keyframes"], k=10)
    ctx = P.Context(0)
    ctx.set_params(P.default_params(k_correspondences=10))
    ctx.set_source(prob["source"])
    ctx.compute_covariances(P.SOURCE)
    ctx.set_params(P.default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32,
                                    transformation_epsilon=0.01))
    ctx.set_target(sub)
    ctx.set_covariances(P.TARGET, np.ascontiguousarray(kcov[prob["subset"]]))
    for _ in range(20):
        ctx.align(prob["guess"].astype(np.float32))
    ctx.synchronize()
    if sys.argv[1] == "prelude_closed":   # as bench.py does before its legs
        ctx.close()
    else:
        keep.append(ctx)
if sys.argv[1] == "churn":   # ctxs made and destroyed, no work
    for _ in range(10):
        P.Context(0).close()
args = types.SimpleNamespace(batch_frames=1000, batch_streams=4)
r = bench.batched_leg(None, 0, 1, 0, args)
print(sys.argv[1], r["ms_per_pair"], r["ms_per_pair_morton_tie_order"], flush=True)
