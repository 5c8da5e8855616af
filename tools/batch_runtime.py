"""Which HIP runtime the library binds to, and the frame-parallel S2S speed
under it: argv[1] == "torch" imports torch (its bundled libamdhip64) before
the library, "lib" loads the library first (diagnostics, used via gpurun)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if sys.argv[1] == "torch":
    import torch  # noqa: F401
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import scene  # noqa: E402

P.load()
libs = sorted({ln.split()[-1] for ln in open("/proc/self/maps") if "amdhip64" in ln or "hsa-runtime" in ln})
print(sys.argv[1], "runtime libs:", libs, flush=True)
frames = scene.loop_sequence(64, 2048, 0, 1000, device=0)[0]
keep = None
if len(sys.argv) > 2:   # argv[2] == "ctx": one more ctx (2 streams) alive during the batch, as in bench.py
    keep = P.Context(0)
    keep.set_source(frames[0])
    keep.compute_covariances(P.SOURCE)
c = P.Context(0)
for f in frames:
    c.set_source(f)
c.close()
params = P.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32,
                          transformation_epsilon=0.01)
P.s2s_batch(frames[:9], params, device=0, nstreams=4)
for ex in ("1", "0"):
    os.environ["DDLO_TIE_EXACT"] = ex
    t0 = time.perf_counter()
    P.s2s_batch(frames, params, device=0, nstreams=4)
    print(f"{' '.join(sys.argv[1:])} tie_exact {ex}: {1e3 * (time.perf_counter() - t0) / 999:.4f} ms/pair", flush=True)
