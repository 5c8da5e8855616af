"""Frame-parallel S2S over cfg 5's 1000 frames: worker streams vs pairs/s in
both tie orders (diagnostics, used via gpurun)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import scene  # noqa: E402

frames = scene.loop_sequence(64, 2048, 0, 1000, device=0)[0]
for f in frames:
    torch.from_numpy(f).to("cuda:0")
torch.cuda.synchronize()
params = P.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32,
                          transformation_epsilon=0.01)
P.s2s_batch(frames[:17], params, device=0, nstreams=8)
for ns in [int(a) for a in sys.argv[1:]] or (3, 4, 6, 8):
    for ex in ("1", "0"):
        os.environ["DDLO_TIE_EXACT"] = ex
        t0 = time.perf_counter()
        P.s2s_batch(frames, params, device=0, nstreams=ns)
        el = time.perf_counter() - t0
        print(f"streams {ns} tie_exact {ex}: {1e3 * el / (len(frames) - 1):.4f} ms/pair", flush=True)
