"""One frame-parallel S2S batch (200 frames, 4 streams) in the tie order given
by argv[1] ("1" nanoflann, "0" Morton), for a rocprofv3 kernel trace
(diagnostics, used via gpurun)."""
import os
import sys
import time

os.environ["DDLO_TIE_EXACT"] = sys.argv[1]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import scene  # noqa: E402

frames = scene.loop_sequence(64, 2048, 0, 201, device=0)[0]
for f in frames:
    torch.from_numpy(f).to("cuda:0")
torch.cuda.synchronize()
params = P.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32,
                          transformation_epsilon=0.01)
P.s2s_batch(frames[:9], params, device=0, nstreams=4)
t0 = time.perf_counter()
P.s2s_batch(frames, params, device=0, nstreams=4)
print(f"tie_exact={sys.argv[1]}: {1e3 * (time.perf_counter() - t0) / 200:.4f} ms/pair", flush=True)
