"""Host-page state vs. the frame-parallel S2S leg: the same 400 frames as
fresh host copies (never DMA-read), as pages the GPU has read once, and
after a torch .to(device) pre-read -- nanoflann vs Morton tie order
(diagnostics, used via gpurun)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import scene  # noqa: E402

frames = scene.loop_sequence(64, 2048, 0, 400, device=0)[0]
params = P.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32,
                          transformation_epsilon=0.01)
P.s2s_batch(frames[:9], params, device=0, nstreams=4)


def run(tag, fr, exact):
    os.environ["DDLO_TIE_EXACT"] = exact
    t0 = time.perf_counter()
    P.s2s_batch(fr, params, device=0, nstreams=4)
    el = time.perf_counter() - t0
    print(f"{tag}: {1e3 * el / (len(fr) - 1):.4f} ms/pair", flush=True)


f1 = [np.array(f, copy=True) for f in frames]
run("nanoflann cold", f1, "1")
run("nanoflann warm", f1, "1")
run("morton warm", f1, "0")
f3 = [np.array(f, copy=True) for f in frames]
run("morton cold", f3, "0")
run("morton warm", f3, "0")
f2 = [np.array(f, copy=True) for f in frames]
for f in f2:
    torch.from_numpy(f).to("cuda:0")
torch.cuda.synchronize()
run("nanoflann after torch pre-read", f2, "1")
run("morton after torch pre-read", f2, "0")
