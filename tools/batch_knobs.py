"""Frame-parallel S2S (400 frames) under the lazy tie search's knobs: partial
tree levels and worker streams, nanoflann vs Morton order (diagnostics, used
via gpurun).  The env knobs are read at ctx creation."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import scene  # noqa: E402

frames = scene.loop_sequence(64, 2048, 0, 400, device=0)[0]
for f in frames:
    torch.from_numpy(f).to("cuda:0")
torch.cuda.synchronize()
params = P.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32,
                          transformation_epsilon=0.01)
P.s2s_batch(frames[:9], params, device=0, nstreams=4)


def run(tag, ns, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    best = 1e9
    for _ in range(2):
        t0 = time.perf_counter()
        P.s2s_batch(frames, params, device=0, nstreams=ns)
        best = min(best, time.perf_counter() - t0)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    print(f"{tag:40s} streams {ns}: {1e3 * best / (len(frames) - 1):.4f} ms/pair", flush=True)


for ns in (3, 6):
    run("morton", ns, {"DDLO_TIE_EXACT": "0"})
    for lv in (2, 3, 5, 7):
        run(f"nanoflann lazy L={lv}", ns, {"DDLO_TIE_EXACT": "1", "DDLO_TIE_PARTIAL_LEVELS": str(lv)})
    run("nanoflann whole tree", ns, {"DDLO_TIE_EXACT": "1", "DDLO_TIE_LAZY": "0"})
