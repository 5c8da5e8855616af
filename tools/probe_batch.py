"""Developer probe: cfg5 frame-parallel S2S throughput vs streams, and a per-stage split of one pair."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import scene, SOURCE

frames, _ = scene.sequence(64, 2048, 41, 20)
p = P.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32, transformation_epsilon=0.01)
P.s2s_batch(frames[:9], p, nstreams=4)
for ns in (1, 2, 4, 8):
    t = time.perf_counter(); P.s2s_batch(frames, p, nstreams=ns); dt = time.perf_counter() - t
    print(f"streams {ns}: {1e3 * dt / 40:.3f} ms/pair")
c = P.Context(0); c.set_params(p); c.set_target(frames[0]); c.compute_covariances(1); c.synchronize()
for rep in range(3):
    t0 = time.perf_counter(); c.set_source(frames[1]); c.synchronize(); t1 = time.perf_counter()
    c.compute_covariances(SOURCE); c.synchronize(); t2 = time.perf_counter()
    out, r = c.align(); t3 = time.perf_counter()
    print(f"set_source {1e3*(t1-t0):.3f} ms, covariances {1e3*(t2-t1):.3f} ms, align {1e3*(t3-t2):.3f} ms ({r.iterations_run} it)")
