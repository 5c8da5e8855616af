"""Developer probe: verified-reuse pass rate per outer iteration (cfg3 S2M LM, cfg2 S2S GN)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic_direct_lidar_odometry_amd import scene, Context, default_params, SOURCE, TARGET, GAUSS_NEWTON  # noqa


def run(c, n, mk, guess, iters, label):
    for it in iters:
        c.set_params(mk(it))
        c.debug_stats(True)
        _, r = c.align(guess)
        st = c.debug_stats(True, read=True)
        st = st[: (n + 15) // 16]
        npass = (st[:, 6] >> 8) & 0xff
        tasks = st[:, 2] & 0xffff
        print(f"{label} iter {it-1}: pass {npass.sum()}/{n} ({100.0*npass.sum()/n:.1f}%), groups all-pass "
              f"{(npass == 16).sum()}/{len(st)}, tasks {tasks.sum()}, blocks {st[:,0].sum()}")
    c.debug_stats(False)


prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
c = Context(0)
c.set_params(default_params(k_correspondences=10))
c.set_target(sub); c.set_source(prob["source"])
c.compute_covariances(SOURCE); c.compute_covariances(TARGET)
n = len(prob["source"])
run(c, n, lambda it: default_params(k_correspondences=10, max_correspondence_distance=2.0, max_iterations=it,
                                    transformation_epsilon=1e-9, rotation_epsilon=1e-9),
    prob["guess"].astype(np.float32), (1, 2, 3, 4, 5), "cfg3")
src, tgt, _ = scene.s2s_pair(64, 2048, 2)
c2 = Context(0)
c2.set_params(default_params(k_correspondences=10))
c2.set_target(tgt); c2.set_source(src)
c2.compute_covariances(SOURCE); c2.compute_covariances(TARGET)
run(c2, len(src), lambda it: default_params(k_correspondences=10, max_correspondence_distance=1.0, optimizer=GAUSS_NEWTON,
                                            fixed_iterations=it, max_iterations=it), None, (1, 2, 3, 4, 6, 10, 20), "cfg2")
