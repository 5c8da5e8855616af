"""Developer probe: per-wave search counters of the cfg3 S2M search, per outer iteration."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic_direct_lidar_odometry_amd import scene, Context, default_params, SOURCE, TARGET  # noqa

prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
sub = np.ascontiguousarray(np.concatenate(prob["keyframes"])[prob["subset"]])
c = Context(0)
c.set_params(default_params(k_correspondences=10))
c.set_target(sub); c.set_source(prob["source"])
c.compute_covariances(SOURCE); c.compute_covariances(TARGET)
guess = prob["guess"].astype(np.float32)
dump = {}
for it in (1, 2, 3):
    c.set_params(default_params(k_correspondences=10, max_correspondence_distance=2.0, max_iterations=it,
                                transformation_epsilon=1e-9))
    c.debug_stats(True)
    c.align(guess)
    st = c.debug_stats(True, read=True)
    corr, sqd = c.correspondences()
    dump[f"st{it-1}"] = st.copy(); dump[f"sqd{it-1}"] = sqd; dump[f"pose{it-1}"] = c.align(guess)[0] if False else 0
    st = st[st[:, 7] == 1]
    cyc = st[:, 4].astype(np.float64); col = st[:, 5].astype(np.float64)
    print(f"iter {it-1}: groups {len(st)}  blocks mean {st[:,0].mean():.1f} p90 {np.percentile(st[:,0],90):.0f}"
          f"  exact(leaves listed) mean {st[:,2].mean():.1f} p90 {np.percentile(st[:,2],90):.0f}"
          f"  scanned mean {st[:,3].mean():.1f} p90 {np.percentile(st[:,3],90):.0f} max {st[:,3].max()}"
          f"  splits mean {(st[:,6]>>16).mean():.2f} seeded-lanes mean {(st[:,6]&0xffff).mean():.2f}")
    pro = (st[:, 1] & 0xffff).astype(float) * 16; trv = (st[:, 1] >> 16).astype(float) * 16
    print(f"   phases (mean cycles): prologue {pro.mean():.0f}  traverse-end {trv.mean():.0f}  collect-end {col.mean():.0f}  total {cyc.mean():.0f}")
    print(f"   cycles mean {cyc.mean():.0f} p50 {np.percentile(cyc,50):.0f} p90 {np.percentile(cyc,90):.0f} max {cyc.max():.0f};"
          f" collect-phase mean {col.mean():.0f}; corr(scan,cyc) {np.corrcoef(st[:,3],cyc)[0,1]:.2f} corr(blocks,cyc) {np.corrcoef(st[:,0],cyc)[0,1]:.2f}")
c.debug_stats(False)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/probe_cfg3.npz", **dump)
# timing per iteration (profiling mode)
c.set_params(default_params(k_correspondences=10, max_correspondence_distance=2.0, max_iterations=32, transformation_epsilon=0.01))
c.set_profiling(True)
for _ in range(3):
    out, res = c.align(guess)
print("linearize ms total", res.linearize_ms, "iters", res.iterations_run)
