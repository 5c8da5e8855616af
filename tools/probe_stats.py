"""Developer probe: per-wave search statistics of the linearize kernel."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic_direct_lidar_odometry_amd import scene, Context, default_params, SOURCE, TARGET  # noqa
from oracle import oracle as O  # noqa


def summarize(tag, st_all):
    b = st_all[st_all[:, 7] == 2]
    if len(b):
        cyc = b[:, 4].astype(np.float64)
        print(f"[{tag} phase B] waves {len(b)} deferred {(b[:,6]&0xffff).sum()} rounds mean {b[:,5].mean():.2f} max {b[:,5].max()}")
        for i, name in enumerate(["blocks", "cand", "listed", "batches"]):
            v = b[:, i]
            print(f"  {name:6s} mean {v.mean():8.1f} p90 {np.percentile(v,90):6.0f} p99 {np.percentile(v,99):6.0f} max {v.max():6d}")
        print(f"  cycles mean {cyc.mean():.0f} p90 {np.percentile(cyc,90):.0f} max {cyc.max():.0f}")
        w = np.argsort(-cyc)[:3]
        for t in w:
            print(f"   worst B wave: n {b[t,6]&0xffff} rounds {b[t,5]} blocks {b[t,0]} cand {b[t,1]} listed {b[t,2]} batches {b[t,3]} splits {b[t,6]>>16} cycles {b[t,4]}")
    st = st_all[(st_all[:, 7] & 0xffff) == 1]
    pro = (st[:, 5] & 0xffff).astype(float); scn = (st[:, 5] >> 16).astype(float) * 16; blk = (st[:, 7] >> 16).astype(float) * 16
    print(f"[{tag}] phase-A cycles: prologue mean {pro.mean():.0f}, flush_blocks mean {blk.mean():.0f}, flush_scan mean {scn.mean():.0f}, total mean {st[:,4].mean():.0f}")
    print(f"[{tag}] groups {len(st)}")
    for i, name in enumerate(["blocks", "cand", "listed", "batches"]):
        v = st[:, i]
        print(f"  {name:6s} mean {v.mean():8.1f} p50 {np.percentile(v,50):6.0f} p90 {np.percentile(v,90):6.0f} p99 {np.percentile(v,99):6.0f} max {v.max():6d} sum {v.sum()}")
    cyc = st[:, 4].astype(np.float64); mcyc = np.zeros(len(st))
    print(f"  search cycles mean {cyc.mean():.0f} p50 {np.percentile(cyc,50):.0f} p90 {np.percentile(cyc,90):.0f} max {cyc.max():.0f}; collect-phase cycles mean {mcyc.mean():.0f} max {mcyc.max():.0f}")
    print(f"  cycles per scanned leaf {cyc.sum()/max(1,st[:,3].sum()):.0f}; corr(scan, cycles) {np.corrcoef(st[:,3], cyc)[0,1]:.2f} corr(box, cycles) {np.corrcoef(st[:,1], cyc)[0,1]:.2f}")
    print(f"  deferred lanes mean {(st[:,6]&0xffff).mean():.2f} total {(st[:,6]&0xffff).sum()}; splits mean {(st[:,6]>>16).mean():.3f} max {(st[:,6]>>16).max()}")
    top = np.argsort(-st[:, 3])[:5]
    for t in top:
        print(f"   worst group {t}: scan {st[t,3]} exact {st[t,2]} box {st[t,1]} cycles {st[t,4]}")


def main():
    src, tgt, T = scene.s2s_pair(64, 2048, 1)
    ctx = Context(0)
    ctx.set_params(default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32, transformation_epsilon=5e-4))
    ctx.set_target(tgt); ctx.set_source(src)
    ctx.debug_stats(True)
    ctx.linearize(np.eye(4))
    summarize("S2S iter0", ctx.debug_stats(True, read=True))
    ctx.align()
    summarize("S2S last iter", ctx.debug_stats(True, read=True))

    prob = scene.s2m_problem(64, 2048, 4, 500000, 3)
    sub = np.concatenate(prob["keyframes"])[prob["subset"]]
    c2 = Context(0)
    c2.set_params(default_params(k_correspondences=10, max_correspondence_distance=2.0, max_iterations=32, transformation_epsilon=0.01))
    c2.set_target(sub); c2.set_source(prob["source"])
    c2.debug_stats(True)
    c2.linearize(prob["guess"].astype(np.float64))
    summarize("S2M iter0", c2.debug_stats(True, read=True))
    c2.align(prob["guess"])
    summarize("S2M last iter", c2.debug_stats(True, read=True))


if __name__ == "__main__":
    main()
