"""How often do exact distance ties occur on the cfg 5 workload?  (decides
whether nanoflann's tree should be built eagerly or only when a tie shows up)

Per frame of the 1000-frame plaza loop (GPU ray caster): the k = 10
covariance pass of the raw scan (tied queries, DDLO_TIE_DEBUG), then the
odometry driver's S2S / S2M correspondence ties (gicp_result.ties_resolved,
tie_reruns).

    python tools/probe_cov_ties.py [--frames 200]
"""
import argparse
import os
import sys

os.environ.setdefault("DDLO_TIE_DEBUG", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dynamic_direct_lidar_odometry_amd as P  # noqa: E402
from dynamic_direct_lidar_odometry_amd import SOURCE, scene  # noqa: E402
from dynamic_direct_lidar_odometry_amd import odometry as OD  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    a = ap.parse_args()
    frames = scene.loop_sequence(64, 2048, 0, a.frames, device=0)[0]
    c = P.Context(0)
    c.set_params(P.default_params(k_correspondences=10))
    for f in frames[:20]:
        c.set_source(f)
        c.compute_covariances(SOURCE)   # stderr: [ties] n k tied
    c.close()
    odo = OD.Odometry(0)
    s2s = s2m = reruns = 0
    for i, f in enumerate(frames):
        r = odo.process(f)
        s2s += r.s2s.ties_resolved
        s2m += r.s2m.ties_resolved
        reruns += r.s2s.tie_reruns + r.s2m.tie_reruns
        if r.s2s.ties_resolved or r.s2m.ties_resolved or r.s2s.tie_reruns or r.s2m.tie_reruns:
            print(f"frame {i}: s2s ties {r.s2s.ties_resolved} s2m ties {r.s2m.ties_resolved} "
                  f"reruns {r.s2s.tie_reruns + r.s2m.tie_reruns}", flush=True)
    odo.close()
    print(f"odometry over {len(frames)} frames: correspondence ties s2s {s2s} s2m {s2m}, align re-runs {reruns}")


if __name__ == "__main__":
    main()
