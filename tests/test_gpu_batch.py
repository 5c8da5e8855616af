"""GPU parity of the frame-parallel S2S batch (gicp_s2s_batch, SURVEY.md
§8(e) cfg 5) against (1) the same pairs aligned one by one through a single
ctx chained exactly as OdomNode does (odom.cc:754-768) — bit-identical
poses, iteration counts and flags, since every pair runs the same kernels
on the same inputs — and (2) the CPU oracle on a few pairs (poses within
1e-5, the cfg-2 tolerance of DESIGN.md §2)."""
import numpy as np
import pytest

import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import scene
from oracle import oracle as O

pytestmark = pytest.mark.gpu

S2S = dict(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32, transformation_epsilon=5e-4)


@pytest.fixture(scope="module")
def frames():
    f, _ = scene.sequence(64, 512, 9, 5)
    return f


def sequential(frames, params):
    c = P.Context(0)
    c.set_params(params)
    c.set_target(frames[0])
    poses, res = [np.eye(4, dtype=np.float32)], [None]
    for t in range(1, len(frames)):
        c.set_source(frames[t])
        out, r = c.align()
        poses.append(out)
        res.append(r)
        c.swap_source_target()
    c.close()
    return np.stack(poses), res


@pytest.mark.parametrize("nstreams", [1, 3, 8])
def test_batch_equals_chained_single_ctx(frames, nstreams):
    p = P.default_params(**S2S)
    bp, br = P.s2s_batch(frames, p, nstreams=nstreams)
    sp, sr = sequential(frames, p)
    assert np.array_equal(bp[0], np.eye(4, dtype=np.float32))
    assert np.array_equal(bp, sp)
    for t in range(1, len(frames)):
        assert br[t].iterations_run == sr[t].iterations_run
        assert br[t].converged == sr[t].converged and br[t].lm_failed == sr[t].lm_failed
        assert br[t].num_correspondences == sr[t].num_correspondences


def test_batch_matches_oracle(frames):
    p = P.default_params(**S2S)
    bp, br = P.s2s_batch(frames, p, nstreams=4)
    for t in (1, 5, 6):   # 5 -> 6 is the repeated turn-around frame (zero motion)
        g = O.Gicp(frames[t], frames[t - 1], O.as_params(p))
        op, ores = g.align()
        assert br[t].iterations_run == ores.iterations_run
        assert np.abs(bp[t] - op).max() < 1e-5


def test_batch_single_frame_and_errors(frames):
    p = P.default_params(**S2S)
    out, _ = P.s2s_batch(frames[:1], p)
    assert np.array_equal(out[0], np.eye(4, dtype=np.float32))
    with pytest.raises(P.GicpError):
        P.s2s_batch(frames[:3], p, nstreams=0)
    with pytest.raises(P.GicpError):
        P.s2s_batch([frames[0], np.zeros((0, 3), np.float32)], p)


def test_batch_nonfinite_frame_leaves_pool_clean(frames):
    """A frame with a NaN fails the batch with GICP_ENONFINITE (the reference
    would feed NaNs to its kd-tree); the buffers its worker had started
    filling (index, the early nanoflann tree on the second stream) go back to
    the device pool only after that stream has drained, so a batch run right
    after, on the same pool, is bit-identical to the chained single-ctx run."""
    p = P.default_params(**S2S)
    bad = [f.copy() for f in frames]
    bad[3][17] = np.nan
    with pytest.raises(P.GicpError) as e:
        P.s2s_batch(bad, p, nstreams=3)
    assert e.value.status == 8
    bp, _ = P.s2s_batch(frames, p, nstreams=3)
    sp, _ = sequential(frames, p)
    assert np.array_equal(bp, sp)

def test_batch_gated_tree_equals_chained_single_ctx():
    """cfg 5's 64x2048 frames, about half of whose scans have tied k = 10
    neighbourhoods (tools/gpu_tiecount.sh): the batch workers build the
    partial tree after the covariance kernel, gated on the tie count, on their
    own stream; the single ctx builds it beside the kernel on its second
    stream. Same covariances, so bit-identical poses."""
    fr, _ = scene.loop_sequence(64, 2048, 0, 9, device=0)
    p = P.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32,
                         transformation_epsilon=0.01)
    bp, br = P.s2s_batch(fr, p, nstreams=3)
    sp, sr = sequential(fr, p)
    assert np.array_equal(bp, sp)
    for t in range(1, len(fr)):
        assert br[t].iterations_run == sr[t].iterations_run
        assert br[t].num_correspondences == sr[t].num_correspondences
