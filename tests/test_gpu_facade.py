"""The C++ NanoGICP facade (include/nano_gicp/nano_gicp.hpp) replaying
OdomNode's per-scan S2S -> S2M call sequence (odom.cc:487-488,518-532,
745-793,921-939) on a synthetic drive, compared frame by frame with the
oracle driven through the same sequence in Python."""
import os
import struct
import subprocess

import numpy as np
import pytest

from dynamic_direct_lidar_odometry_amd import scene
from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "facade_replay")


def _ensure_binary():
    if os.path.exists(BIN):
        return BIN
    lib = os.path.join(ROOT, "dynamic_direct_lidar_odometry_amd", "_lib")
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"), "-o", BIN,
                    os.path.join(ROOT, "tests", "cpp", "facade_replay.cpp"), f"-L{lib}", "-lddlo_gicp",
                    f"-Wl,-rpath,{lib}"], check=True)
    return BIN


def _sequence(nframes=6, rows=16, cols=1024, seed=1042):
    sc = scene.make_scene(seed)
    poses = scene.trajectory(nframes, seed)
    frames = [scene.raycast(sc, P, rows, cols, seed=seed + i) for i, P in enumerate(poses)]
    P0inv = np.linalg.inv(poses[0])
    world0 = [scene.transform(f, P0inv @ P) for f, P in zip(frames, poses)]
    covs = [O.covariances(w, 10) for w in world0]     # per-keyframe covariances (odom.cc:1147-1149)
    allp = np.concatenate(world0)
    allc = np.concatenate(covs)
    sub = np.sort(np.random.default_rng(seed).choice(len(allp), size=min(30000, len(allp)), replace=False))
    return frames, np.ascontiguousarray(allp[sub]), np.ascontiguousarray(allc[sub])


def _write(path, frames, sub, subcov):
    with open(path, "wb") as f:
        f.write(struct.pack("<i", len(frames)))
        for fr in frames:
            f.write(struct.pack("<i", len(fr)))
            f.write(np.ascontiguousarray(fr, np.float32).tobytes())
        f.write(struct.pack("<i", len(sub)))
        f.write(np.ascontiguousarray(sub, np.float32).tobytes())
        f.write(np.ascontiguousarray(subcov, np.float64).tobytes())


def _oracle_replay(frames, sub, subcov):
    s2s_p = O.default_params(k_correspondences=10, max_correspondence_distance=1.0, max_iterations=32,
                             transformation_epsilon=0.01)
    s2m_p = O.default_params(k_correspondences=20, max_correspondence_distance=2.0, max_iterations=32,
                             transformation_epsilon=0.01)
    out = []
    T_prev = np.eye(4, dtype=np.float32)
    for i in range(1, len(frames)):
        s2s = O.Gicp(frames[i], frames[i - 1], s2s_p)
        s2s.compute_covariances(0)
        s2s.compute_covariances(1)
        T_s2s, _ = s2s.align()
        guess = np.zeros((4, 4), np.float32)            # float accumulation in the facade driver's order
        for r in range(4):
            for c in range(4):
                s = np.float32(0)
                for k in range(4):
                    s = np.float32(s + np.float32(T_prev[r, k] * T_s2s[k, c]))
                guess[r, c] = s
        s2m = O.Gicp(frames[i], sub, s2m_p)
        s2m.set_covariances(0, s2s.get_covariances(0))
        s2m.set_covariances(1, subcov)
        T, _ = s2m.align(guess)
        out.append((T_s2s, T))
        T_prev = T
    return out


def test_facade_replay_matches_oracle(tmp_path):
    frames, sub, subcov = _sequence()
    path = tmp_path / "frames.bin"
    _write(path, frames, sub, subcov)
    r = subprocess.run([_ensure_binary(), str(path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("frame")]
    ref = _oracle_replay(frames, sub, subcov)
    assert len(lines) == len(ref) == len(frames) - 1
    for line, (T_s2s, T) in zip(lines, ref):
        tok = line.split()
        s2s = np.array(tok[3:19], np.float64).reshape(4, 4)
        s2m = np.array(tok[20:36], np.float64).reshape(4, 4)
        assert int(tok[37]) == len(frames[0]) or int(tok[37]) > 0
        np.testing.assert_allclose(s2s, T_s2s, atol=1e-5)
        np.testing.assert_allclose(s2m, T, atol=1e-5)
