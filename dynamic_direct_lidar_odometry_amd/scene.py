"""Deterministic synthetic "kantplatz-shaped" plaza scenes for the GICP hot path.

The reference ships no datasets or fixtures; its authors replay
external rosbags (``DDLO/launch/play_kantplatz_data.launch:8-17``).  This module
ray-casts a ring LiDAR inside an urban plaza so that every BASELINE.json config
can be produced on any box without network access:

* ground plane z = 0, building facades enclosing a 60 m x 40 m square (50 m
  tall, so every ray of a +/-45 deg ring returns), facade pilasters and
  recesses, lamp poles (vertical cylinders), benches and ~20 pedestrian boxes;
* sensor 1.5 m above ground, 64 rows over +/-22.5 deg or 128 rows over
  +/-45 deg, 1024/2048 columns, range noise N(0, 0.01 m), ranges 0.5-80 m,
  no-return pixels dropped (GICP inputs must be finite, ``odom.cc:469-475``);
* trajectory 1.0 m/s at 10 Hz with a gentle yaw rate (<= 10 deg/s).

Seeds follow SURVEY.md §8(d): ``1000 + config id (+ frame index)``.  All
randomness goes through ``numpy.random.default_rng`` so the clouds are
bit-identical across runs on one platform.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

PLAZA_X = 30.0   # half extent of the square (m)
PLAZA_Y = 20.0
FACADE_H = 50.0
SENSOR_Z = 1.5


@dataclass
class Scene:
    boxes_lo: np.ndarray      # (B,3) axis-aligned solid boxes (pilasters, benches, kiosks)
    boxes_hi: np.ndarray
    poles: np.ndarray         # (P,4) cx, cy, radius, height
    peds_lo: np.ndarray       # (Q,3) pedestrian boxes at t = 0
    peds_hi: np.ndarray
    peds_vel: np.ndarray      # (Q,2) xy velocity (m/s); zero for static ones


# cfg 5's closed loop (loop_trajectory): an ellipse inside the square
# (~110 m around), driven at 1.5 m/s, so a 1000-frame (150 m) sequence stays
# in the plaza and revisits its first keyframes; range noise 3 cm (a
# 64-beam sensor's spec), so scan-to-scan leaves work for scan-to-map
LOOP_X, LOOP_Y = 22.0, 12.0
LOOP_STEP = 0.15
LOOP_NOISE = 0.03


def _near_loop(x, y, margin):
    """|distance| from the loop ellipse below ~margin (radial measure)."""
    r = math.sqrt((x / LOOP_X) ** 2 + (y / LOOP_Y) ** 2)
    return abs(r - 1.0) * min(LOOP_X, LOOP_Y) < margin


def make_scene(seed: int = 1000, n_peds: int = 20, moving: bool = False, loop: bool = False) -> Scene:
    """loop = True: objects keep 2.5 m (pedestrians 1.5 m) clear of the cfg 5 loop path (loop_trajectory)."""
    rng = np.random.default_rng(seed)
    lo, hi = [], []
    # facade pilasters: shallow boxes attached to the four walls, irregular spacing
    for wall in range(4):
        n = 14 if wall < 2 else 10
        span = PLAZA_Y if wall < 2 else PLAZA_X
        pos = np.sort(rng.uniform(-span + 1.0, span - 1.0, n))
        for p in pos:
            w = rng.uniform(0.4, 1.2)
            d = rng.uniform(0.2, 0.8)
            h = rng.uniform(6.0, FACADE_H)
            if wall == 0:   # x = +PLAZA_X wall
                lo.append([PLAZA_X - d, p - w, 0.0]); hi.append([PLAZA_X + 0.1, p + w, h])
            elif wall == 1:  # x = -PLAZA_X
                lo.append([-PLAZA_X - 0.1, p - w, 0.0]); hi.append([-PLAZA_X + d, p + w, h])
            elif wall == 2:  # y = +PLAZA_Y
                lo.append([p - w, PLAZA_Y - d, 0.0]); hi.append([p + w, PLAZA_Y + 0.1, h])
            else:            # y = -PLAZA_Y
                lo.append([p - w, -PLAZA_Y - 0.1, 0.0]); hi.append([p + w, -PLAZA_Y + d, h])
    # balconies / cornices: horizontal slabs that break facade symmetry in z
    for _ in range(16):
        wall = rng.integers(0, 4)
        z = rng.uniform(3.0, 20.0)
        span = PLAZA_Y if wall < 2 else PLAZA_X
        c = rng.uniform(-span + 3, span - 3)
        w = rng.uniform(1.0, 4.0)
        d = rng.uniform(0.6, 1.5)
        if wall == 0:
            lo.append([PLAZA_X - d, c - w, z]); hi.append([PLAZA_X, c + w, z + 0.3])
        elif wall == 1:
            lo.append([-PLAZA_X, c - w, z]); hi.append([-PLAZA_X + d, c + w, z + 0.3])
        elif wall == 2:
            lo.append([c - w, PLAZA_Y - d, z]); hi.append([c + w, PLAZA_Y, z + 0.3])
        else:
            lo.append([c - w, -PLAZA_Y, z]); hi.append([c + w, -PLAZA_Y + d, z + 0.3])
    # benches and kiosks inside the square
    for _ in range(12):
        cx, cy = rng.uniform(-PLAZA_X + 4, PLAZA_X - 4), rng.uniform(-PLAZA_Y + 4, PLAZA_Y - 4)
        while loop and _near_loop(cx, cy, 4.5):
            cx, cy = rng.uniform(-PLAZA_X + 4, PLAZA_X - 4), rng.uniform(-PLAZA_Y + 4, PLAZA_Y - 4)
        if abs(cy) < 2.5 and -15 < cx < 15 and not loop:   # keep the driving corridor free
            cy += 5.0 * np.sign(cy if cy != 0 else 1.0)
        ang = rng.uniform(0, math.pi)
        L = rng.uniform(1.5, 4.0)
        W = rng.uniform(0.5, 2.5)
        H = rng.uniform(0.45, 3.0)
        ex = abs(L * math.cos(ang)) + abs(W * math.sin(ang))
        ey = abs(L * math.sin(ang)) + abs(W * math.cos(ang))
        lo.append([cx - ex / 2, cy - ey / 2, 0.0]); hi.append([cx + ex / 2, cy + ey / 2, H])
    poles = []
    for _ in range(18):
        cx, cy = rng.uniform(-PLAZA_X + 2, PLAZA_X - 2), rng.uniform(-PLAZA_Y + 2, PLAZA_Y - 2)
        while loop and _near_loop(cx, cy, 2.5):
            cx, cy = rng.uniform(-PLAZA_X + 2, PLAZA_X - 2), rng.uniform(-PLAZA_Y + 2, PLAZA_Y - 2)
        if abs(cy) < 2.0 and -15 < cx < 15 and not loop:
            cy += 4.0 * np.sign(cy if cy != 0 else 1.0)
        poles.append([cx, cy, rng.uniform(0.06, 0.25), rng.uniform(3.0, 8.0)])
    plo, phi, pvel = [], [], []
    for _ in range(n_peds):
        cx, cy = rng.uniform(-PLAZA_X + 3, PLAZA_X - 3), rng.uniform(-PLAZA_Y + 3, PLAZA_Y - 3)
        while loop and _near_loop(cx, cy, 1.5):
            cx, cy = rng.uniform(-PLAZA_X + 3, PLAZA_X - 3), rng.uniform(-PLAZA_Y + 3, PLAZA_Y - 3)
        if abs(cy) < 1.5 and -15 < cx < 15 and not loop:
            cy += 3.0 * np.sign(cy if cy != 0 else 1.0)
        w = rng.uniform(0.3, 0.6)
        plo.append([cx - w / 2, cy - w / 2, 0.0]); phi.append([cx + w / 2, cy + w / 2, rng.uniform(1.5, 1.95)])
        if moving:
            a = rng.uniform(0, 2 * math.pi)
            s = rng.uniform(0.5, 1.5)
            pvel.append([s * math.cos(a), s * math.sin(a)])
        else:
            pvel.append([0.0, 0.0])
    return Scene(np.asarray(lo), np.asarray(hi), np.asarray(poles),
                 np.asarray(plo), np.asarray(phi), np.asarray(pvel))


def _ray_box(o, inv, lo, hi, tbest):
    """Slab test of rays (o + t d), inv = 1/d, against one AABB; updates tbest in place."""
    tmin = np.zeros_like(tbest)
    tmax = tbest.copy()
    for a in range(3):
        t1 = (lo[a] - o[a]) * inv[a]
        t2 = (hi[a] - o[a]) * inv[a]
        np.maximum(tmin, np.minimum(t1, t2), out=tmin)
        np.minimum(tmax, np.maximum(t1, t2), out=tmax)
    better = (tmax >= tmin) & (tmin > 1e-6) & (tmin < tbest)
    tbest[better] = tmin[better]


def _ray_cylinder(o, d, cx, cy, r, h, tbest):
    ox, oy = o[0] - cx, o[1] - cy
    a = d[:, 0] ** 2 + d[:, 1] ** 2
    b = 2 * (ox * d[:, 0] + oy * d[:, 1])
    c = ox * ox + oy * oy - r * r
    disc = b * b - 4 * a * c
    ok = (disc >= 0) & (a > 1e-12)
    with np.errstate(invalid="ignore", divide="ignore"):
        t = (-b - np.sqrt(np.where(ok, disc, 0.0))) / (2 * a)
    z = o[2] + t * d[:, 2]
    good = ok & (t > 1e-6) & (z >= 0) & (z <= h) & (t < tbest)
    tbest[good] = t[good]


def lidar_dirs(rows: int, cols: int) -> np.ndarray:
    """Unit ray directions (rows*cols, 3) of a ring LiDAR in the sensor frame (row-major)."""
    vfov = 22.5 if rows <= 64 else 45.0
    elev = np.deg2rad(np.linspace(-vfov, vfov, rows))
    azim = np.deg2rad(np.arange(cols) * (360.0 / cols))
    E, A = np.meshgrid(elev, azim, indexing="ij")
    return np.stack([np.cos(E) * np.cos(A), np.cos(E) * np.sin(A), np.sin(E)], axis=-1).reshape(-1, 3)


def raycast(scene: Scene, pose: np.ndarray, rows: int, cols: int, seed: int, t: float = 0.0,
            organized: bool = False, noise: float = 0.01) -> np.ndarray:
    """Ray-cast one scan from world pose ``pose`` (4x4, world <- sensor).

    Returns float32 points (N,3) in the SENSOR frame, organized row-major with
    no-return pixels dropped; with ``organized`` all rows*cols pixels, NaN for
    no return, top beam first.
    """
    rng = np.random.default_rng(seed)
    dirs_s = lidar_dirs(rows, cols)
    R, o = pose[:3, :3], pose[:3, 3]
    d = dirs_s @ R.T
    tbest = np.full(d.shape[0], np.inf)
    # ground
    with np.errstate(divide="ignore", invalid="ignore"):
        tg = -o[2] / d[:, 2]
    tbest = np.where((d[:, 2] < 0) & (tg > 0), tg, tbest)
    # facades (inside of the square)
    with np.errstate(divide="ignore", invalid="ignore"):
        for axis, ext in ((0, PLAZA_X), (1, PLAZA_Y)):
            tp = (ext - o[axis]) / d[:, axis]
            tn = (-ext - o[axis]) / d[:, axis]
            tw = np.where(d[:, axis] > 0, tp, tn)
            zw = o[2] + tw * d[:, 2]
            ok = (tw > 0) & (zw <= FACADE_H) & (tw < tbest)
            tbest = np.where(ok, tw, tbest)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = [1.0 / np.where(d[:, a] == 0.0, 1e-30, d[:, a]) for a in range(3)]
    for lo, hi in zip(scene.boxes_lo, scene.boxes_hi):
        _ray_box(o, inv, lo, hi, tbest)
    for cx, cy, r, h in scene.poles:
        _ray_cylinder(o, d, cx, cy, r, h, tbest)
    for lo, hi, v in zip(scene.peds_lo, scene.peds_hi, scene.peds_vel):
        shift = np.array([v[0] * t, v[1] * t, 0.0])
        _ray_box(o, inv, lo + shift, hi + shift, tbest)
    rng_noise = rng.normal(0.0, noise, size=tbest.shape)
    r = tbest + rng_noise
    valid = np.isfinite(tbest) & (r >= 0.5) & (r <= 80.0)
    if organized:
        pts = np.where(valid[:, None], dirs_s * np.where(valid, r, 0.0)[:, None], np.nan).astype(np.float32)
        # row 0 = the top beam, the last row = the lowest (the range-image convention of detection.cpp:463)
        return pts.reshape(rows, cols, 3)[::-1].reshape(-1, 3).copy()
    pts = dirs_s[valid] * r[valid, None]
    return pts.astype(np.float32)


def rpy_to_R(roll, pitch, yaw):
    cr, sr, cp, sp, cy, sy = math.cos(roll), math.sin(roll), math.cos(pitch), math.sin(pitch), math.cos(yaw), math.sin(yaw)
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1.0]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    return Rz @ Ry @ Rx


def make_pose(t, rpy=(0.0, 0.0, 0.0)):
    T = np.eye(4)
    T[:3, :3] = rpy_to_R(*rpy)
    T[:3, 3] = t
    return T


def trajectory(n_frames: int, seed: int = 1000) -> list:
    """Ground-truth sensor poses: 1.0 m/s at 10 Hz, slowly varying yaw rate."""
    rng = np.random.default_rng(seed)
    x, y, yaw = -12.0, -1.0, 0.0
    poses = []
    yaw_rate = 0.0
    for _ in range(n_frames):
        poses.append(make_pose([x, y, SENSOR_Z], (0.0, 0.0, yaw)))
        yaw_rate = float(np.clip(yaw_rate + rng.normal(0, 0.5), -10.0, 10.0))  # deg/s
        yaw += math.radians(yaw_rate) * 0.1
        x += 0.1 * math.cos(yaw)
        y += 0.1 * math.sin(yaw)
        if abs(y) > 8.0:       # keep inside the square
            yaw -= 0.05 * np.sign(y)
    return poses


# The S2S perturbation of SURVEY.md §8(d): t = (0.30, -0.20, 0.05) m, yaw 2 deg, roll/pitch 0.5 deg
PERTURB = make_pose([0.30, -0.20, 0.05], (math.radians(0.5), math.radians(0.5), math.radians(2.0)))


def transform(pts: np.ndarray, T: np.ndarray) -> np.ndarray:
    return (pts.astype(np.float64) @ T[:3, :3].T + T[:3, 3]).astype(np.float32)


def s2s_pair(rows: int, cols: int, cfg_id: int):
    """Two scans: target from pose P, source from pose P * PERTURB (guess = I).

    Returns (source, target, T_true) with T_true mapping source-frame points
    into the target frame (what align() should recover).
    """
    scene = make_scene(1000 + cfg_id)
    P = make_pose([-6.0, 2.0, SENSOR_Z], (0.0, 0.0, math.radians(15.0)))
    tgt = raycast(scene, P, rows, cols, seed=1000 + cfg_id)
    Q = P @ PERTURB
    src = raycast(scene, Q, rows, cols, seed=1000 + cfg_id + 1)
    return src, tgt, PERTURB.copy()


def s2m_problem(rows: int, cols: int, n_keyframes: int, submap_size: int, cfg_id: int):
    """Scan vs fused keyframe submap (SURVEY.md §8(d) cfg 3/4).

    Keyframes are scans taken every 10 frames (1 m, ``ddlo.yaml`` threshD) and
    moved into the world frame; the submap is their concatenation truncated to
    ``submap_size`` by a seeded subset.  Returns a dict with the source scan
    (sensor frame), the per-keyframe world clouds, the subset indices, the
    ground-truth pose and the perturbed initial guess.
    """
    seed = 1000 + cfg_id
    scene = make_scene(seed)
    poses = trajectory(10 * n_keyframes + 6, seed)
    kfs = []
    for k in range(n_keyframes):
        P = poses[10 * k]
        kfs.append(transform(raycast(scene, P, rows, cols, seed=seed + 10 * k), P))
    cur = poses[10 * n_keyframes + 5]
    src = raycast(scene, cur, rows, cols, seed=seed + 10 * n_keyframes + 5)
    total = sum(len(k) for k in kfs)
    rng = np.random.default_rng(seed + 7)
    if submap_size < total:
        subset = np.sort(rng.choice(total, size=submap_size, replace=False))
    else:
        subset = np.arange(total)
    guess = cur @ PERTURB
    return {"source": src, "keyframes": kfs, "subset": subset, "T_true": cur, "guess": guess}


def odometry_sequence(rows: int, cols: int, n_frames: int, cfg_id: int = 5, moving: bool = True):
    """Consecutive ray-cast frames along the ground-truth trajectory (forward
    only), with moving pedestrians: the input of the odometry driver (cfg 5's
    S2M chain).  Returns (frames, world poses)."""
    seed = 1000 + cfg_id
    scene = make_scene(seed, moving=moving)
    poses = trajectory(n_frames, seed)
    return [raycast(scene, poses[k], rows, cols, seed=seed + k, t=0.1 * k) for k in range(n_frames)], poses


def sequence(rows: int, cols: int, n_frames: int, n_unique: int, cfg_id: int = 5):
    """Scan sequence for the batched-odometry case (SURVEY.md §8(d) cfg 5):
    ``n_unique`` consecutive ray-cast frames of the plaza with MOVING
    pedestrians (1.0 m/s at 10 Hz), replayed forward and backward
    (0..u-1, u-1..0, 0..) up to ``n_frames`` so that every consecutive pair
    stays a real adjacent-pose pair while only ``n_unique`` frames are cast.
    Returns (frames list of sensor-frame clouds, per-frame world poses)."""
    seed = 1000 + cfg_id
    scene = make_scene(seed, moving=True)
    poses = trajectory(n_unique, seed)
    uniq = [raycast(scene, poses[k], rows, cols, seed=seed + k, t=0.1 * k) for k in range(n_unique)]
    order = []
    k, step = 0, 1
    while len(order) < n_frames:
        order.append(k)
        if not 0 <= k + step < n_unique:
            step = -step
            order.append(k)  # the turn-around frame repeats (a zero-motion pair)
        k += step
    order = order[:n_frames]
    return [uniq[i] for i in order], [poses[i] for i in order]


# ---------------------------------------------------------------------------
# cfg 5 at its named size (BASELINE.json configs[4]: 1000 frames): a closed
# loop, pedestrians bouncing inside the square, frames synthesised by the GPU
# twin of raycast() (tools/raycast, test/bench infrastructure) when it is
# built and a device is visible, else by raycast() itself.
def loop_trajectory(n_frames: int, seed: int = 1005) -> list:
    """Ground-truth poses along the LOOP_X x LOOP_Y ellipse at 10 Hz, LOOP_STEP m per frame, heading
    along the path with a small yaw wobble; 1000 frames are ~1.4 laps."""
    rng = np.random.default_rng(seed)
    th, poses = -math.pi / 2, []
    wob = 0.0
    for _ in range(n_frames):
        x, y = LOOP_X * math.cos(th), LOOP_Y * math.sin(th)
        dx, dy = -LOOP_X * math.sin(th), LOOP_Y * math.cos(th)
        wob = float(np.clip(0.9 * wob + rng.normal(0, 0.01), -0.05, 0.05))
        poses.append(make_pose([x, y, SENSOR_Z], (0.0, 0.0, math.atan2(dy, dx) + wob)))
        th += LOOP_STEP / math.hypot(dx, dy)
    return poses


def _bounce(c, v, t, lo, hi):
    """Position c + v t reflected into [lo, hi] (a pedestrian walking back and forth)."""
    span = hi - lo
    u = (c + v * t - lo) % (2 * span)
    return lo + (u if u <= span else 2 * span - u)


def ped_boxes(scene: Scene, t: float):
    """Pedestrian AABBs at time t, bouncing inside the square (loop scenes)."""
    lo = scene.peds_lo.copy()
    hi = scene.peds_hi.copy()
    for q in range(len(lo)):
        for a, lim in ((0, PLAZA_X - 2.0), (1, PLAZA_Y - 2.0)):
            half = 0.5 * (hi[q, a] - lo[q, a])
            c = _bounce(0.5 * (lo[q, a] + hi[q, a]), scene.peds_vel[q, a], t, -lim, lim)
            lo[q, a], hi[q, a] = c - half, c + half
    return lo, hi


def _raycast_lib():
    import ctypes as C
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "raycast",
                        "libddlo_raycast.so")
    if not os.path.exists(path):
        return None
    from . import load
    load()   # torch's HIP runtime first (see load())
    L = C.CDLL(path)
    P = C.c_void_p
    L.ddlo_raycast.restype = C.c_int
    L.ddlo_raycast.argtypes = [C.c_int, C.c_int, C.c_int, P, P, C.c_int, P, P, C.c_int, P, C.c_int, P, P, P, P,
                               C.c_double, C.c_double, C.c_double]
    return L


def loop_sequence(rows: int, cols: int, first: int, count: int, cfg_id: int = 5, device: int = 0,
                  gpu: bool = True):
    """Frames first .. first+count-1 of cfg 5's 1000-frame loop (moving pedestrians), sensor frame, no-return
    pixels dropped; frame k uses seed 1000 + cfg_id + k and time 0.1 k.  Returns (frames, world poses)."""
    seed = 1000 + cfg_id
    sc = make_scene(seed, moving=True, loop=True)
    poses = loop_trajectory(first + count, seed)[first:]
    L = _raycast_lib() if gpu else None
    if L is None:
        out = []
        for j, P in enumerate(poses):
            k = first + j
            lo, hi = ped_boxes(sc, 0.1 * k)
            s2 = Scene(sc.boxes_lo, sc.boxes_hi, sc.poles, lo, hi, np.zeros_like(sc.peds_vel))
            out.append(raycast(s2, P, rows, cols, seed=seed + k, noise=LOOP_NOISE))
        return out, poses
    import ctypes as C
    dirs = np.ascontiguousarray(lidar_dirs(rows, cols), np.float64)
    nr = rows * cols
    frames = []
    bl, bh = np.ascontiguousarray(sc.boxes_lo, np.float64), np.ascontiguousarray(sc.boxes_hi, np.float64)
    pl = np.ascontiguousarray(sc.poles, np.float64)
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)
    for b0 in range(0, count, 64):
        nb = min(64, count - b0)
        T = np.ascontiguousarray(np.stack(poses[b0:b0 + nb]), np.float64)
        plo = np.empty((nb, len(sc.peds_lo), 3))
        phi = np.empty_like(plo)
        noise = np.empty((nb, nr))
        for j in range(nb):
            k = first + b0 + j
            plo[j], phi[j] = ped_boxes(sc, 0.1 * k)
            noise[j] = np.random.default_rng(seed + k).normal(0.0, LOOP_NOISE, size=nr)
        out = np.empty((nb, nr, 3), np.float32)
        rc = L.ddlo_raycast(device, nb, nr, ptr(dirs), ptr(T), len(bl), ptr(bl), ptr(bh), len(pl), ptr(pl),
                            len(sc.peds_lo), ptr(plo), ptr(phi), ptr(noise), ptr(out), PLAZA_X, PLAZA_Y, FACADE_H)
        if rc != 0:
            raise RuntimeError(f"ddlo_raycast failed ({rc})")
        for j in range(nb):
            f = out[j]
            frames.append(np.ascontiguousarray(f[np.isfinite(f[:, 0])]))
    return frames, poses
