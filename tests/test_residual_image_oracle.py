"""CPU check of the residual-image restatement (oracle.residual_image) against
a literal pure-Python transcription of the reference loop (odom.cc:810-826:
sequential writes, so the last point on a pixel wins; static_cast<int>
truncates toward zero; out-of-range pixels skipped) on a small random cloud."""
import math

import numpy as np

from oracle import oracle as O


def literal(points, residuals, tmin, tmax, W, H):
    img = np.zeros((H, W), np.float32)
    for i, (x, y, z) in enumerate(points.astype(np.float32)):
        xz2 = float(np.float32(x * x) + np.float32(z * z))
        theta = math.atan2(float(x), float(z))
        phi = math.atan2(float(y), math.sqrt(xz2))
        u = int((theta - tmin) / (tmax - tmin) * W)
        v = int((phi - tmin) / (tmax - tmin) * H)
        if u < 0 or u >= W or v < 0 or v >= H:
            continue
        img[v, u] = np.float32(residuals[i])
    return img


def test_restatement_matches_literal_loop():
    rng = np.random.default_rng(3)
    pts = rng.normal(0, 5, (3000, 3)).astype(np.float32)
    pts[:, 2] = np.abs(pts[:, 2]) + 1.0
    res = rng.uniform(0, 2, 3000)
    tmin, tmax = -math.pi / 3, math.pi / 3
    img, win = O.residual_image(pts, res, tmin, tmax, 48, 40)
    assert np.array_equal(img, literal(pts, res, tmin, tmax, 48, 40))
    assert (win >= 0).sum() > 500      # collisions present: 3000 points, 1920 pixels
