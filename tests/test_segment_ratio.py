"""The segmentation labeller's edge test (csrc/segment.hip, Labeller::component)
decides `atan2(y, x) > theta` from the ratio y / x whenever it lies outside
[tan(theta (1 - 1e-6)), tan(theta (1 + 1e-6))] and calls atan2 only inside
that band (and for x <= 0).  The reference computes the float atan2
(detection.cpp:603-606).  This checks the band argument against a float32
atan2 (numpy's, within an ulp like glibc's atan2f) on random edges and on
edges built within a few ulps of the threshold."""
import numpy as np

THETA = np.float32(60.0 / 180.0 * np.pi)   # ddlo_seg_default_params / ddlo.yaml segment theta


def ratio_decision(y, x, theta):
    th = float(theta)
    lo, hi = np.tan(th * (1.0 - 1e-6)), np.tan(th * (1.0 + 1e-6))
    ref = np.arctan2(y, x).astype(np.float32) > theta
    with np.errstate(divide="ignore", invalid="ignore"):
        r = y.astype(np.float64) / x.astype(np.float64)
    pos = x > 0
    out = ref.copy()
    out[pos & (r > hi)] = True
    out[pos & (r < lo)] = False
    return out, ref, pos & ((r > hi) | (r < lo))


def edges_random(rng, m):
    d = rng.uniform(0.5, 80.0, (2, m)).astype(np.float32)
    d1, d2 = np.maximum(d[0], d[1]), np.minimum(d[0], d[1])
    ang = np.float32(360.0 / 512.0) if rng.random() < 0.5 else np.float32(2 * 15.0 / 511)
    sa = np.float32(np.sin(ang / 180.0 * np.pi))
    ca = np.float32(np.cos(ang / 180.0 * np.pi))
    y = (d2 * sa).astype(np.float32)
    x = (d1 - d2 * ca).astype(np.float32)
    return y, x


def edges_near_threshold(rng, m):
    x = rng.uniform(1e-3, 10.0, m).astype(np.float32)
    y = (x.astype(np.float64) * np.tan(float(THETA))).astype(np.float32)
    k = rng.integers(-40, 41, m)
    y = np.array([np.float32(v) for v in y])
    for i in range(m):   # walk k ulps from the threshold ratio
        y[i] = np.nextafter(y[i], np.float32(np.inf) if k[i] > 0 else np.float32(0), dtype=np.float32) if k[i] else y[i]
        for _ in range(abs(int(k[i])) - 1):
            y[i] = np.nextafter(y[i], np.float32(np.inf) if k[i] > 0 else np.float32(0), dtype=np.float32)
    return y, x


def test_ratio_decisions_equal_atan2_on_random_edges():
    rng = np.random.default_rng(7)
    y, x = edges_random(rng, 200_000)
    out, ref, decided = ratio_decision(y, x, THETA)
    assert np.array_equal(out, ref)
    assert decided.mean() > 0.99   # the division decides almost every edge


def test_ratio_decisions_equal_atan2_next_to_the_threshold():
    rng = np.random.default_rng(11)
    y, x = edges_near_threshold(rng, 4000)
    out, ref, decided = ratio_decision(y, x, THETA)
    assert np.array_equal(out, ref)
    assert 0 < decided.mean() < 1   # some edges fall inside the band and are left to atan2
