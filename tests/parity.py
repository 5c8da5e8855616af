"""Shared parity assertions for the GPU tests."""
import numpy as np


def assert_cov_parity(pts, k, gpu, ref, atol=1e-12):
    """Covariances equal to atol at EVERY point.  Points whose k-neighbourhood
    has an exact distance tie at its boundary (k-th == (k+1)-th squared
    distance) included: the device resolves them with nanoflann's own tree
    (nftree.hip), so the neighbour set is the reference's.  Returns the
    number of mismatches (always 0)."""
    scale = max(np.abs(ref).max(), 1.0)
    bad = np.where(np.abs(gpu - ref).max(axis=1) > atol * scale)[0]
    assert len(bad) == 0, f"{len(bad)} covariance mismatches, first at points {bad[:10]}"
    return 0
