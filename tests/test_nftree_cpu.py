"""CPU checks behind the device build of nanoflann's kd-tree (nftree.hip),
the structure that fixes the reference's order among exactly equidistant
points (DESIGN.md "Tie order").

* The oracle's tree restatement (oracle/cpu_ref.cpp) is pinned to the
  reference's own nanoflann compiled from /root/reference (oracle/_ref):
  identical vind permutation, leaves and divfeat / divlow / divhigh.
* planeSplit's two Hoare loops (reference impl/nanoflann_impl.hpp:1107-1143)
  equal the rank pairing the device uses to run them in parallel: with
  L = #{good}, the r-th bad element of [0, L) (ascending) swaps with the r-th
  good element of [L, n) (descending)."""
import numpy as np
import pytest

from oracle import oracle as O


def _plane_split_loop(v, cut):
    """planeSplit (:1107-1143) literally, on a value array (returns the permutation)."""
    ind = list(range(len(v)))
    count = len(v)
    left, right = 0, count - 1
    while True:
        while left <= right and v[ind[left]] < cut:
            left += 1
        while right and left <= right and v[ind[right]] >= cut:
            right -= 1
        if left > right or not right:
            break
        ind[left], ind[right] = ind[right], ind[left]
        left += 1
        right -= 1
    lim1 = left
    right = count - 1
    while True:
        while left <= right and v[ind[left]] <= cut:
            left += 1
        while right and left <= right and v[ind[right]] > cut:
            right -= 1
        if left > right or not right:
            break
        ind[left], ind[right] = ind[right], ind[left]
        left += 1
        right -= 1
    return np.array(ind), lim1, left


def _rank_pair(ind, good, lo, hi):
    """One pass as the device runs it: good zone [lo, hi), the rest [hi, n)."""
    ind = ind.copy()
    g = good[ind]
    bad_left = np.where(~g[lo:hi])[0] + lo
    good_right = (np.where(g[hi:])[0] + hi)[::-1]
    assert len(bad_left) == len(good_right)
    a, b = ind[bad_left].copy(), ind[good_right].copy()
    ind[bad_left], ind[good_right] = b, a
    return ind


def _plane_split_pairs(v, cut):
    n = len(v)
    ind = np.arange(n)
    lim1 = int(np.sum(v < cut))
    lim2 = int(np.sum(v <= cut))
    ind = _rank_pair(ind, v < cut, 0, lim1)
    ind = _rank_pair(ind, v == cut, lim1, lim2)
    return ind, lim1, lim2


@pytest.mark.parametrize("seed", range(40))
def test_hoare_equals_rank_pairing(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(101, 700))
    levels = int(rng.integers(1, 12))   # few distinct values: many elements equal to the cut
    v = rng.integers(0, levels, n).astype(np.float32) if seed % 2 else rng.standard_normal(n).astype(np.float32)
    cut = v[rng.integers(0, n)] if seed % 3 else np.float32(np.median(v))
    a, l1a, l2a = _plane_split_loop(v, cut)
    b, l1b, l2b = _plane_split_pairs(v, cut)
    assert (l1a, l2a) == (l1b, l2b)
    np.testing.assert_array_equal(a, b)


def _clouds():
    rng = np.random.default_rng(7)
    lat = np.stack(np.meshgrid(np.arange(30), np.arange(30), np.arange(6), indexing="ij"), -1).reshape(-1, 3)
    return {
        "normal": (rng.standard_normal((40000, 3)) * [20, 20, 3]).astype(np.float32),
        "lattice": lat.astype(np.float32),
        "duplicates": np.repeat((rng.standard_normal((3000, 3)) * 5).astype(np.float32), 4, axis=0),
        "leaf_only": rng.standard_normal((57, 3)).astype(np.float32),
        "outliers": np.concatenate([(rng.standard_normal((20000, 3)) * 0.5).astype(np.float32),
                                    np.array([[1e4, 1e4, 1e4], [-5e3, 2, 3]], np.float32)]),
        "flat": np.concatenate([(rng.standard_normal((9000, 2)) * 10), np.zeros((9000, 1))], 1).astype(np.float32),
    }


@pytest.mark.parametrize("name", sorted(_clouds()))
def test_oracle_tree_is_reference_tree(name):
    pts = _clouds()[name]
    ref = O.ref_tree(pts)
    if ref is None:
        pytest.skip("reference nanoflann (oracle/_ref) not built here")
    assert O.same_tree(O.tree(pts), ref) is None
