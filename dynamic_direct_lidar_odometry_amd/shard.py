"""Spatially sharded S2M registration across GPUs (cfg 4).

The reference aligns a scan against the keyframe submap on one host
(``NanoGICP::linearize``, reference ``include/nano_gicp/impl/nano_gicp_impl.hpp:277-342``,
summing per-OpenMP-thread H/b partials at :330-339).  When the submap
outgrows one GPU, the same sum is split by SPACE instead of by thread:

* the target submap is cut into ``nranks`` slabs along its longest axis at
  count-balanced fp32 cut points; rank r keeps the points of slab
  ``[lo_r, hi_r)`` plus a halo of ``max_correspondence_distance`` on both
  sides (and the covariances of those points, computed on the whole cloud);
* every rank holds the whole source scan; each outer iteration it transforms
  all source points and searches only those whose transformed coordinate
  falls in its own slab (exactly one rank owns each point), so every exact
  bounded 1-NN it needs lies in its slab + halo;
* the 80 moment doubles of the owned points (H, b, cost and the LM trial-cost
  moments) are summed with ONE RCCL all-reduce per iteration inside the
  align graph, and every rank runs the identical LM step on identical sums.

The work of a rank is its OWNED SOURCE points, not its target points: a
lidar scan is dense near the sensor, so target-count-balanced slabs gave one
rank up to 2.65x the mean query count at 8 ranks.  Two balanced modes:

* ``mode="slabs"``: the cuts are quantiles of the source transformed by the
  align's initial guess along its longest extent (plan_slabs_by_source), the
  target keeps the slab + halo rule above;
* ``mode="groups"`` (default while the submap fits one GPU — 2M points are
  ~200 MB of the 288 GB): the target is replicated and rank r owns the
  16-point groups of the source's spatial order = r (mod nranks)
  (``gicp_set_shard_groups``), SURVEY.md §8(e)'s replicated-target
  alternative with the same single all-reduce; query counts differ by at most
  one group and every rank's queries span the whole scan.

This module is the host side: slab planning (pure numpy, testable on CPU)
and a per-rank driver over the C-ABI (``gicp_set_shard`` /
``gicp_set_shard_groups`` / ``gicp_set_comm``).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

__all__ = ["Slab", "plan_slabs", "plan_slabs_by_source", "halo_indices", "owner_of", "group_owner",
           "ShardedGicp"]


@dataclass(frozen=True)
class Slab:
    axis: int
    lo: float   # float32 value; -inf for the first slab
    hi: float   # float32 value; +inf for the last slab


def plan_slabs(points: np.ndarray, nranks: int, axis: int | None = None) -> list[Slab]:
    """Count-balanced slabs of the target along `axis` (default: longest extent).

    Cut values are float32, exactly the values the search kernel compares
    the fp32 transformed query coordinate against, so ownership is a
    partition of the real line: slab r owns q with lo_r <= q < hi_r.
    """
    if nranks < 1:
        raise ValueError("nranks must be >= 1")
    p = np.asarray(points, np.float32)[:, :3]
    if axis is None:
        axis = int(np.argmax(p.max(axis=0) - p.min(axis=0))) if len(p) else 0
    coord = np.sort(p[:, axis]) if len(p) else np.zeros(1, np.float32)
    cuts = [coord[min(len(coord) - 1, (len(coord) * r) // nranks)] for r in range(1, nranks)]
    cuts = np.maximum.accumulate(np.asarray(cuts, np.float32)) if cuts else np.zeros(0, np.float32)
    bounds = [np.float32(-np.inf)] + [np.float32(c) for c in cuts] + [np.float32(np.inf)]
    return [Slab(axis, float(bounds[r]), float(bounds[r + 1])) for r in range(nranks)]


def transform_f32(points: np.ndarray, T: np.ndarray) -> np.ndarray:
    """The kernels' fp32 query transform, (r0 x + r1 y) + (r2 z + t) (oracle/cpu_ref.cpp)."""
    p = np.asarray(points, np.float32)[:, :3]
    R = np.asarray(T, np.float64)[:3, :3].astype(np.float32)
    t = np.asarray(T, np.float64)[:3, 3].astype(np.float32)
    return np.stack([(R[r, 0] * p[:, 0] + R[r, 1] * p[:, 1]) + (R[r, 2] * p[:, 2] + t[r]) for r in range(3)], 1)


def plan_slabs_by_source(source: np.ndarray, guess: np.ndarray, nranks: int, axis: int | None = None) -> list[Slab]:
    """Slabs that balance the queries each rank OWNS: count-balanced cuts of the source transformed by the
    align's initial guess (the pose of the first search), along its longest extent."""
    return plan_slabs(transform_f32(source, guess), nranks, axis)


def group_owner(n: int, nranks: int) -> np.ndarray:
    """Rank owning each sorted source position under gicp_set_shard_groups: (position // 16) % nranks."""
    return (np.arange(n) // 16) % nranks


def halo_width(max_corr: float) -> float:
    """Halo beyond the slab: max_corr plus a margin that covers the fp32
    rounding of the transformed query and of the squared distance."""
    return float(max_corr) * (1.0 + 1e-4) + 1e-3


def halo_indices(points: np.ndarray, slab: Slab, max_corr: float) -> np.ndarray:
    """Indices of the target points rank `slab` must hold: its slab widened by the halo."""
    c = np.asarray(points, np.float32)[:, slab.axis].astype(np.float64)
    h = halo_width(max_corr)
    return np.flatnonzero((c >= slab.lo - h) & (c <= slab.hi + h)).astype(np.int64)


def owner_of(q: np.ndarray, slabs: list[Slab]) -> np.ndarray:
    """Rank owning each (fp32) transformed query point — the kernel's predicate."""
    c = np.asarray(q, np.float32)[:, slabs[0].axis]
    lo = np.array([s.lo for s in slabs], np.float32)
    hi = np.array([s.hi for s in slabs], np.float32)
    own = (c[:, None] >= lo[None, :]) & (c[:, None] < hi[None, :])
    return np.argmax(own, axis=1)


class ShardedGicp:
    """One rank of a sharded S2M align (one process per GPU).

    ``unique_id`` comes from :func:`dynamic_direct_lidar_odometry_amd.comm_unique_id`
    on rank 0, broadcast by the caller (e.g. over ``torch.distributed``).
    ``nranks == 1`` runs the same code path with a one-rank communicator.
    """

    def __init__(self, device: int, rank: int, nranks: int, unique_id: bytes, params, mode: str = "groups"):
        from . import Context
        if mode not in ("groups", "slabs"):
            raise ValueError("mode must be 'groups' or 'slabs'")
        self.rank, self.nranks = rank, nranks
        self.params = params
        self.mode = mode
        self.ctx = Context(device)
        self.ctx.set_params(params)
        self.ctx.set_comm(unique_id, nranks, rank)
        self.slab: Slab | None = None
        self.local_index: np.ndarray | None = None

    def set_target(self, points: np.ndarray, covs: np.ndarray, axis: int | None = None,
                   source: np.ndarray | None = None, guess: np.ndarray | None = None):
        """Whole submap + its covariances (computed on the whole cloud, as the
        per-keyframe covariances of odom.cc:1147-1149,1302-1310 are).  Slab
        mode balances the owned source at `guess` when source and guess are
        given (else the target count)."""
        from . import TARGET, GicpError
        if self.mode == "groups":
            self.slab = None
            self.local_index = np.arange(len(points), dtype=np.int64)
            self.ctx.set_target(np.ascontiguousarray(np.asarray(points, np.float32)[:, :3]))
            self.ctx.set_covariances(TARGET, np.ascontiguousarray(covs))
            self.ctx.set_shard(-1)
            self.ctx.set_shard_groups(self.nranks, self.rank)
            return None
        if source is not None and guess is not None:
            slabs = plan_slabs_by_source(source, guess, self.nranks, axis)
        else:
            slabs = plan_slabs(points, self.nranks, axis)
        self.slab = slabs[self.rank]
        whole = np.ascontiguousarray(np.asarray(points, np.float32)[:, :3])
        idx = self._slab_index(whole, self.slab)
        self.local_index = idx
        self.ctx.set_target(np.ascontiguousarray(whole[idx]))
        self.ctx.set_covariances(TARGET, np.ascontiguousarray(covs[idx]))
        # exact ties in the whole submap's nanoflann order: each rank holds that
        # tree restricted to its slab + halo, built and cut once per submap on
        # rank 0 and sent to its rank (tietree.hip); nothing with Morton ties
        if self.ctx.tie_order():
            if self.nranks == 1:
                self.ctx.set_tie_target(whole, idx)
            else:
                blobs = None
                if self.rank == 0:
                    try:
                        self.ctx.tie_builder_set(whole)
                        blobs = [self.ctx.tie_builder_export(self._slab_index(whole, s)) for s in slabs]
                    except Exception:
                        # the other ranks are already waiting in the collective: enter it with no blobs
                        # (a failure word goes out, every rank raises) before re-raising here
                        try:
                            self.ctx.set_tie_trees_from_root(0, None)
                        except GicpError:
                            pass
                        raise
                    finally:
                        self.ctx.tie_builder_set(None)
                self.ctx.set_tie_trees_from_root(0, blobs)
        self.ctx.set_shard_groups(0, 0)
        self.ctx.set_shard(self.slab.axis, self.slab.lo, self.slab.hi)
        return self.slab

    def _slab_index(self, whole: np.ndarray, slab: Slab) -> np.ndarray:
        idx = halo_indices(whole, slab, self.params.max_correspondence_distance)
        if len(idx) == 0:  # an empty rank still needs a valid cloud; it owns no queries
            idx = np.zeros(1, np.int64)
        return idx

    def set_source(self, points: np.ndarray, covs: np.ndarray | None = None):
        from . import SOURCE
        self.ctx.set_source(points)
        if covs is not None:
            self.ctx.set_covariances(SOURCE, covs)
        else:
            self.ctx.compute_covariances(SOURCE)

    def align(self, guess=None):
        return self.ctx.align(guess)

    def residuals(self):
        return self.ctx.residuals()

    def close(self):
        self.ctx.set_comm(None, 0, 0)
        self.ctx.close()
