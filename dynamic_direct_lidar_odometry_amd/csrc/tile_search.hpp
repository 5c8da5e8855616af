// tile_search.hpp — exact bounded 1-NN correspondence search, one wavefront
// per 64 Morton-consecutive source points (lane = query).
//
// Replaces the per-query nanoflann descent of update_correspondences
// (reference include/nano_gicp/impl/nano_gicp_impl.hpp:249-258 ->
// nanoflann_impl.hpp:1495-1566) with a "brute tile" over the leaves that
// the wave's 64 query balls can reach:
//   1. union box of the active lanes' balls (split at Morton jumps when it
//      is wider than kSplitExtent, <= 4 sub-ranges);
//   2. walk the target's upper levels (cached in LDS per workgroup) -> the
//      level-1 blocks overlapping the box; load their leaf boxes (lane =
//      leaf, 4 blocks per round trip) -> union-box candidates;
//   3. every candidate leaf is tested EXACTLY against every lane's own ball
//      (box distance <= the lane's bound); a leaf needed by any lane joins
//      the wave's scan list;
//   4. the scan list is streamed through LDS 16 leaves per round trip
//      (global_load_lds, 2 leaves per instruction) and every lane scans
//      every listed point against its own query.
// The search runs in two phases per outer iteration:
//   phase A (k_nn_tile_a) — the lane's bound is min(b, R0^2), where b is a
//     valid upper bound of the 1-NN distance (triangle inequality from the
//     previous correspondence: |q - p_prev| <= sqrt(sqd_prev) + |q - q_prev|,
//     else max_corr^2).  A query whose result is <= min(b, R0^2) is exact.
//   phase B (k_nn_tile_b) — the remaining queries (NN farther than R0 and
//     no tight b: the first iteration of an align, points off the map) are
//     compacted into a list and searched, 64 per wave, with their full
//     bound (the phase-A best, which is <= b).
// Exactness: a leaf is skipped only if its box is farther than the lane's
// current bound, bounds only shrink, the squared distance is nanoflann's
// fp32 ((dx^2 + dy^2) + dz^2) without contraction, and ties are broken by
// the lower sorted position — the result is the unique minimum of
// (distance, position) whatever the order leaves are visited in.
#pragma once
#include "search.hpp"

namespace ddlo {

constexpr int kTileChunk = 24;      // candidate leaves staged in LDS at once
constexpr int kTileRow = kLeafSize + 1;  // padded leaf row (f4v): spreads LDS banks
constexpr int kTileBlkMax = 64;     // level-1 blocks listed per walk
constexpr int kDeferGroups = 1;     // phase-A groups merged into one phase-B wave

struct TileLds {
  int cand[kTileChunk];             // leaf ids of the staged chunk
  int blocks[kTileBlkMax];
  int defer[kDeferGroups * 64];     // phase B: deferred source positions, in order
  f4v pts[kTileChunk * kTileRow];   // staged leaves (x, y, z, idx bits)
};
constexpr int kTileLdsBytes = (int)sizeof(TileLds);

struct TileStats {
  unsigned blocks = 0, cand = 0, listed = 0, batches = 0, splits = 0;
  unsigned long long cyc_scan = 0, cyc_blocks = 0;  // s_memtime spent in flush_scan / flush_blocks
};

// Per-lane query + wave-uniform list state.
struct TileSearch {
  CloudDev c;       // by value: kernel arguments stay in SGPRs
  TileLds* L;
  const f4v* U;     // upper-level box cache (LDS)
  int nup;
  float qx, qy, qz;
  bool active;      // lane takes part in the current (sub-range) leaf tests
  bool alive;       // lane has a query: every scanned leaf updates it
  float cap;        // pruning cap (phase A: R0^2, phase B: +inf)
  float best;       // squared distance of the current best (or the bound)
  int bestj;        // its sorted target position (-1: none, bound only)
  float bx, by, bz; // coordinates of the best point (valid when bestj >= 0)
  int nscan;        // wave-uniform number of staged candidates
  unsigned need;    // per lane: bit c = staged candidate c may hold a closer point
  int nblocks;      // wave-uniform block-list length
  WaveBox box;
  float split_ext;  // union-box extent above which the wave splits (m)
  TileStats st;

  __device__ __forceinline__ float bound() const { return active ? fminf(best, cap) : -1.f; }

  // Scan the staged chunk.  Every lane walks only the candidates its own
  // ball reaches (bit mask `need`), one candidate per step, reading the
  // points from LDS at its own address: the wave runs max-over-lanes steps
  // instead of scanning every candidate for all 64 queries.
  __device__ __forceinline__ void flush_scan() {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const int n = nscan;
    if (n > 0) {
      const int lane = lane_id();
      // stage the n candidate leaves: one 32-lane DMA per leaf into its padded row
      for (int cc = 0; cc < n; ++cc) {
        const int lf = __builtin_amdgcn_readfirstlane(L->cand[cc]);
        if (lane < kLeafSize) {
          const float4* src = c.pts + (size_t)lf * kLeafSize + lane;
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                           (__attribute__((address_space(3))) void*)&L->pts[cc * kTileRow], 16, 0, 0);
        }
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the chunk is in LDS
      __builtin_amdgcn_wave_barrier();
      float b = best;
      unsigned bj = (unsigned)bestj;
      float px = bx, py = by, pz = bz;
      unsigned m = alive ? need : 0u;
      const f2v qx2 = {qx, qx}, qy2 = {qy, qy}, qz2 = {qz, qz};
      while (__any(m != 0u)) {
        st.batches += 1;
        const int cc = m ? __builtin_ctz(m) : 0;
        m &= m - 1;
        const f4v* pp = &L->pts[cc * kTileRow];
        float mn = INFINITY;
        int a = 0;
#pragma unroll 4
        for (int h = 0; h < kLeafSize; h += 2) {
          const f4v p0 = pp[h], p1 = pp[h + 1];
          const f2v dx = qx2 - f2v{p0.x, p1.x};
          const f2v dy = qy2 - f2v{p0.y, p1.y};
          const f2v dz = qz2 - f2v{p0.z, p1.z};
          const f2v d = (dx * dx + dy * dy) + dz * dz;
          // strict '<' keeps the lower position among equal distances
          if (d.x < mn) { mn = d.x; a = h; }
          if (d.y < mn) { mn = d.y; a = h + 1; }
        }
        const unsigned pos = (unsigned)(L->cand[cc] * kLeafSize + a);
        const f4v w = pp[a];
        if (mn < b || (mn == b && pos < bj)) {
          b = mn;
          bj = pos;
          px = w.x;
          py = w.y;
          pz = w.z;
        }
      }
      // every live lane (not only the current sub-range's) owns its mask bits
      if (alive) {
        best = b;
        bestj = (int)bj;
        bx = px;
        by = py;
        bz = pz;
      }
      __builtin_amdgcn_wave_barrier();
    }
    nscan = 0;
    need = 0u;
    st.cyc_scan += __builtin_amdgcn_s_memtime() - t0;
  }

  // stage candidate `leaf` for the lanes whose ball reaches it
  __device__ __forceinline__ void list_leaf(int leaf, bool lane_needs) {
    if (nscan == kTileChunk) flush_scan();
    if (lane_id() == 0) L->cand[nscan] = leaf;
    __builtin_amdgcn_wave_barrier();
    if (lane_needs) need |= 1u << nscan;
    nscan += 1;
  }

  // leaf filter of the listed level-1 blocks, 4 blocks per round trip
  __device__ __forceinline__ void flush_blocks() {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long s0 = st.cyc_scan;
    const int lane = lane_id();
    const int nb = nblocks;
    for (int b0 = 0; b0 < nb; b0 += 4) {
      float4 lo[4], hi[4];
      int base[4], cnt[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int bi = min(b0 + u, nb - 1);
        base[u] = __builtin_amdgcn_readfirstlane(L->blocks[bi]) * kFanout;
        cnt[u] = (b0 + u < nb) ? min(kFanout, c.cnt0 - base[u]) : 0;
        const int li = min(base[u] + lane, c.cnt0 - 1);
        lo[u] = ldg4(c.box_lo, li);
        hi[u] = ldg4(c.box_hi, li);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (cnt[u] == 0) continue;
        st.blocks += 1;
        const bool ov = lane < cnt[u] && box_overlap(box, lo[u], hi[u]);
        unsigned long long m = __ballot(ov);
        st.cand += __popcll(m);
        const float bnd = bound();
        while (m) {
          const int b = __builtin_ctzll(m);
          m &= m - 1;
          const float4 blo = make_float4(readlane_f(lo[u].x, b), readlane_f(lo[u].y, b), readlane_f(lo[u].z, b), 0.f);
          const float4 bhi = make_float4(readlane_f(hi[u].x, b), readlane_f(hi[u].y, b), readlane_f(hi[u].z, b), 0.f);
          const bool nd = box_dist2(qx, qy, qz, blo, bhi) <= bnd;
          if (__any(nd)) {
            st.listed += 1;
            list_leaf(base[u] + b, nd);
          }
        }
      }
    }
    nblocks = 0;
    st.cyc_blocks += (__builtin_amdgcn_s_memtime() - t0) - (st.cyc_scan - s0);
  }

  __device__ __forceinline__ void push_block(int node) {
    if (nblocks == kTileBlkMax) flush_blocks();
    if (lane_id() == 0) L->blocks[nblocks] = node;
    __builtin_amdgcn_wave_barrier();
    nblocks += 1;
  }

  __device__ __forceinline__ bool upper_ov(int level, int idx) const {
    const int k = lvl_off(c, level) - c.off1 + idx;
    return box_overlap_v(box, U[k], U[nup + k]);
  }

  template <int LV>
  __device__ __forceinline__ void walk(int base, unsigned long long mask) {
    while (mask) {  // nodes of level LV (>= 2) overlapping the box
      const int ci = __builtin_ctzll(mask);
      mask &= mask - 1;
      const int cb = (base + ci) * kFanout;
      const int cnt = min(kFanout, lvl_cnt(c, LV - 1) - cb);
      unsigned long long m = __ballot(lane_id() < cnt && upper_ov(LV - 1, cb + lane_id()));
      if constexpr (LV == 2) {
        while (m) {
          const int b = __builtin_ctzll(m);
          m &= m - 1;
          push_block(cb + b);
        }
      } else {
        walk<LV - 1>(cb, m);
      }
    }
  }

  // all level-1 blocks overlapping the current box -> filtered leaves
  __device__ __forceinline__ void collect() {
    const int T = c.nlevels - 1;
    if (T == 0) {
      push_block(0);
    } else {
      unsigned long long m = __ballot(lane_id() < lvl_cnt(c, T) && upper_ov(T, lane_id()));
      if (T == 1) {
        while (m) {
          const int b = __builtin_ctzll(m);
          m &= m - 1;
          push_block(b);
        }
      } else if (T == 2) {
        walk<2>(0, m);
      } else if (T == 3) {
        walk<3>(0, m);
      } else {
        walk<4>(0, m);
      }
    }
    flush_blocks();
  }

  // Lanes in `need` take, as a candidate, the exact distance to the best
  // point of every lane in `have` (spatially adjacent queries in Morton
  // order find nearby surface points): a valid (distance, position) pair,
  // so exactness is kept while the bound gets tight before a wide search.
  __device__ __forceinline__ void seed_from_lanes(bool need, unsigned long long have) {
    if (!__any(need) || !have) return;
    float b = best;
    unsigned bj = (unsigned)bestj;
    float px = bx, py = by, pz = bz;
    while (have) {
      const int k = __builtin_ctzll(have);
      have &= have - 1;
      const float sx = readlane_f(bx, k), sy = readlane_f(by, k), sz = readlane_f(bz, k);
      const unsigned sj = (unsigned)readlane_i(bestj, k);
      const float d = dist2(qx, qy, qz, sx, sy, sz);
      if (d < b || (d == b && sj < bj)) {
        b = d;
        bj = sj;
        px = sx;
        py = sy;
        pz = sz;
      }
    }
    if (need) {
      best = b;
      bestj = (int)bj;
      bx = px;
      by = py;
      bz = pz;
    }
  }

  // the whole search for the wave's active lanes; key = source Morton key
  __device__ __forceinline__ void run(unsigned long long key) {
    nscan = 0;
    need = 0u;
    nblocks = 0;
    const bool base_active = active;
    alive = active;
    const WaveBox whole = make_wave_box(active, qx, qy, qz, bound());
    if (!(box_extent(whole) > split_ext)) {
      box = whole;
      collect();
    } else {
      st.splits += 1;
      const int qi = lane_id();
      const int sp = morton_jump_split<64>(key, 0, 64);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int lo = h == 0 ? 0 : sp, hi = h == 0 ? sp : 64;
        if (lo >= hi) continue;
        active = base_active && qi >= lo && qi < hi;
        const WaveBox hb = make_wave_box(active, qx, qy, qz, bound());
        if (box_extent(hb) > split_ext && hi - lo > 4) {
          st.splits += 1;
          const int s2 = morton_jump_split<64>(key, lo, hi);
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const int l2 = h2 == 0 ? lo : s2, r2 = h2 == 0 ? s2 : hi;
            active = base_active && qi >= l2 && qi < r2;
            if (!__any(active)) continue;
            box = make_wave_box(active, qx, qy, qz, bound());
            collect();
          }
        } else if (__any(active)) {
          box = hb;
          collect();
        }
      }
      active = base_active;
    }
    flush_scan();
  }
};

}  // namespace ddlo
