// nn_tasks.hpp — task-based exact bounded 1-NN: the correspondence search of
// the GICP loop (update_correspondences, reference
// include/nano_gicp/impl/nano_gicp_impl.hpp:249-258, whose per-query
// nanoflann descent is nanoflann_impl.hpp:1495-1566).
//
// Two kernels per outer iteration, both latency-tolerant and load-balanced:
//
//   k_nn_collect   one wavefront per 16 Morton-consecutive source points
//                  (a sub-group): transform, seed an exact upper bound
//                  (previous match / Morton window / neighbours' points),
//                  walk the LDS-cached upper levels with the union box of the
//                  16 balls, test every candidate leaf box EXACTLY against
//                  each query's ball and append one TASK per needed leaf:
//                  (leaf, sub-group, 16-bit query mask).
//   k_nn_scan      every wavefront pulls tasks from the shared list and scans
//                  the leaf's 32 points for the masked queries (lane = query
//                  x quarter of the leaf), merging (distance, position) keys
//                  into the per-query result with a 64-bit atomicMin.
//
// The list spreads the leaf scans of a hard sub-group (a query with a wide
// ball drags hundreds of leaves in) over the whole chip instead of
// serialising them on one wavefront, which set the old single-kernel
// search's duration.  Exactness: a leaf is skipped only if its box is
// farther than the query's seed bound, and the result is the minimum of
// (squared distance, sorted position) over every listed leaf and the seed
// (the same key order as search.hpp's dkey), independent of task order.
#pragma once
#include <hip/hip_runtime.h>

#include "gicp_types.hpp"
#include "search.hpp"

namespace ddlo {

constexpr int kTaskQ = 16;          // queries per sub-group (= per task)
constexpr int kTaskBuf = 320;       // per-wave LDS task buffer: flushed once more than 64 are held (4 blocks add <= 256)

// (leaf, sub-group, mask) in one word: leaf < 2^24, sub-group < 2^24
__device__ __forceinline__ unsigned long long make_task(int leaf, int sg, unsigned mask) {
  return ((unsigned long long)(unsigned)leaf << 40) | ((unsigned long long)(unsigned)sg << 16) |
         (unsigned long long)(mask & 0xffffu);
}

// Scan one task: lane = (query qi = lane & 15, quarter s = lane >> 4), each
// lane takes 8 of the leaf's 32 points; returns, in every lane of query qi,
// the minimum (distance, position) key over the leaf, and in sd the
// smallest squared distance of the leaf's other points.  `q` = the lane's
// query (x, y, z), loaded by the caller.
__device__ __forceinline__ unsigned long long scan_leaf16(const CloudDev& tgt, int leaf, float qx, float qy, float qz,
                                                          float& sd) {
  const int s = lane_id() >> 4;
  const long b = (long)leaf * kLeafSize + s * 8;
  f3v pt[8];
#pragma unroll
  for (int h = 0; h < 8; ++h) pt[h] = ldg3(tgt.pts, b + h);
  const f2v qx2 = {qx, qx}, qy2 = {qy, qy}, qz2 = {qz, qz};
  float bd = INFINITY;
  int bh = 0;
  sd = INFINITY;
#pragma unroll
  for (int h = 0; h < 8; h += 2) {
    // two points at once (v_pk_* ops), same IEEE ops as dist2(); increasing
    // position, so strict < keeps the lowest position among equal distances
    const f2v dx = qx2 - f2v{pt[h].x, pt[h + 1].x};
    const f2v dy = qy2 - f2v{pt[h].y, pt[h + 1].y};
    const f2v dz = qz2 - f2v{pt[h].z, pt[h + 1].z};
    const f2v d = (dx * dx + dy * dy) + dz * dz;
    if (d.x < bd) { sd = bd; bd = d.x; bh = h; } else { sd = fminf(sd, d.x); }
    if (d.y < bd) { sd = bd; bd = d.y; bh = h + 1; } else { sd = fminf(sd, d.y); }
  }
  unsigned long long bk = dkey(bd, (int)b + bh);
  xor_top2<16>(bk, sd);   // quarters s and s ^ 1
  xor_top2<32>(bk, sd);   // quarters s and s ^ 2
  return bk;
}

// Fold a leaf's (best key k2, second distance sd2) into a query's running
// (key, sec): every examined point except the final best ends up <= sec.
// The displaced key counts only if it names a real point, and a point met
// twice (a block reached by two walk entries) is not its own second.
__device__ __forceinline__ void fold_top2(unsigned long long& key, float& sec, unsigned long long k2, float sd2) {
  if (k2 != key) {
    const unsigned long long hi = k2 < key ? key : k2;
    if (key_real(hi)) sec = fminf(sec, key_dist(hi));
  }
  sec = fminf(sec, sd2);
  key = umin64(key, k2);
}

// Per-wave LDS of the collect kernel.
struct TaskLds {
  f4v q[kTaskQ];                       // per query: x, y, z, bound (bound < 0: inactive)
  int ntasks, nsr, pad0, pad1;
  int lvl_off[kMaxLevels], lvl_cnt[kMaxLevels], pad2[6];   // the cloud's level table (runtime-indexed)
  int sr_lo[4], sr_hi[4];              // query sub-ranges of a split wave
  f4v sb_lo[kFanout], sb_hi[kFanout];  // boxes of a block's leaves that pass the union test
  int sb_leaf[kFanout];
  unsigned long long tasks[kTaskBuf];
};
constexpr int kTaskLdsBytes = (int)sizeof(TaskLds);

// Where a sub-group's tasks go: region (g % kTaskRegions) of the list, with
// one append counter per region (a 128-B line each: kCtrStride words).
struct TaskList {
  unsigned long long* tasks;   // [kTaskRegions][cap_r]
  unsigned* ctr;               // [kTaskRegions * kCtrStride]
  int cap_r;
};

struct TaskCollector {
  TaskLds* L;
  const f4v* U;     // upper-level box cache (levels >= 1)
  int nup;
  WaveBox box;
  float qx, qy, qz;
  bool active;
  unsigned long long bk;   // the lane's query key (seed; lowered by inline scans)
  float wr;                // walk radius (squared): leaves farther than this are skipped
  float sec = INFINITY;    // smallest squared distance of an inline-scanned non-best point
  int sg;                  // sub-group index (this wave's 16 queries)
  unsigned st_blocks = 0, st_tasks = 0, st_inline = 0, st_splits = 0;
  unsigned tm_walk = 0;   // s_memtime after the walk (diagnostics)
  unsigned st_iters = 0;
  bool knn = false;        // kNN-k mode (knn_tasks.hip): a full region is an overflow, no inline scan
  bool ovf = false;
  int nfull = 0;           // kNN mode: leaves < nfull hold 32 real points
  float tight = INFINITY;  // kNN mode: min over tested full leaves of the farthest-corner distance (squared)
  int pf_ratio = 0;        // 1-NN mode: lane-per-leaf pair tests while queries < pf_ratio * ceil(leaves / 4)

  __device__ __forceinline__ float bound() const { return __uint_as_float((unsigned)(bk >> 32)); }

  // Append the buffered tasks to the global list.
  __device__ __forceinline__ void flush_tasks(const CloudDev& c, const TaskList& tl) {
    const int lane = lane_id();
    const int n = L->ntasks;
    if (n == 0) return;
    const int r = sg % kTaskRegions;
    int base = 0;
    if (lane == 0) base = (int)atomicAdd(tl.ctr + r * kCtrStride, (unsigned)n);
    base = __builtin_amdgcn_readfirstlane(base);
    // the slots that fit are published; the rest (region full) are scanned
    // right here into the lane's own key (exact either way) — in kNN mode
    // the sub-group is flagged instead and recomputed by the fallback kernel
    const int fit = max(0, min(n, tl.cap_r - base));
    unsigned long long* dst = tl.tasks + (size_t)r * tl.cap_r + base;
    for (int k = lane; k < fit; k += 64) dst[k] = L->tasks[k];
    st_tasks += fit;
    if (knn) {
      ovf = ovf || fit < n;
    } else {
      for (int k = fit; k < n; ++k) {
        const unsigned long long t = L->tasks[k];
        float sd2;
        const unsigned long long k2 = scan_leaf16(c, (int)(t >> 40), qx, qy, qz, sd2);
        if (active && ((t >> (lane & 15)) & 1ull)) fold_top2(bk, sec, k2, sd2);
      }
    }
    st_inline += n - fit;
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) L->ntasks = 0;
    __builtin_amdgcn_wave_barrier();
  }

  // (leaf, query) pair tests of the cm staged leaves against the queries
  // of qmask; a leaf any of them needs becomes one task.  Few queries or
  // many leaves: lane = leaf, one test per query (a broadcast LDS read and a
  // box distance each); else 4 leaves x 16 queries per round (each round an
  // append).  A block whose 64 leaves all pass the union box takes 16 cheap
  // query steps instead of 16 rounds.
  __device__ __forceinline__ void pair_filter(int cm, unsigned qmask) {
    const int lane = lane_id();
    const int nq = __popc(qmask);
    // the queries come from registers: lane l holds query l & 15 (its slices
    // too), so the lane-per-leaf loop reads query k with v_readlane at a
    // constant lane (no LDS round trip per query step)
    const float qw = active ? wr : -1.f;
    if (nq <= 2 || (!knn && nq < pf_ratio * ((cm + 3) >> 2))) {
      const unsigned qm_u = (unsigned)__builtin_amdgcn_readfirstlane((int)qmask);
      unsigned m16 = 0u;
      f4v blo = f4v{0.f, 0.f, 0.f, 0.f}, bhi = blo;
      if (lane < cm) {
        blo = L->sb_lo[lane];
        bhi = L->sb_hi[lane];
      }
      const float4 lo4 = make_float4(blo.x, blo.y, blo.z, 0.f), hi4 = make_float4(bhi.x, bhi.y, bhi.z, 0.f);
#pragma unroll
      for (int k = 0; k < kTaskQ; ++k) {
        if ((qm_u >> k) & 1u) {
          const float kx = readlane_f(qx, k), ky = readlane_f(qy, k), kz = readlane_f(qz, k), kw = readlane_f(qw, k);
          if (lane < cm && kw >= 0.f && box_dist2(kx, ky, kz, lo4, hi4) <= kw) m16 |= 1u << k;
        }
      }
      if (knn) {   // per query: the nearest full leaf's farthest corner bounds its k-th neighbour
        const bool full = lane < cm && L->sb_leaf[lane] < nfull;
#pragma unroll
        for (int k = 0; k < kTaskQ; ++k) {
          if ((qm_u >> k) & 1u) {
            const float kx = readlane_f(qx, k), ky = readlane_f(qy, k), kz = readlane_f(qz, k);
            float v = full ? box_maxdist2(kx, ky, kz, blo, bhi) : INFINITY;
            v = wave_min(v);
            if ((lane & 15) == k) tight = fminf(tight, v);
          }
        }
      }
      const unsigned long long lm = __ballot(m16 != 0u);
      const int cl = __popcll(lm);
      if (cl == 0) return;
      const int n0 = L->ntasks;
      if (m16 != 0u) {
        const int slot =
            n0 + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(lm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)lm, 0u));
        L->tasks[slot] = make_task(L->sb_leaf[lane], sg, m16);
      }
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) L->ntasks = n0 + cl;
      __builtin_amdgcn_wave_barrier();
      return;
    }
    for (int r0 = 0; r0 < cm; r0 += 4) {
      const int li = r0 + (lane >> 4);
      bool need = false;
      if (li < cm && ((qmask >> (lane & 15)) & 1u)) {
        const f4v blo = L->sb_lo[li], bhi = L->sb_hi[li];   // the lane's own query (lane & 15) is in its registers
        need = qw >= 0.f && box_dist2(qx, qy, qz, make_float4(blo.x, blo.y, blo.z, 0.f),
                                      make_float4(bhi.x, bhi.y, bhi.z, 0.f)) <= qw;
        if (knn && L->sb_leaf[li] < nfull) tight = fminf(tight, box_maxdist2(qx, qy, qz, blo, bhi));
      }
      const unsigned long long bal = __ballot(need);
      const unsigned m16 = (unsigned)((bal >> (lane & ~15)) & 0xffffull);
      const bool lead = (lane & 15) == 0 && li < cm && m16 != 0u;
      const unsigned long long lm = __ballot(lead);
      const int cl = __popcll(lm);
      if (cl == 0) continue;
      const int n0 = L->ntasks;
      if (lead) {
        const int slot =
            n0 + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(lm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)lm, 0u));
        L->tasks[slot] = make_task(L->sb_leaf[li], sg, m16);
      }
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) L->ntasks = n0 + cl;
      __builtin_amdgcn_wave_barrier();
    }
  }

  // Exact leaf filter of the level-1 blocks cb + bit (bits of m), 4 blocks
  // per round trip: (1) lane = leaf, one test against the union box of the
  // wave's balls; (2) the survivors' (leaf, query) pair tests.
  __device__ __forceinline__ void filter_blocks(const CloudDev& c, const TaskList& tl, int cb,
                                                unsigned long long m, unsigned qmask) {
    const WaveBox& wb = box;
    const int lane = lane_id();
    while (m) {
      float4 lo[4], hi[4];
      int base[4], cnt[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        cnt[u] = 0;
        base[u] = 0;
        if (m) {
          base[u] = (cb + __builtin_ctzll(m)) * kFanout;
          m &= m - 1;
          cnt[u] = min(kFanout, c.cnt0 - base[u]);
        }
        const int li = min(base[u] + lane, c.cnt0 - 1);
        lo[u] = ldg4(c.box_lo, li);
        hi[u] = ldg4(c.box_hi, li);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (cnt[u] == 0) continue;
        st_blocks += 1;
        const bool pass = lane < cnt[u] && box_overlap(wb, lo[u], hi[u]);
        const unsigned long long pm = __ballot(pass);
        const int cm = __popcll(pm);
        if (cm == 0) continue;
        if (pass) {
          const int slot = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(pm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)pm, 0u));
          L->sb_lo[slot] = f4v{lo[u].x, lo[u].y, lo[u].z, 0.f};
          L->sb_hi[slot] = f4v{hi[u].x, hi[u].y, hi[u].z, 0.f};
          L->sb_leaf[slot] = base[u] + lane;
        }
        __builtin_amdgcn_wave_barrier();
        pair_filter(cm, qmask);
      }
      if (L->ntasks > kTaskBuf - 4 * kFanout) flush_tasks(c, tl);  // keep room for 4 more blocks
    }
  }

  // level table lookups go through LDS: a runtime index into the CloudDev
  // fields would put the whole struct on the scratch stack
  __device__ __forceinline__ bool upper_ov(const CloudDev& c, int level, int idx) const {
    const int k = L->lvl_off[level] - c.off1 + idx;
    return box_overlap_v(box, U[k], U[nup + k]);
  }

  // Depth-first walk of the upper levels with the wave box (explicit
  // per-level stack of 64-bit child masks in scalar registers).  Reaching a
  // level-2 node yields the 64-bit mask of its overlapping level-1 blocks,
  // which are filtered at once (one call site whatever the depth).  Clouds
  // with one or two levels are walked from a virtual level-2 root.
  __device__ __forceinline__ void walk(const CloudDev& c, const TaskList& tl, unsigned qmask) {
    const int T = c.nlevels - 1;
    const int lane = lane_id();
    unsigned long long m2 = 0, m3 = 0, m4 = 0;
    int b2 = 0, b3 = 0;
    int top;
    if (T <= 1) {
      top = 2;
      m2 = 1ull;   // virtual root: its children are the level-1 nodes (T == 1) or the single block (T == 0)
    } else {
      top = T;
      const bool ov = lane < L->lvl_cnt[T] && upper_ov(c, T, lane);
      const unsigned long long m = __ballot(ov);
      if (T == 2) m2 = m; else if (T == 3) m3 = m; else m4 = m;
    }
    int lv = top;
    while (true) {
      st_iters += 1;
      unsigned long long m = lv == 2 ? m2 : lv == 3 ? m3 : m4;
      if (m == 0ull) {
        if (lv == top) break;
        ++lv;
        continue;
      }
      const int base = lv == 2 ? b2 : lv == 3 ? b3 : 0;
      const int node = base + __builtin_ctzll(m);
      m &= m - 1;
      if (lv == 2) m2 = m; else if (lv == 3) m3 = m; else m4 = m;
      const int cb = node * kFanout;
      if (lv == 2) {   // children = level-1 blocks
        unsigned long long cm = 1ull;   // T == 0: the single block
        if (T >= 1) {
          const int cnt = min(kFanout, c.cnt1 - cb);
          cm = __ballot(lane < cnt && upper_ov(c, 1, cb + lane));
        }
        filter_blocks(c, tl, cb, cm, qmask);
        continue;
      }
      const int cnt = min(kFanout, L->lvl_cnt[lv - 1] - cb);
      const unsigned long long cm = __ballot(lane < cnt && upper_ov(c, lv - 1, cb + lane));
      --lv;
      if (lv == 2) { m2 = cm; b2 = cb; } else { m3 = cm; b3 = cb; }
    }
  }

  // Whole collect of the wave's 16 queries, walked as up to 4 entries, each
  // a query mask with its own wave box (used by the walk AND the leaf
  // filter): the group is cut at Morton jumps when its union box is wider
  // than split_extent (<= 4 compact sub-ranges).
  __device__ __forceinline__ void run(const CloudDev& c, const TaskList& tl, unsigned long long key, float split_extent) {
    const int lane = lane_id();
    const int qi = lane & 15;
    if (lane < kTaskQ) L->q[lane] = f4v{qx, qy, qz, active ? wr : -1.f};
    if (lane < kMaxLevels) {
      L->lvl_off[lane] = lane == 0 ? c.off0 : lane == 1 ? c.off1 : lane == 2 ? c.off2 : lane == 3 ? c.off3 : c.off4;
      L->lvl_cnt[lane] = lane == 0 ? c.cnt0 : lane == 1 ? c.cnt1 : lane == 2 ? c.cnt2 : lane == 3 ? c.cnt3 : c.cnt4;
    }
    if (lane == 0) L->ntasks = 0;
    __builtin_amdgcn_wave_barrier();
    unsigned long long rng = 0xffffull;   // up to 4 query masks, 16 bits each (no scratch array)
    int nr = 1;
    const WaveBox whole = make_wave_box(active, qx, qy, qz, wr);
    if (box_extent(whole) > split_extent) {
      st_splits += 1;
      const int sp = morton_jump_split<kTaskQ>(key, 0, kTaskQ);
      nr = 0;
      rng = 0ull;
      for (int h = 0; h < 2; ++h) {
        const int lo = h == 0 ? 0 : sp, hi = h == 0 ? sp : kTaskQ;
        if (lo >= hi) continue;
        const unsigned half = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
        const bool act = active && qi >= lo && qi < hi;
        const WaveBox hb = make_wave_box(act, qx, qy, qz, wr);
        if (box_extent(hb) > split_extent && hi - lo > 4) {
          st_splits += 1;
          const int s2 = morton_jump_split<kTaskQ>(key, lo, hi);
          rng |= (unsigned long long)(half & ((1u << s2) - 1u)) << (16 * nr++);
          rng |= (unsigned long long)(half & ~((1u << s2) - 1u)) << (16 * nr++);
        } else {
          rng |= (unsigned long long)half << (16 * nr++);
        }
      }
    }
    // a block reached by two entries is filtered twice: its tasks are
    // scanned twice, which leaves every minimum unchanged
    for (int e = 0; e < nr; ++e) {
      const unsigned em = (unsigned)(rng >> (16 * e)) & 0xffffu;
      if (!__any(active && ((em >> qi) & 1u))) continue;
      box = make_wave_box(active && ((em >> qi) & 1u), qx, qy, qz, wr);
      walk(c, tl, em);
    }
    tm_walk = (unsigned)__builtin_amdgcn_s_memtime();
    flush_tasks(c, tl);
  }
};

}  // namespace ddlo
