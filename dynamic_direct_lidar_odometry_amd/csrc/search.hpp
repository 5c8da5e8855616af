// search.hpp — exact nearest-neighbour search on gfx950, one wavefront
// cooperating on 64 spatially coherent queries.
//
// Replaces nanoflann's per-query recursive kd-tree descent
// (reference include/nano_gicp/impl/nanoflann_impl.hpp:1495-1566) with a
// divergence-free scheme sized for 64-lane wavefronts:
//   * the cloud is sorted by Morton key and cut into 32-point leaves; each
//     internal level groups 64 nodes, so testing a node's children is ONE
//     wave-wide instruction group (lane c tests child c) + a 64-bit ballot;
//   * the traversal is wave-uniform (node ids live in SGPRs); a node is
//     entered when its box overlaps the union of the lanes' search balls;
//   * a leaf is scanned when ANY lane's exact box distance is within that
//     lane's bound; all 64 lanes then test all 32 points (points are loaded
//     by lanes 0..31 and broadcast with v_readlane).
// Exactness: the squared distance is computed exactly like nanoflann's
// L2_Simple_Adaptor (((q-p)_x^2 + (q-p)_y^2) + (q-p)_z^2 in fp32, no FMA —
// the file is compiled with -ffp-contract=off), box distances use the same
// monotone operation order so they never exceed the distance of a point
// inside the box, and ties are broken by the lower sorted position, so the
// result is the exact minimum of (distance, position) independent of the
// traversal order.
#pragma once
#include <hip/hip_runtime.h>

#include "gicp_types.hpp"

namespace ddlo {

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Global-address-space view of a generic pointer: loads through it compile to
// global_load (counted on vmcnt only) instead of flat_load, whose lgkmcnt
// share would make every scalar-load wait drain the prefetched leaf.
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gp(const T* p) {
  return (const __attribute__((address_space(1))) T*)p;
}
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gpw(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}
typedef float f4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));
// 16-byte global load of a float4 element
__device__ __forceinline__ float4 ldg4(const float4* p, long i) {
  const f4v v = ((const __attribute__((address_space(1))) f4v*)p)[i];
  return make_float4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float uniform_f(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// Wave-wide min/max with DPP (no LDS round trips): quad xor 1 / 2, half-row
// and row mirrors give every lane its 16-lane row's value, then row_bcast15
// / row_bcast31 fold the rows into lane 63, which is read back.
template <bool MAX>
__device__ __forceinline__ float dpp_fold(float v, int ctrl_sel) {
  const int x = __float_as_int(v);
  int r;
  switch (ctrl_sel) {
    case 0: r = __builtin_amdgcn_update_dpp(x, x, 0xb1, 0xf, 0xf, false); break;   // quad_perm [1,0,3,2]
    case 1: r = __builtin_amdgcn_update_dpp(x, x, 0x4e, 0xf, 0xf, false); break;   // quad_perm [2,3,0,1]
    case 2: r = __builtin_amdgcn_update_dpp(x, x, 0x141, 0xf, 0xf, false); break;  // row_half_mirror
    case 3: r = __builtin_amdgcn_update_dpp(x, x, 0x140, 0xf, 0xf, false); break;  // row_mirror
    case 4: r = __builtin_amdgcn_update_dpp(x, x, 0x142, 0xa, 0xf, false); break;  // row_bcast15 -> rows 1, 3
    default: r = __builtin_amdgcn_update_dpp(x, x, 0x143, 0xc, 0xf, false); break; // row_bcast31 -> rows 2, 3
  }
  const float o = __int_as_float(r);
  return MAX ? fmaxf(v, o) : fminf(v, o);
}
template <bool MAX>
__device__ __forceinline__ float wave_fold(float v) {
#pragma unroll
  for (int c = 0; c < 6; ++c) v = dpp_fold<MAX>(v, c);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_min(float v) { return wave_fold<false>(v); }
__device__ __forceinline__ float wave_max(float v) { return wave_fold<true>(v); }

// squared distance, nanoflann L2_Simple_Adaptor order (no contraction)
__device__ __forceinline__ float dist2(float qx, float qy, float qz, float px, float py, float pz) {
  const float dx = qx - px, dy = qy - py, dz = qz - pz;
  return (dx * dx + dy * dy) + dz * dz;
}

// lower bound of dist2 to any point of the box, same monotone op order
__device__ __forceinline__ float box_dist2(float qx, float qy, float qz, float4 lo, float4 hi) {
  const float dx = fmaxf(fmaxf(lo.x - qx, qx - hi.x), 0.f);
  const float dy = fmaxf(fmaxf(lo.y - qy, qy - hi.y), 0.f);
  const float dz = fmaxf(fmaxf(lo.z - qz, qz - hi.z), 0.f);
  return (dx * dx + dy * dy) + dz * dz;
}

// Morton code (21 bits per axis) of a point in a cloud's quantisation.
__device__ __forceinline__ unsigned long long spread21(unsigned int v) {
  unsigned long long x = v & 0x1fffffULL;
  x = (x | (x << 32)) & 0x1f00000000ffffULL;
  x = (x | (x << 16)) & 0x1f0000ff0000ffULL;
  x = (x | (x << 8)) & 0x100f00f00f00f00fULL;
  x = (x | (x << 4)) & 0x10c30c30c30c30c3ULL;
  x = (x | (x << 2)) & 0x1249249249249249ULL;
  return x;
}
__device__ __forceinline__ unsigned int quant21(float v, float lo, float scale) {
  float f = (v - lo) * scale;
  f = fminf(fmaxf(f, 0.f), 2097151.f);
  return (unsigned int)f;
}
__device__ __forceinline__ unsigned long long morton_key(float x, float y, float z, const float* quant) {
  return spread21(quant21(x, quant[0], quant[3])) | (spread21(quant21(y, quant[1], quant[3])) << 1) |
         (spread21(quant21(z, quant[2], quant[3])) << 2);
}

// Key directory of a sorted cloud: dir[p] = first sorted position whose
// Morton key has top kDirBits bits >= p (p = 0 .. 2^kDirBits), so the
// lower_bound of any key lies in [dir[p], dir[p + 1]] for its prefix p.
__device__ __forceinline__ void dir_range(const int* dir, unsigned long long key, int& lo, int& hi) {
  const unsigned p = (unsigned)(key >> (63 - kDirBits));
  lo = gp(dir)[p];
  hi = gp(dir)[p + 1];
}

// Seed position of a key in the sorted keys (a Morton window is centred on
// it): the coarse bucket's range and its fine slot in one round trip, the
// refinement's lower bound in a second.  A bucket of <= kFineMin keys gives
// its middle (the window covers the bucket); an empty bucket gives the exact
// lower bound.  Returns false, with the coarse range, for a bucket without a
// slot (>= 2^16 keys): the caller searches it.
__device__ __forceinline__ bool seed_pos(const int* dir, unsigned long long key, int& pos, int& lo, int& hi) {
  const unsigned c = (unsigned)(key >> (63 - kDirBits));
  const int* fslot = dir + (1 << kDirBits) + 2;
  lo = gp(dir)[c];
  hi = gp(dir)[c + 1];
  const int slot = gp(fslot)[c];
  pos = (lo + hi) >> 1;
  if (hi - lo <= kFineMin) return true;
  if (slot < 0) return false;
  const unsigned short* fine = reinterpret_cast<const unsigned short*>(fslot + (1 << kDirBits));
  const unsigned f = (unsigned)(key >> (63 - kDirBits - kFineBits)) & ((1u << kFineBits) - 1u);
  pos = lo + (int)gp(fine)[((size_t)slot << kFineBits) + f];
  return true;
}

// Wave-parallel lower_bound of a (uniform) key in the sorted key array:
// 64 pivots per step, 4 dependent loads for 500k keys instead of 19.
__device__ __forceinline__ int wave_lower_bound(const unsigned long long* keys, int n, unsigned long long key) {
  int lo = 0, hi = n;  // answer in [lo, hi]
  const int lane = lane_id();
  while (hi - lo > 64) {
    const int step = (hi - lo + 63) / 64;
    const int idx = lo + lane * step;
    const bool less = idx < hi && gp(keys)[idx] < key;
    const int cnt = __popcll(__ballot(less));   // pivots strictly below key
    // answer lies in (lo + (cnt-1)*step, lo + cnt*step]
    const int nlo = cnt == 0 ? lo : lo + (cnt - 1) * step + 1;
    const int nhi = min(hi, lo + cnt * step);
    lo = nlo;
    hi = nhi;
  }
  const int idx = lo + lane;
  const bool less = idx < hi && gp(keys)[idx] < key;
  return lo + __popcll(__ballot(less));
}

// Per-lane lower_bound (divergent keys).
__device__ __forceinline__ int wave_lower_bound_lane(const unsigned long long* keys, int n, unsigned long long key) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (gp(keys)[mid] < key)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// Per-query lower_bound for Q-query groups: the S = 64/Q lanes of a query
// test S pivots per step ((S+1)-ary search), ~log_{S+1}(n) dependent loads.
template <int Q>
__device__ __forceinline__ int group_lower_bound(const unsigned long long* keys, int n, unsigned long long key,
                                                 int lo0 = 0, int hi0 = -1) {
  constexpr int S = 64 / Q;
  const int lane = lane_id();
  const int s = lane / Q, qi = lane % Q;
  int lo = lo0, hi = hi0 < 0 ? n : hi0;  // answer in [lo, hi]
  while (__any(hi - lo > 0)) {
    const int len = hi - lo;
    // pivots lo + (t+1)*len/(S+1), t = 0..S-1
    const int piv = lo + (int)(((long long)(s + 1) * len) / (S + 1));
    const bool less = len > 0 && gp(keys)[min(piv, n - 1)] < key && piv < hi;
    const unsigned long long bal = __ballot(less);
    int cnt = 0;
#pragma unroll
    for (int t = 0; t < S; ++t) cnt += (int)((bal >> (qi + t * Q)) & 1ull);
    if (len > 0) {
      const int nlo = cnt == 0 ? lo : lo + (int)(((long long)cnt * len) / (S + 1)) + 1;
      const int nhi = cnt == S ? hi : lo + (int)(((long long)(cnt + 1) * len) / (S + 1));
      lo = nlo;
      hi = max(nhi, nlo);
      if (hi - lo <= 0) hi = lo;
    }
  }
  return lo;
}

// ---------------------------------------------------------------------------
// Wave box: union over active lanes of the AABB of each lane's search ball.
struct WaveBox {
  float lx, ly, lz, hx, hy, hz;  // uniform values held in VGPRs
};

__device__ __forceinline__ float ball_radius(float bound2) {
  // conservative radius for a squared fp32 bound (covers rounding of the
  // distance evaluation and of q +/- r; coordinates are O(100 m))
  return bound2 < 0.f ? -1.f : sqrtf(bound2) * 1.0001f + 1e-4f;
}

// Squared distance from q to the farthest corner of a box: an upper bound on
// the fp32 squared distance to every point inside (same operation order as
// dist2(), each axis term at least the point's).
__device__ __forceinline__ float box_maxdist2(float qx, float qy, float qz, f4v lo, f4v hi) {
  const float dx = fmaxf(fabsf(qx - lo.x), fabsf(qx - hi.x));
  const float dy = fmaxf(fabsf(qy - lo.y), fabsf(qy - hi.y));
  const float dz = fmaxf(fabsf(qz - lo.z), fabsf(qz - hi.z));
  return (dx * dx + dy * dy) + dz * dz;
}

__device__ __forceinline__ WaveBox make_wave_box(bool active, float qx, float qy, float qz, float bound2) {
  const float r = ball_radius(bound2);
  const bool use = active && r >= 0.f;
  WaveBox b;
  b.lx = wave_min(use ? qx - r : INFINITY);
  b.ly = wave_min(use ? qy - r : INFINITY);
  b.lz = wave_min(use ? qz - r : INFINITY);
  b.hx = wave_max(use ? qx + r : -INFINITY);
  b.hy = wave_max(use ? qy + r : -INFINITY);
  b.hz = wave_max(use ? qz + r : -INFINITY);
  return b;
}

__device__ __forceinline__ bool box_overlap(const WaveBox& w, float4 lo, float4 hi) {
  return lo.x <= w.hx && hi.x >= w.lx && lo.y <= w.hy && hi.y >= w.ly && lo.z <= w.hz && hi.z >= w.lz;
}

// ---------------------------------------------------------------------------
// Per-wavefront LDS slice used by the leaf machinery.  Boxes of the current
// leaf block and the points of the leaf being scanned are broadcast to all
// lanes with ds_read_b128 (every lane reads the same address: conflict-free),
// which keeps the uniform data in VGPRs instead of SGPRs.
struct WaveLds {
  f4v blo[kFanout];          // leaf-block boxes
  f4v bhi[kFanout];
  float px[kLeafSize];       // current leaf, SoA
  float py[kLeafSize];
  float pz[kLeafSize];
};
constexpr int kWaveLdsBytes = sizeof(WaveLds);

// ---------------------------------------------------------------------------
// Generic cooperative traversal.  Visitor V provides:
//   WaveBox box;                                  current wave box (VGPR-uniform)
//   bool need(float4 lo, float4 hi)               per-lane exact leaf test
//   void process(const WaveLds*, int start)       scan the 32 staged points
//   float bound()                                 per-lane squared bound
//   bool active; float qx, qy, qz; int skip_lo, skip_hi;
//
// Leaves are handled a block at a time (the <= 64 children of one level-1
// node): lane c loads leaf c's box into LDS, the wave-box filter and then the
// EXACT per-lane filter run on the staged boxes, and the surviving leaves are
// scanned with the next leaf's points prefetched into registers, so a
// wavefront keeps one global load in flight instead of a dependent chain.
// Clouds are padded to a multiple of 32 with far sentinel points, so a scan
// never needs a per-point bound check.
template <class V>
__device__ __forceinline__ void stage_points(WaveLds* L, float4 p) {
  const int lane = lane_id();
  if (lane < kLeafSize) {
    L->px[lane] = p.x;
    L->py[lane] = p.y;
    L->pz[lane] = p.z;
  }
}

template <class V>
__device__ __forceinline__ void leaf_block(const CloudDev& c, int base, int cnt, V& vis, WaveLds* L) {
  const int lane = lane_id();
  bool ov = false;
  if (lane < cnt) {
    const float4 lo = ldg4(c.box_lo, base + lane);
    const float4 hi = ldg4(c.box_hi, base + lane);
    L->blo[lane] = f4v{lo.x, lo.y, lo.z, 0.f};
    L->bhi[lane] = f4v{hi.x, hi.y, hi.z, 0.f};
    ov = box_overlap(vis.box, lo, hi) && !(base + lane >= vis.skip_lo && base + lane <= vis.skip_hi);
  }
  vis.prof_mark(3);
  unsigned long long mask = __ballot(ov);
  vis.st_blocks += 1;
  vis.st_box += __popcll(mask);
  unsigned long long ex = 0ull;
  const float before = vis.bound();
  // two leaves per step: both boxes read from LDS together (one LDS round
  // trip per pair), then tested in leaf order as before
  while (mask) {
    const int b = __builtin_ctzll(mask);
    mask &= mask - 1;
    const int b2 = mask ? __builtin_ctzll(mask) : b;
    if (mask) mask &= mask - 1;
    const f4v blo = L->blo[b], bhi = L->bhi[b];
    const f4v blo2 = L->blo[b2], bhi2 = L->bhi[b2];
    vis.note_leaf(blo, bhi, base + b);   // a visitor may tighten its bound from the box alone
    if (__any(vis.active && vis.need(make_float4(blo.x, blo.y, blo.z, 0.f), make_float4(bhi.x, bhi.y, bhi.z, 0.f))))
      ex |= 1ull << b;
    if (b2 != b) {
      vis.note_leaf(blo2, bhi2, base + b2);
      if (__any(vis.active && vis.need(make_float4(blo2.x, blo2.y, blo2.z, 0.f), make_float4(bhi2.x, bhi2.y, bhi2.z, 0.f))))
        ex |= 1ull << b2;
    }
  }
  vis.st_exact += __popcll(ex);
  bool shrink = __any(vis.bound() < before);   // tightened by a box: later blocks see the smaller wave box
  vis.prof_mark(4);
  if (ex) shrink |= vis.scan_leaves(c, base, ex, L);
  if (shrink) vis.box = make_wave_box(vis.active, vis.qx, vis.qy, vis.qz, vis.bound());
}

// Generic LDS-staged, prefetching scan of the leaves in `ex` (bit b = leaf
// base + b) used by visitors whose process() reads the staged SoA points.
// Rotated pipeline: at the top of each step the only load in flight is the
// one being consumed, the next leaf's load is issued before the scan.
template <class V>
__device__ __forceinline__ bool scan_leaves_lds(const CloudDev& c, int base, unsigned long long ex, V& vis, WaveLds* L) {
  const int lane = lane_id();
  int nxt = __builtin_ctzll(ex);
  ex &= ex - 1;
  float4 pn = make_float4(0.f, 0.f, 0.f, 0.f);
  if (lane < kLeafSize) pn = ldg4(c.pts, (base + nxt) * kLeafSize + lane);
  bool improved = false;
  while (nxt >= 0) {
    const int cur = nxt;
    const float4 p = pn;
    nxt = -1;
    if (ex) {
      nxt = __builtin_ctzll(ex);
      ex &= ex - 1;
      if (lane < kLeafSize) pn = ldg4(c.pts, (base + nxt) * kLeafSize + lane);
    }
    const f4v blo = L->blo[cur], bhi = L->bhi[cur];
    if (__any(vis.active && vis.need(make_float4(blo.x, blo.y, blo.z, 0.f), make_float4(bhi.x, bhi.y, bhi.z, 0.f)))) {
      const float before = vis.bound();
      vis.st_scan += 1;
      vis.prof_mark(0);
      stage_points<V>(L, p);
      vis.prof_mark(1);
      vis.process(L, (base + cur) * kLeafSize);
      vis.prof_mark(2);
      improved |= __any(vis.bound() < before);
    }
  }
  return improved;
}

// Depth-first walk with an explicit per-level stack of child masks (uniform
// values: scalar registers), so leaf_block — and the visitor's scan it
// inlines — has ONE call site whatever the depth (the kernels must stay
// small enough for the instruction cache).  A single-level cloud is walked
// as the children of a virtual level-1 node 0.
template <class V>
__device__ __forceinline__ void traverse(const CloudDev& c, V& vis, WaveLds* L) {
  const int T = c.nlevels - 1;
  const int Tt = T < 1 ? 1 : T;
  const int lane = lane_id();
  unsigned long long m1 = 0, m2 = 0, m3 = 0, m4 = 0;
  int b1 = 0, b2 = 0, b3 = 0;
  if (T == 0) {
    m1 = 1ull;
  } else {
    bool ov = false;
    if (lane < lvl_cnt(c, T)) {
      const int o = lvl_off(c, T) + lane;
      ov = box_overlap(vis.box, ldg4(c.box_lo, o), ldg4(c.box_hi, o));
    }
    const unsigned long long m = __ballot(ov);
    if (T == 1) m1 = m; else if (T == 2) m2 = m; else if (T == 3) m3 = m; else m4 = m;
  }
  int lv = Tt;
  while (true) {
    unsigned long long m = lv == 1 ? m1 : lv == 2 ? m2 : lv == 3 ? m3 : m4;
    if (m == 0ull) {
      if (lv == Tt) break;
      ++lv;
      continue;
    }
    const int base = lv == 1 ? b1 : lv == 2 ? b2 : lv == 3 ? b3 : 0;
    const int node = base + __builtin_ctzll(m);
    m &= m - 1;
    if (lv == 1) m1 = m; else if (lv == 2) m2 = m; else if (lv == 3) m3 = m; else m4 = m;
    const int cb = node * kFanout;
    const int cnt = min(kFanout, lvl_cnt(c, lv - 1) - cb);
    if (lv == 1) {
      leaf_block(c, cb, cnt, vis, L);
      continue;
    }
    bool ov = false;
    if (lane < cnt) {
      const int o = lvl_off(c, lv - 1) + cb + lane;
      ov = box_overlap(vis.box, ldg4(c.box_lo, o), ldg4(c.box_hi, o));
    }
    const unsigned long long cm = __ballot(ov);
    --lv;
    if (lv == 1) { m1 = cm; b1 = cb; } else if (lv == 2) { m2 = cm; b2 = cb; } else { m3 = cm; b3 = cb; }
  }
}

struct VisitStats {
  unsigned st_blocks = 0, st_box = 0, st_exact = 0, st_scan = 0, st_splits = 0;
  // developer timing hook (k_covariances2's -DDDLO_COV_PROF build): 0 before a
  // leaf's points are staged, 1 after, 2 after its scan; 3 / 4 around a leaf
  // block's box tests
  __device__ __forceinline__ void prof_mark(int) {}
};

// ---------------------------------------------------------------------------
// Compact sub-groups.  A wavefront's 64 queries are consecutive in Morton
// order, which is spatially compact except where the Z-curve jumps: a group
// straddling a jump has a union box of tens of metres and would drag
// thousands of leaves through the filters.  split_search() measures the union
// box and, if it exceeds kSplitExtent, splits the lane range at its largest
// Morton jump (at most twice => <= 4 sub-groups), searching each sub-range
// with the other lanes inactive.  `key` is the lane's Morton key in the
// query cloud's own quantisation (rigid transforms keep the geometry).
constexpr float kSplitExtent = 5.0f;   // tuned on cfg3 (3 m: 0.59, 5 m: 0.50, 10 m: 0.52 ms/scan)

template <int Q = 64>
__device__ __forceinline__ int morton_jump_split(unsigned long long key, int lo, int hi) {
  // query index (lane % Q) with the largest (key ^ previous key) in (lo, hi)
  const int lane = lane_id();
  const int qi = lane % Q;
  // previous lane's key by DPP wave_shr:1 (no LDS-permute address registers)
  const unsigned plo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)key, 0x138, 0xf, 0xf, false);
  const unsigned phi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(key >> 32), 0x138, 0xf, 0xf, false);
  const unsigned long long prev = ((unsigned long long)phi << 32) | plo;
  int score = -1;
  if (lane < Q && qi > lo && qi < hi) score = (64 - __clzll(key ^ prev)) * 64 + qi;
  const int best = (int)wave_max((float)score);   // |score| < 2^13: exact in fp32
  return best < 0 ? (lo + hi) / 2 : (best & 63);
}

template <int Q, class V>
__device__ __forceinline__ void search_range(const CloudDev& c, V& vis, bool base_active, int lo, int hi, WaveLds* L) {
  const int qi = lane_id() % Q;
  vis.active = base_active && qi >= lo && qi < hi;
  vis.box = make_wave_box(vis.active, vis.qx, vis.qy, vis.qz, vis.bound());
  traverse(c, vis, L);
}

__device__ __forceinline__ float box_extent(const WaveBox& b) {
  return fmaxf(fmaxf(b.hx - b.lx, b.hy - b.ly), b.hz - b.lz);
}

template <class V, int Q = 64>
__device__ __forceinline__ void split_search(const CloudDev& c, V& vis, unsigned long long key, WaveLds* L) {
  const bool base_active = vis.active;
  const int qi = lane_id() % Q;
  // sub-ranges as a list of cut points (8 bits each): [cut_r, cut_{r+1})
  unsigned long long cuts = (unsigned long long)Q << 8;   // {0, Q}: the whole group
  int ncut = 2;
  const WaveBox whole = make_wave_box(base_active, vis.qx, vis.qy, vis.qz, vis.bound());
  if (box_extent(whole) > kSplitExtent) {
    vis.st_splits += 1;
    const int sp = morton_jump_split<Q>(key, 0, Q);
    cuts = 0;
    ncut = 1;
    for (int h = 0; h < 2; ++h) {
      const int lo = h == 0 ? 0 : sp, hi = h == 0 ? sp : Q;
      if (lo < hi) {
        const bool act = base_active && qi >= lo && qi < hi;
        const WaveBox hb = make_wave_box(act, vis.qx, vis.qy, vis.qz, vis.bound());
        if (box_extent(hb) > kSplitExtent && hi - lo > 4) {
          vis.st_splits += 1;
          cuts |= (unsigned long long)morton_jump_split<Q>(key, lo, hi) << (8 * ncut);
          ++ncut;
        }
      }
      cuts |= (unsigned long long)hi << (8 * ncut);
      ++ncut;
    }
  }
  // one traversal site for every sub-range
  for (int r = 0; r + 1 < ncut; ++r) {
    const int lo = (int)((cuts >> (8 * r)) & 0xff), hi = (int)((cuts >> (8 * (r + 1))) & 0xff);
    if (lo >= hi) continue;
    const bool act = base_active && qi >= lo && qi < hi;
    if (!__any(act)) continue;
    vis.active = act;
    vis.box = make_wave_box(act, vis.qx, vis.qy, vis.qz, vis.bound());
    traverse(c, vis, L);
  }
  vis.active = base_active;
}

// (squared distance, sorted position) as one order-preserving 64-bit key:
// non-negative fp32 bit patterns sort like their values, so the exact
// lexicographic rule (d < b) || (d == b && j < bj) is one u64 compare.
__device__ __forceinline__ unsigned long long dkey(float d, int j) {
  return ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)j;
}

typedef float f2v __attribute__((ext_vector_type(2)));

// 1-NN visitor for Q queries per wavefront: lane = (query lane % Q, slice
// lane / Q); each of the S = 64/Q slices scans 32/S of a leaf's points and
// the per-query partial minima are merged after every leaf, so every lane of
// a query always holds the query's exact running (best, bestj).
// u64 min across lanes l and l ^ 32 / l ^ 16 with the gfx950 permlane swaps
// (register-only; no LDS round trip)
__device__ __forceinline__ unsigned long long umin64(unsigned long long a, unsigned long long b) { return a < b ? a : b; }
template <int M>
__device__ __forceinline__ unsigned long long xor_min64(unsigned long long v) {
  const unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
  unsigned a0, a1, b0, b1;
  if constexpr (M == 32) {
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a0 = rl[0]; b0 = rl[1]; a1 = rh[0]; b1 = rh[1];
  } else if constexpr (M == 16) {
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    a0 = rl[0]; b0 = rl[1]; a1 = rh[0]; b1 = rh[1];
  } else {
    return umin64(v, __shfl_xor(v, M));
  }
  return umin64(((unsigned long long)a1 << 32) | a0, ((unsigned long long)b1 << 32) | b0);
}

// the mirrored key of tie_scan 3: same distance, complemented position
__device__ __forceinline__ unsigned long long mirror_key(unsigned long long k) { return k ^ 0xffffffffull; }

// xor_min64 that also records in td the distance of two lanes' keys that are
// equal in distance (two distinct points: a tie at that distance)
template <int M>
__device__ __forceinline__ unsigned long long xor_min64_eq(unsigned long long v, unsigned& td) {
  static_assert(M == 16 || M == 32, "xor_min64_eq: M = 16 or 32");
  const unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
  unsigned a0, a1, b0, b1;
  if constexpr (M == 32) {
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a0 = rl[0]; b0 = rl[1]; a1 = rh[0]; b1 = rh[1];
  } else {
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    a0 = rl[0]; b0 = rl[1]; a1 = rh[0]; b1 = rh[1];
  }
  td = a1 == b1 ? min(td, a1) : td;   // the lanes hold disjoint points: equal distances are two points
  return umin64(((unsigned long long)a1 << 32) | a0, ((unsigned long long)b1 << 32) | b0);
}

// xor_min64 carrying the winning key's point coordinates along (lanes l and
// l ^ M; equal keys name the same point)
template <int M>
__device__ __forceinline__ void xor_min64_xyz(unsigned long long& v, float& x, float& y, float& z) {
  static_assert(M == 16 || M == 32, "xor_min64_xyz: M = 16 or 32");
  const unsigned in[5] = {(unsigned)v, (unsigned)(v >> 32), __float_as_uint(x), __float_as_uint(y), __float_as_uint(z)};
  unsigned a[5], b[5];
#pragma unroll
  for (int e = 0; e < 5; ++e) {
    if constexpr (M == 32) {
      const auto r = __builtin_amdgcn_permlane32_swap(in[e], in[e], false, false);
      a[e] = r[0]; b[e] = r[1];
    } else {
      const auto r = __builtin_amdgcn_permlane16_swap(in[e], in[e], false, false);
      a[e] = r[0]; b[e] = r[1];
    }
  }
  const unsigned long long ka = ((unsigned long long)a[1] << 32) | a[0], kb = ((unsigned long long)b[1] << 32) | b[0];
  const bool ta = ka < kb;
  v = ta ? ka : kb;
  x = __uint_as_float(ta ? a[2] : b[2]);
  y = __uint_as_float(ta ? a[3] : b[3]);
  z = __uint_as_float(ta ? a[4] : b[4]);
}

// squared distance of a (distance, position) key
__device__ __forceinline__ float key_dist(unsigned long long k) { return __uint_as_float((unsigned)(k >> 32)); }
// a key names a real point (not a bound without one: position 0xffffffff)
__device__ __forceinline__ bool key_real(unsigned long long k) { return (unsigned)k != 0xffffffffu; }

// Top-2 merge across lanes l and l ^ M (M = 16 / 32, permlane swaps): k =
// the smaller key of the two lanes, sd = the smallest distance of every
// other point either lane holds (both seconds and the larger key).  The two
// lanes hold disjoint point sets.
template <int M>
__device__ __forceinline__ void xor_top2(unsigned long long& k, float& sd) {
  const unsigned lo = (unsigned)k, hi = (unsigned)(k >> 32), sb = __float_as_uint(sd);
  unsigned a0, a1, b0, b1, s0, s1;
  if constexpr (M == 32) {
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const auto rs = __builtin_amdgcn_permlane32_swap(sb, sb, false, false);
    a0 = rl[0]; b0 = rl[1]; a1 = rh[0]; b1 = rh[1]; s0 = rs[0]; s1 = rs[1];
  } else {
    static_assert(M == 16, "xor_top2: M = 16 or 32");
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const auto rs = __builtin_amdgcn_permlane16_swap(sb, sb, false, false);
    a0 = rl[0]; b0 = rl[1]; a1 = rh[0]; b1 = rh[1]; s0 = rs[0]; s1 = rs[1];
  }
  const unsigned long long ka = ((unsigned long long)a1 << 32) | a0, kb = ((unsigned long long)b1 << 32) | b0;
  const unsigned long long kmax = ka < kb ? kb : ka;
  sd = fminf(fminf(__uint_as_float(s0), __uint_as_float(s1)), key_dist(kmax));
  k = umin64(ka, kb);
}

typedef float f3v __attribute__((ext_vector_type(3)));
__device__ __forceinline__ f3v ldg3(const float4* p, long i) {
  return ((const __attribute__((address_space(1))) f3v*)(p + i))[0];
}

// 1-NN visitor for Q queries per wavefront: lane = (query lane % Q, slice
// lane / Q); each of the S = 64/Q slices loads and scans 32/S of a leaf's
// points straight into registers (next leaf prefetched), and the per-query
// partial minima are merged after every leaf with permlane swaps, so every
// lane of a query always holds the query's exact running (best, bestj).
template <int Q>
struct NNVisitor : VisitStats {
  static constexpr int S = 64 / Q;
  static constexpr int P = kLeafSize / S;   // points per lane per leaf
  WaveBox box;
  float qx, qy, qz;
  float best;   // squared distance bound (strict <, ties by position)
  int bestj;    // sorted position, -1 none
  bool active;
  int skip_lo, skip_hi;  // leaves already scanned (seeding), uniform

  __device__ __forceinline__ float bound() const { return best; }
  __device__ __forceinline__ bool need(float4 lo, float4 hi) const { return box_dist2(qx, qy, qz, lo, hi) <= best; }
  __device__ __forceinline__ void note_leaf(f4v, f4v, int) {}

  __device__ __forceinline__ void merge_slices(unsigned long long& bk) const {
    if constexpr (Q <= 16) bk = xor_min64<16>(bk);
    if constexpr (Q <= 32) bk = xor_min64<32>(bk);
    if constexpr (Q < 16) {
#pragma unroll
      for (int m = Q; m < 16; m <<= 1) bk = umin64(bk, __shfl_xor(bk, m));
    }
  }

  __device__ __forceinline__ void scan_regs(const f3v (&pt)[P], int start) {
    unsigned long long bk = dkey(best, bestj);
    const int off = (lane_id() / Q) * P;
    const f2v qx2 = {qx, qx}, qy2 = {qy, qy}, qz2 = {qz, qz};
#pragma unroll
    for (int h = 0; h < P; h += 2) {
      // two points at once (v_pk_* ops), same IEEE ops as dist2()
      const f2v dx = qx2 - f2v{pt[h].x, pt[h + 1].x};
      const f2v dy = qy2 - f2v{pt[h].y, pt[h + 1].y};
      const f2v dz = qz2 - f2v{pt[h].z, pt[h + 1].z};
      const f2v d = (dx * dx + dy * dy) + dz * dz;
      const int pj = start + off + h;
      bk = umin64(bk, dkey(d.x, pj));
      bk = umin64(bk, dkey(d.y, pj + 1));
    }
    merge_slices(bk);
    if (active) {
      best = __uint_as_float((unsigned)(bk >> 32));
      bestj = (int)(unsigned)bk;
    }
  }

  __device__ __forceinline__ void load_leaf(const CloudDev& c, int leaf, f3v (&pt)[P]) const {
    const long b = (long)leaf * kLeafSize + (lane_id() / Q) * P;
#pragma unroll
    for (int h = 0; h < P; ++h) pt[h] = ldg3(c.pts, b + h);
  }

  __device__ __forceinline__ bool scan_leaves(const CloudDev& c, int base, unsigned long long ex, WaveLds*) {
    int nxt = base + __builtin_ctzll(ex);
    ex &= ex - 1;
    f3v pn[P];
    load_leaf(c, nxt, pn);
    bool improved = false;
    while (nxt >= 0) {
      const int cur = nxt;
      f3v p[P];
#pragma unroll
      for (int h = 0; h < P; ++h) p[h] = pn[h];
      nxt = -1;
      if (ex) {
        nxt = base + __builtin_ctzll(ex);
        ex &= ex - 1;
        load_leaf(c, nxt, pn);
      }
      const float before = best;
      st_scan += 1;
      scan_regs(p, cur * kLeafSize);
      improved |= __any(best < before);
    }
    return improved;
  }

  __device__ __forceinline__ void scan_leaf(const CloudDev& c, int leaf, WaveLds*) {
    f3v p[P];
    load_leaf(c, leaf, p);
    scan_regs(p, leaf * kLeafSize);
  }
};
using NN1Visitor = NNVisitor<64>;


}  // namespace ddlo

namespace ddlo {

// Upper levels of a cloud's hierarchy, cached in LDS by the correspondence
// walk (nn_tasks.hpp).
__device__ __forceinline__ int upper_count(const CloudDev& c) {
  return c.nlevels <= 1 ? 0 : (lvl_off(c, c.nlevels - 1) + lvl_cnt(c, c.nlevels - 1) - c.off1);
}

// Upper-level box cache shared by a workgroup: boxes of levels >= 1 in the
// cloud's level order (index = global box index - lvl_off(c, 1)); lo at
// [0, n), hi at [n, 2n).  Cooperative fill by the whole workgroup.
__device__ __forceinline__ void fill_upper(const CloudDev& c, f4v* U) {
  const int n = upper_count(c);
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const float4 lo = ldg4(c.box_lo, c.off1 + k), hi = ldg4(c.box_hi, c.off1 + k);
    U[k] = f4v{lo.x, lo.y, lo.z, 0.f};
    U[n + k] = f4v{hi.x, hi.y, hi.z, 0.f};
  }
}

__device__ __forceinline__ bool box_overlap_v(const WaveBox& w, f4v lo, f4v hi) {
  return lo.x <= w.hx && hi.x >= w.lx && lo.y <= w.hy && hi.y >= w.ly && lo.z <= w.hz && hi.z >= w.lz;
}


}  // namespace ddlo
