// kernels.hip — hand-written gfx950 kernels of the GICP hot path.
//
//   K1 index build      k_pack_bbox, k_bbox_final, k_morton, k_gather,
//                       k_leaf_soa_boxes, k_level_boxes   (radix sort: hipcub, capi.hip)
//   K2 kNN-k covariance k_covariances<KCAP,EXACT>        calculate_covariances
//                                                       nano_gicp_impl.hpp:373-441
//   K3 correspondences  k_cell_lookup (candidate cells,  update_correspondences
//                       cellgrid.hip), k_nn_seed +      :234-275 (1-NN part)
//                       k_nn_scan (the walk)
//   K4 moments          k_moments                       update_correspondences
//                                                       (M) + linearize :277-336
//   K5 LM / GN step     k_lm_step                       lsq_registration_impl.hpp:95-232
//                                                       (+ compute_error :339-383
//                                                       evaluated from the moments)
//   K6 outputs          k_residuals, k_transform,       getResiduals :225-232,
//                       k_export_corr                   transformPointCloud lsq:125
// Compiled with -ffp-contract=off: fp32 distance / transform arithmetic must
// not be contracted into FMAs so that correspondences equal the oracle's.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdlib>
#include <cstring>

#include "gicp_types.hpp"
#include "search.hpp"
#include "nn_tasks.hpp"
#include "nftree.hpp"
#include "cov_math.hpp"
#include "launch.hpp"
#include "devknobs.hpp"

#include <algorithm>

namespace ddlo {

// ============================================================================
// K1: cloud packing, bbox, Morton keys, hierarchy boxes
// ============================================================================
__global__ __launch_bounds__(256) void k_pack_bbox(const unsigned char* __restrict__ raw, size_t stride, int n,
                                                   float4* __restrict__ out, float* __restrict__ partial,
                                                   int* __restrict__ nonfinite) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float x = 0.f, y = 0.f, z = 0.f;
  bool ok = false;
  if (i < n) {
    const float* p = reinterpret_cast<const float*>(raw + (size_t)i * stride);
    x = p[0];
    y = p[1];
    z = p[2];
    ok = isfinite(x) && isfinite(y) && isfinite(z);
    out[i] = make_float4(x, y, z, __int_as_float(i));
  }
  // one flag write per wavefront holding a non-finite point (one word takes ~88 atomics per us)
  const unsigned long long bad = __ballot(i < n && !ok);
  if (bad && __lane_id() == (unsigned)__builtin_ctzll(bad)) atomicOr(nonfinite, 1);
  __shared__ float red[6][4];
  float v[6] = {ok ? x : INFINITY, ok ? y : INFINITY, ok ? z : INFINITY,
                ok ? x : -INFINITY, ok ? y : -INFINITY, ok ? z : -INFINITY};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    v[a] = wave_min(v[a]);
    v[a + 3] = wave_max(v[a + 3]);
  }
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0)
    for (int a = 0; a < 6; ++a) red[a][w] = v[a];
  __syncthreads();
  if (threadIdx.x < 6) {
    const int a = threadIdx.x;
    float r = red[a][0];
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) r = a < 3 ? fminf(r, red[a][k]) : fmaxf(r, red[a][k]);
    partial[blockIdx.x * 6 + a] = r;
  }
}

__global__ __launch_bounds__(256) void k_bbox_final(const float* __restrict__ partial, int nparts,
                                                    float* __restrict__ quant) {
  // one block of 256 threads: strided partial min/max, then wave + LDS reduce
  __shared__ float red[6][4];
  __shared__ float bb[6];
  float v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int k = threadIdx.x; k < nparts; k += blockDim.x) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      v[a] = fminf(v[a], partial[k * 6 + a]);
      v[a + 3] = fmaxf(v[a + 3], partial[k * 6 + a + 3]);
    }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    v[a] = wave_min(v[a]);
    v[a + 3] = wave_max(v[a + 3]);
  }
  if (lane_id() == 0)
    for (int a = 0; a < 6; ++a) red[a][threadIdx.x >> 6] = v[a];
  __syncthreads();
  if (threadIdx.x < 6) {
    const int a = threadIdx.x;
    float r = red[a][0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = a < 3 ? fminf(r, red[a][w]) : fmaxf(r, red[a][w]);
    bb[a] = r;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float ext = fmaxf(fmaxf(bb[3] - bb[0], bb[4] - bb[1]), bb[5] - bb[2]);
    quant[0] = bb[0];
    quant[1] = bb[1];
    quant[2] = bb[2];
    quant[3] = ext > 0.f ? 2097151.f / ext : 1.f;
    quant[4] = bb[3];
    quant[5] = bb[4];
    quant[6] = bb[5];
  }
}

__global__ __launch_bounds__(256) void k_morton(const float4* __restrict__ pts, int n, const float* __restrict__ quant,
                                                unsigned long long* __restrict__ keys, int* __restrict__ vals) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = pts[i];
  keys[i] = morton_key(p.x, p.y, p.z, quant);
  vals[i] = i;
}

// Sorted gather; positions [n, npad) get far sentinels (squared distance
// ~3e36 to any real point) so leaf scans never need a bound check.
constexpr float kFar = 1e18f;
__global__ __launch_bounds__(256) void k_gather(const float4* __restrict__ raw, const int* __restrict__ perm, int n,
                                                int npad, float4* __restrict__ sorted, int* __restrict__ inv_perm) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npad) return;
  if (i >= n) {
    sorted[i] = make_float4(kFar, kFar, kFar, __int_as_float(-1));
    return;
  }
  const int o = perm[i];
  sorted[i] = raw[o];
  inv_perm[o] = i;
}

// one 32-lane half-wave per leaf
// Key directory (search.hpp dir_range): thread i of the sorted keys fills
// the prefixes in (prefix(i - 1), prefix(i)] with i; the last thread also
// fills the prefixes past the largest key with n.
__global__ __launch_bounds__(256) void k_key_dir(const unsigned long long* __restrict__ keys, int n, int* __restrict__ dir) {
  // dir[p] = first sorted position whose top kDirBits Morton bits are >= p
  // (p in [0, 2^kDirBits]); one thread per entry, a lower-bound search each,
  // so empty stretches of the Morton space cost no serial fill
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p > (1 << kDirBits)) return;
  constexpr int sh = 63 - kDirBits;
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((long)(keys[mid] >> sh) < (long)p) lo = mid + 1;
    else hi = mid;
  }
  dir[p] = lo;
}

// Fine directory: a bucket of more than kFineMin keys (and fewer than 2^16)
// takes a slot, and lane f of the wavefront refining it stores the lower
// bound of refinement f (the next kFineBits Morton bits) relative to the
// bucket start.  Two launches: k_key_big (a lane per bucket) assigns the
// slots and leaves each slot's bucket in the slot's first int; k_key_fine (a
// wavefront per possible slot) refines.  A wavefront per bucket spent ~30 us
// per cloud launching 2^18 mostly idle wavefronts.  Slot order depends on
// scheduling, the contents do not.
__global__ __launch_bounds__(256) void k_key_big(int* __restrict__ dir) {
  const int c = (int)blockIdx.x * blockDim.x + (int)threadIdx.x;
  if (c >= (1 << kDirBits)) return;
  int* const ctr = dir + (1 << kDirBits) + 1;
  int* const fslot = ctr + 1;
  unsigned short* const fine = reinterpret_cast<unsigned short*>(fslot + (1 << kDirBits));
  const int nk = dir[c + 1] - dir[c];
  const bool big = nk > kFineMin && nk <= 65535;
  const unsigned long long m = __ballot(big);
  int base = 0;
  if (m) {
    if (lane_id() == __builtin_ctzll(m)) base = atomicAdd(ctr, __popcll(m));
    base = __shfl(base, __builtin_ctzll(m));
  }
  int slot = -1;
  if (big) {
    slot = base + __popcll(m & ((1ull << lane_id()) - 1));
    reinterpret_cast<int*>(fine + ((size_t)slot << kFineBits))[0] = c;
  }
  fslot[c] = slot;
}

__global__ __launch_bounds__(256) void k_key_fine(const unsigned long long* __restrict__ keys, int* __restrict__ dir) {
  const int slot = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  const int lane = lane_id();
  int* const ctr = dir + (1 << kDirBits) + 1;
  if (slot >= __builtin_amdgcn_readfirstlane(*ctr)) return;
  int* const fslot = ctr + 1;
  unsigned short* const fine = reinterpret_cast<unsigned short*>(fslot + (1 << kDirBits));
  const int c = __builtin_amdgcn_readfirstlane(reinterpret_cast<const int*>(fine + ((size_t)slot << kFineBits))[0]);
  const int lo = dir[c], hi = dir[c + 1];
  constexpr int sh = 63 - kDirBits - kFineBits;
  const unsigned long long want = ((unsigned long long)c << kFineBits) | (unsigned long long)lane;
  int a = lo, b = hi;
  while (a < b) {
    const int mid = (a + b) >> 1;
    if ((keys[mid] >> sh) < want) a = mid + 1;
    else b = mid;
  }
  __builtin_amdgcn_wave_barrier();   // every lane has read the slot's bucket id before lanes 0-1 overwrite it
  fine[((size_t)slot << kFineBits) + lane] = (unsigned short)(a - lo);
}

// Per-leaf SoA copy of the sorted points (leaf l = x[32], y[32], z[32], so
// that a lane's 8 consecutive coordinates are two 16-B loads per axis and
// pairs of them feed the packed-math distance directly, k_nn_scan) and each
// leaf's box over its real points, in one pass: thread = sorted position,
// 32 threads per leaf (8 leaves per block).
__global__ __launch_bounds__(256) void k_leaf_soa_boxes(const float4* __restrict__ pts, int n, int nleaves,
                                                        float* __restrict__ soa, float4* __restrict__ lo,
                                                        float4* __restrict__ hi) {
  const int leaf = blockIdx.x * 8 + (threadIdx.x >> 5);
  const int sub = threadIdx.x & 31;
  const int p = leaf * kLeafSize + sub;
  float v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  if (leaf < nleaves) {   // the sentinel-padded positions of the last leaf are copied too
    const float4 q = pts[p];
    float* o = soa + (size_t)leaf * 3 * kLeafSize;
    o[sub] = q.x;
    o[kLeafSize + sub] = q.y;
    o[2 * kLeafSize + sub] = q.z;
    if (p < n) {
      v[0] = v[3] = q.x;
      v[1] = v[4] = q.y;
      v[2] = v[5] = q.z;
    }
  }
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      v[a] = fminf(v[a], __shfl_xor(v[a], m));
      v[a + 3] = fmaxf(v[a + 3], __shfl_xor(v[a + 3], m));
    }
  }
  if (sub == 0 && leaf < nleaves) {
    lo[leaf] = make_float4(v[0], v[1], v[2], 0.f);
    hi[leaf] = make_float4(v[3], v[4], v[5], 0.f);
  }
}

// one wavefront per parent node, lane = child
__global__ __launch_bounds__(256) void k_level_boxes(const float4* __restrict__ clo, const float4* __restrict__ chi,
                                                     int nchild, int nparent, float4* __restrict__ plo,
                                                     float4* __restrict__ phi) {
  const int parent = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int c = parent * kFanout + lane_id();
  float v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  if (parent < nparent && c < nchild) {
    const float4 a = clo[c], b = chi[c];
    v[0] = a.x; v[1] = a.y; v[2] = a.z;
    v[3] = b.x; v[4] = b.y; v[5] = b.z;
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    v[a] = wave_min(v[a]);
    v[a + 3] = wave_max(v[a + 3]);
  }
  if (lane_id() == 0 && parent < nparent) {
    plo[parent] = make_float4(v[0], v[1], v[2], 0.f);
    phi[parent] = make_float4(v[3], v[4], v[5], 0.f);
  }
}

// ============================================================================
// K2: exact kNN-k (self queries) + covariance
// ============================================================================
// Kept-neighbour list storage: registers, or (KLDS: k up to 64, where a
// register list of 64 u64 keys spilled 213 VGPRs) a lane-interleaved LDS
// array, slot s of a lane at p[64 s].
template <int KCAP, bool KLDS>
struct KeyList {
  unsigned long long v[KCAP];
  __device__ __forceinline__ unsigned long long& operator[](int s) { return v[s]; }
  __device__ __forceinline__ const unsigned long long& operator[](int s) const { return v[s]; }
};
template <int KCAP>
struct KeyList<KCAP, true> {
  unsigned long long* p;   // the lane's slot 0 (LDS)
  __device__ __forceinline__ unsigned long long& operator[](int s) { return p[64 * s]; }
  __device__ __forceinline__ const unsigned long long& operator[](int s) const { return p[64 * s]; }
};

// Compare-exchange of two 64-bit keys: slot = min(key, slot), key = the
// larger, from ONE compare.  Written out because the compiler turns the two
// selects of one predicate into umin + umax and lowers each with its own
// 64-bit compare (9 instructions and a twice as long dependent chain per slot
// of the insertion network that bounds a kNN leaf scan).  The s_nop covers the
// VALU-writes-VCC -> v_cndmask hazard, as the compiler's own code does.
__device__ __forceinline__ void cmp_exchange_u64(unsigned long long& key, unsigned long long& slot) {
  const unsigned long long a = key, b = slot;
  unsigned lo0, lo1, hi0, hi1;
  asm volatile(
      "v_cmp_lt_u64_e32 vcc, %[a], %[b]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_e32 %[lo0], %[b0], %[a0], vcc\n\t"
      "v_cndmask_b32_e32 %[lo1], %[b1], %[a1], vcc\n\t"
      "v_cndmask_b32_e32 %[hi0], %[a0], %[b0], vcc\n\t"
      "v_cndmask_b32_e32 %[hi1], %[a1], %[b1], vcc"
      : [lo0] "=&v"(lo0), [lo1] "=&v"(lo1), [hi0] "=&v"(hi0), [hi1] "=&v"(hi1)
      : [a] "v"(a), [b] "v"(b), [a0] "v"((unsigned)a), [a1] "v"((unsigned)(a >> 32)), [b0] "v"((unsigned)b),
        [b1] "v"((unsigned)(b >> 32))
      : "vcc");
  slot = ((unsigned long long)lo1 << 32) | lo0;
  key = ((unsigned long long)hi1 << 32) | hi0;
}

template <int KCAP, bool EXACT, bool KLDS = false>
struct KnnVisitor : VisitStats {
  WaveBox box;
  float qx, qy, qz;
  bool active;
  int k;
  // kept neighbours as order-preserving (squared distance, sorted position)
  // keys, ascending: the exact rule (d < D) || (d == D && j < J) of
  // KNNResultSet + the position tie-break is one u64 compare per slot
  KeyList<KCAP, KLDS> K;
  unsigned long long wk;   // worst kept key (bound)
  float wd;                // its distance
  float tight;             // min over the tested full leaves of the farthest-corner distance (squared)
  float td;                // smallest distance of an examined point that is not kept (tie detection:
                           // the k-th distance is tied iff it equals td at the end)
  int nfull;               // leaves < nfull hold 32 real points (>= k: each such box bounds the k-th neighbour)
  int skip_lo, skip_hi;

  __device__ __forceinline__ float dist(int s) const { return __uint_as_float((unsigned)(K[s] >> 32)); }
  __device__ __forceinline__ int idx(int s) const { return (int)(unsigned)K[s]; }
  __device__ __forceinline__ void init(int kk) {
    k = kk;
#pragma unroll
    for (int s = 0; s < KCAP; ++s) K[s] = dkey(INFINITY, -1);
    wk = K[0];
    wd = INFINITY;
    tight = INFINITY;
    td = INFINITY;
    nfull = 0;
    skip_lo = 1;
    skip_hi = 0;
  }
  // k-th distance (slot k - 1) and whether an examined point outside the
  // kept k lies at exactly that distance (nanoflann then keeps the one its
  // walk met first)
  __device__ __forceinline__ float kth_dist() const {
    float d = INFINITY;
#pragma unroll
    for (int s = 0; s < KCAP; ++s)
      if (s == k - 1) d = dist(s);
    return d;
  }
  __device__ __forceinline__ float outside_min() const {   // td, plus slot k of an oversized list
    float t = td;
    if constexpr (!EXACT) {
#pragma unroll
      for (int s = 0; s < KCAP; ++s)
        if (s == k) t = fminf(t, dist(s));
    }
    return t;
  }
  // any two of the kept k at the same distance (their order is nanoflann's walk order)
  __device__ __forceinline__ bool inner_tie() const {
    bool t = false;
#pragma unroll
    for (int s = 1; s < KCAP; ++s)
      if (s < k) t |= dist(s) == dist(s - 1);
    return t;
  }
  // the slot j of the one equal-distance pair (j, j + 1) among the kept k, -1
  // if there are more (or three at one distance)
  __device__ __forceinline__ int single_pair() const {
    int cnt = 0, j = -1;
#pragma unroll
    for (int s = 1; s < KCAP; ++s)
      if (s < k && dist(s) == dist(s - 1)) {
        ++cnt;
        j = s - 1;
      }
    return cnt == 1 ? j : -1;
  }
  __device__ __forceinline__ void update_worst() {
    if constexpr (EXACT) {
      wk = K[KCAP - 1];
    } else {
#pragma unroll
      for (int s = 0; s < KCAP; ++s)
        if (s == k - 1) wk = K[s];
    }
    wd = __uint_as_float((unsigned)(wk >> 32));
  }
  __device__ __forceinline__ void insert(unsigned long long key) {
    if constexpr (KLDS) {   // sorted shift from the end (the list lives in LDS)
      const unsigned long long out = K[KCAP - 1];
      if (key >= out) {
        td = fminf(td, key_dist(key));
        return;
      }
      int s = KCAP - 1;
      for (; s > 0; --s) {
        const unsigned long long prev = K[s - 1];
        if (prev <= key) break;
        K[s] = prev;
      }
      K[s] = key;
      td = fminf(td, key_dist(out));   // the key pushed out of the list
    } else {
#pragma unroll
      for (int s = 0; s < KCAP; ++s) cmp_exchange_u64(key, K[s]);
      td = fminf(td, key_dist(key));   // the key pushed out of the list
    }
    update_worst();
  }
  // the k-th neighbour is no farther than the kept k-th key, nor than the
  // farthest corner of any full leaf (32 >= k real points inside)
  __device__ __forceinline__ float bound() const { return fminf(wd, tight); }
  __device__ __forceinline__ bool need(float4 lo, float4 hi) const { return box_dist2(qx, qy, qz, lo, hi) <= bound(); }
  __device__ __forceinline__ void note_leaf(f4v lo, f4v hi, int leaf) {
    if (leaf < nfull && active) tight = fminf(tight, box_maxdist2(qx, qy, qz, lo, hi));
  }
  __device__ __forceinline__ void process(const WaveLds* L, int start) {
    for (int j = 0; j < kLeafSize; ++j) {
      const float d = dist2(qx, qy, qz, L->px[j], L->py[j], L->pz[j]);
      const unsigned long long key = dkey(d, start + j);
      // d > tight: not among the k nearest.  Only an active lane's examined
      // points count for td: an inactive lane (another sub-range of a split
      // group) re-scans leaves whose points it may already keep.
      if (active && key < wk && d <= tight) insert(key);
      else td = fminf(td, active ? d : INFINITY);   // (a select: a second branch cost 24 VGPRs in k_covariances2)
    }
  }
  __device__ __forceinline__ void scan_leaf(const CloudDev& c, int leaf, WaveLds* L) {
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (lane_id() < kLeafSize) p = ldg4(c.pts, leaf * kLeafSize + lane_id());
    stage_points<KnnVisitor>(L, p);
    process(L, leaf * kLeafSize);
  }
  __device__ __forceinline__ bool scan_leaves(const CloudDev& c, int base, unsigned long long ex, WaveLds* L) {
    return scan_leaves_lds(c, base, ex, *this, L);
  }
};

// Mean and biased covariance of the kept neighbours in their order
// (nano_gicp_impl.hpp:392-399), regularised.  The neighbour points are loaded
// four at a time (compiler barriers between the groups): with all KCAP loads
// hoisted, k = 20 held 20 float4s live and spilled.  swap >= 0: slots swap and
// swap + 1 exchanged (cov_order_free).
template <int KCAP, class KL>
__device__ __forceinline__ void cov_compute(const CloudDev& c, const KL& K, int k, int method, int swap, double* out) {
  unsigned long long ka = 0, kb = 0;   // the swapped pair's keys (slot selects, no runtime index into the list)
  if (swap >= 0) {
#pragma unroll
    for (int s = 0; s < KCAP; ++s) {
      if (s == swap) ka = K[s];
      if (s == swap + 1) kb = K[s];
    }
  }
  auto slot_pos = [&](int s) -> int {
    const unsigned long long v = swap < 0 ? K[s] : (s == swap ? kb : (s == swap + 1 ? ka : K[s]));
    return (int)(unsigned)v;
  };
  double mx = 0, my = 0, mz = 0;
#pragma unroll
  for (int s = 0; s < KCAP; ++s) {
    if (s < k) {
      const float4 p = ldg4(c.pts, slot_pos(s));
      mx += (double)p.x;
      my += (double)p.y;
      mz += (double)p.z;
    }
    if ((s & 3) == 3) asm volatile("" ::: "memory");
  }
  mx /= k;
  my /= k;
  mz /= k;
  double C[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < KCAP; ++s) {
    if (s < k) {
      const float4 p = ldg4(c.pts, slot_pos(s));
      const double d0 = (double)p.x - mx, d1 = (double)p.y - my, d2 = (double)p.z - mz;
      C[0] += d0 * d0; C[1] += d0 * d1; C[2] += d0 * d2;
      C[3] += d1 * d0; C[4] += d1 * d1; C[5] += d1 * d2;
      C[6] += d2 * d0; C[7] += d2 * d1; C[8] += d2 * d2;
    }
    if ((s & 3) == 3) asm volatile("" ::: "memory");
  }
  for (int e = 0; e < 9; ++e) C[e] /= k;
  regularize(C, method, out);
}
template <int KCAP, class KL>
__device__ __forceinline__ void cov_from_keys(const CloudDev& c, const KL& K, int k, int method, double* o) {
  double out[6];
  cov_compute<KCAP>(c, K, k, method, -1, out);
  for (int e = 0; e < 6; ++e) o[e] = out[e];
}

// An inner tie whose order cannot change the result: the covariance with the
// tied neighbours j and j + 1 exchanged (the other order nanoflann's walk may
// have met them in) equals the one stored from the Morton order, bit for bit
// after the regularisation.  Then the stored result is nanoflann's whatever
// its order, and the query needs no re-run.
template <int KCAP, class KL>
__device__ __forceinline__ bool cov_order_free(const CloudDev& c, const KL& K, int k, int method, int j, const double* stored) {
  double out[6];
  cov_compute<KCAP>(c, K, k, method, j, out);
  bool same = true;
  for (int e = 0; e < 6; ++e) same = same && __double_as_longlong(out[e]) == __double_as_longlong(stored[e]);
  return same;
}

// Seed a kNN visitor with the leaves [s0, s1] and then run the full traversal.
template <int KCAP, bool EXACT, bool KLDS>
__device__ __forceinline__ void knn_search(const CloudDev& c, KnnVisitor<KCAP, EXACT, KLDS>& vis, int s0, int s1,
                                           WaveLds* L) {
  s0 = max(s0, 0);
  s1 = min(s1, c.cnt0 - 1);
  for (int l = s0; l <= s1; ++l) vis.scan_leaf(c, l, L);
  vis.skip_lo = s0;
  vis.skip_hi = s1;
  vis.box = make_wave_box(vis.active, vis.qx, vis.qy, vis.qz, vis.wd);
  traverse(c, vis, L);
}

// kNN-k of the cloud's own points: seed with the group's own leaves, then a
// split search (keys = the cloud's sorted Morton keys)
template <int KCAP, bool EXACT, bool KLDS>
__device__ __forceinline__ void knn_self_search(const CloudDev& c, KnnVisitor<KCAP, EXACT, KLDS>& vis, int s0, int s1,
                                                unsigned long long key, WaveLds* L) {
  s0 = max(s0, 0);
  s1 = min(s1, c.cnt0 - 1);
  for (int l = s0; l <= s1; ++l) {
    vis.scan_leaf(c, l, L);
    const float4 lo = ldg4(c.box_lo, l), hi = ldg4(c.box_hi, l);   // the seed leaves' boxes bound the k-th too
    vis.note_leaf(f4v{lo.x, lo.y, lo.z, 0.f}, f4v{hi.x, hi.y, hi.z, 0.f}, l);
  }
  vis.skip_lo = s0;
  vis.skip_hi = s1;
  split_search(c, vis, key, L);
}

// covariances of a cloud: wave w handles sorted points [64w, 64w+64) (leaves 2w, 2w+1)
template <int KCAP, bool EXACT>
__global__ __launch_bounds__(256) void k_covariances(CloudDev c, int k, int method, double* __restrict__ cov6,
                                                     const unsigned char* __restrict__ redo, TieList ties) {
  constexpr bool KLDS = KCAP > 32;
  __shared__ WaveLds lds[4];
  __shared__ unsigned long long klist[KLDS ? 4 * 64 * KCAP : 1];   // KLDS: the kept lists (128 KB at k <= 64)
  WaveLds* L = &lds[threadIdx.x >> 6];
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves_total = (gridDim.x * blockDim.x) >> 6;
  const int ngroups = (c.n + 63) >> 6;
  for (int g = wave; g < ngroups; g += nwaves_total) {
    if (redo && !redo[g]) continue;   // only the groups the task path could not finish
    const int i = g * 64 + lane_id();
    KnnVisitor<KCAP, EXACT, KLDS> vis;
    if constexpr (KLDS) vis.K.p = klist + (size_t)(threadIdx.x >> 6) * 64 * KCAP + lane_id();
    vis.init(k);
    vis.nfull = k <= kLeafSize ? c.n / kLeafSize : 0;   // a full leaf holds >= k points only if k <= 32
    vis.active = i < c.n;
    const float4 q = ldg4(c.pts, min(i, c.n - 1));
    vis.qx = q.x;
    vis.qy = q.y;
    vis.qz = q.z;
    knn_self_search(c, vis, 2 * g - 1, 2 * g + 2, gp(c.keys)[min(i, c.n - 1)], L);
    if (!vis.active) continue;
    // a tie at the k-th distance changes the set; one inside the k changes the
    // summation order, which the eigen-decomposition of a degenerate
    // (isotropic) neighbourhood turns into a different regularized covariance
    const bool kth_tie = vis.outside_min() == vis.kth_dist(), inner = vis.inner_tie();
    cov_from_keys<KCAP>(c, vis.K, k, method, cov6 + 6 * (size_t)i);
    if (ties.list && (kth_tie || inner)) {
      const int j = kth_tie ? -1 : vis.single_pair();
      if (j < 0 || !cov_order_free<KCAP>(c, vis.K, k, method, j, cov6 + 6 * (size_t)i)) ties.push(i);
    }
  }
}

// Two lanes per query (lanes l and l + 32, 32 queries per wave): twice the
// wavefronts of k_covariances for the same cloud, and half the serial scan
// per lane.  Each half keeps the exact top-k of its half of every leaf's
// points (positions 0-15 / 16-31); the k-th key of either half bounds the
// k-th of the union (k real points lie within it), so a point is inserted
// only below BOTH halves' k-th keys and a leaf is tested against the smaller
// bound.  At the end the two lists are merged: the union's exact top-k.
// The partner lane's word from a permlane32 swap of (v, v): one of the two
// results is the lane's own word, the other the partner's (equal words make
// the choice immaterial), whatever order the builtin returns them in.
template <class R>
__device__ __forceinline__ unsigned swap_partner(const R& r, unsigned own) { return r[0] == own ? r[1] : r[0]; }

template <int KCAP, bool EXACT>
struct KnnVisitor2 : KnnVisitor<KCAP, EXACT> {
  using Base = KnnVisitor<KCAP, EXACT>;
  unsigned long long wk_other = ~0ull;   // the other half's k-th key
#ifdef DDLO_COV_PROF
  // s_memtime cycles: waiting for a leaf's points, scanning them, a leaf block's box tests
  unsigned long long pt_last = 0, pt_wait = 0, pt_proc = 0, pt_box = 0;
  __device__ __forceinline__ void prof_mark(int k) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (k == 1) pt_wait += t - pt_last;
    else if (k == 2) pt_proc += t - pt_last;
    else if (k == 4) pt_box += t - pt_last;
    pt_last = t;
  }
#endif
  __device__ __forceinline__ unsigned long long wk_both() const { return umin64(this->wk, wk_other); }
  __device__ __forceinline__ float bound() const {
    return fminf(__uint_as_float((unsigned)(wk_both() >> 32)), this->tight);
  }
  __device__ __forceinline__ bool need(float4 lo, float4 hi) const {
    return box_dist2(this->qx, this->qy, this->qz, lo, hi) <= bound();
  }
  __device__ __forceinline__ void exchange() {   // whole wave: wk of lane l ^ 32
    const unsigned lo = (unsigned)this->wk, hi = (unsigned)(this->wk >> 32);
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    wk_other = ((unsigned long long)swap_partner(rh, hi) << 32) | swap_partner(rl, lo);
  }
  // The staged points are read four at a time (one 16-byte LDS read per
  // axis): a per-point loop waited for one LDS round trip per point.  For
  // k = 20 the insertion test is also evaluated without short-circuit
  // branches, with the halves' bound (wk_both) kept in registers and
  // refreshed only after an insertion: k = 20 0.59 -> 0.53 ms per 131k-point
  // scan, while k = 10 measured 3 % slower that way (tools/gpu_r6_x.sh).
  __device__ __forceinline__ void process(const WaveLds* L, int start) {
    const int h0 = (lane_id() >> 5) * (kLeafSize / 2);
    const bool act = this->active;
    unsigned long long wkb = wk_both();
    for (int j0 = 0; j0 < kLeafSize / 2; j0 += 4) {
      const f4v X = *reinterpret_cast<const f4v*>(&L->px[h0 + j0]);
      const f4v Y = *reinterpret_cast<const f4v*>(&L->py[h0 + j0]);
      const f4v Z = *reinterpret_cast<const f4v*>(&L->pz[h0 + j0]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float d = dist2(this->qx, this->qy, this->qz, X[u], Y[u], Z[u]);
        const unsigned long long key = dkey(d, start + h0 + j0 + u);
        if constexpr (KCAP > 16) {
          const bool ins = act & (key < wkb) & (d <= this->tight);
          if (ins) {
            this->insert(key);
            wkb = wk_both();
          }
          this->td = fminf(this->td, (act & !ins) ? d : INFINITY);   // active lanes only (see KnnVisitor::process)
        } else {
          if (act && key < wk_both() && d <= this->tight) this->insert(key);
          else this->td = fminf(this->td, act ? d : INFINITY);   // active lanes only (see KnnVisitor::process)
        }
      }
    }
    exchange();
  }
  __device__ __forceinline__ void scan_leaf(const CloudDev& c, int leaf, WaveLds* L) {
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (lane_id() < kLeafSize) p = ldg4(c.pts, leaf * kLeafSize + lane_id());
    stage_points<KnnVisitor2>(L, p);
    process(L, leaf * kLeafSize);
  }
  __device__ __forceinline__ bool scan_leaves(const CloudDev& c, int base, unsigned long long ex, WaveLds* L) {
    return scan_leaves_lds(c, base, ex, *this, L);
  }
  // whole wave: lanes 0-31 merge their partner's list (lane + 32) into their
  // own; lanes 32-63 keep theirs unchanged, so the partner word each swap
  // returns is still the partner's original list entry (no copy of the list)
  __device__ __forceinline__ void merge_halves() {
    const bool low = lane_id() < 32;
#pragma unroll
    for (int s = 0; s < KCAP; ++s) {
      const unsigned lo = (unsigned)this->K[s], hi = (unsigned)(this->K[s] >> 32);
      const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
      const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
      const unsigned long long other = ((unsigned long long)swap_partner(rh, hi) << 32) | swap_partner(rl, lo);
      if (low) {
        if (other < this->wk) this->insert(other);
        else this->td = fminf(this->td, key_dist(other));
      }
    }
    // both halves' discarded points: the union's
    const unsigned tb = __float_as_uint(this->td);
    const auto rt = __builtin_amdgcn_permlane32_swap(tb, tb, false, false);
    this->td = fminf(__uint_as_float(rt[0]), __uint_as_float(rt[1]));
  }
};

// developer build (-DDDLO_COV_PROF): per 32-query group of k_covariances2,
// (start, end) s_memrealtime stamps (100 MHz), leaves scanned / exact-tested,
// splits, the hardware wave slot and the group's largest k-th distance
// (tools/cov_timeline.py reads them through ddlo_dev_cov_prof)
#ifdef DDLO_COV_PROF
constexpr int kCovProfGroups = 8192;
__device__ unsigned long long g_cov_prof[kCovProfGroups * 4];
__device__ unsigned long long g_cov_prof2[kCovProfGroups * 4];   // cycles: point wait, scan, box tests; blocks
#endif

// covariances with two lanes per query: wave w handles sorted points
// [32w, 32w+32) (leaf w); seeds leaves w-1 .. w+1
template <int KCAP, bool EXACT, int MINW>
__global__ __launch_bounds__(256, MINW) void k_covariances2(CloudDev c, int k, int method, double* __restrict__ cov6,
                                                            TieList ties) {
  __shared__ WaveLds lds[4];
  WaveLds* L = &lds[threadIdx.x >> 6];
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves_total = (gridDim.x * blockDim.x) >> 6;
  const int ngroups = (c.n + 31) >> 5;
  for (int g = wave; g < ngroups; g += nwaves_total) {
#ifdef DDLO_COV_PROF
    const unsigned long long cp_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int i = g * 32 + (lane_id() & 31);
    KnnVisitor2<KCAP, EXACT> vis;
    vis.init(k);
    vis.wk_other = ~0ull;
    vis.nfull = k <= kLeafSize ? c.n / kLeafSize : 0;
    vis.active = i < c.n;
    const float4 q = ldg4(c.pts, min(i, c.n - 1));
    vis.qx = q.x;
    vis.qy = q.y;
    vis.qz = q.z;
    {
      // the seed leaves with the next one's points in flight (as scan_leaves_lds)
      const int s0 = max(g - 1, 0), s1 = min(g + 1, c.cnt0 - 1);
      float4 pn = lane_id() < kLeafSize ? ldg4(c.pts, s0 * kLeafSize + lane_id()) : make_float4(0.f, 0.f, 0.f, 0.f);
      for (int l = s0; l <= s1; ++l) {
        const float4 p = pn;
        if (l < s1 && lane_id() < kLeafSize) pn = ldg4(c.pts, (l + 1) * kLeafSize + lane_id());
        const float4 lo = ldg4(c.box_lo, l), hi = ldg4(c.box_hi, l);
        stage_points<KnnVisitor2<KCAP, EXACT>>(L, p);
        vis.process(L, l * kLeafSize);
        vis.note_leaf(f4v{lo.x, lo.y, lo.z, 0.f}, f4v{hi.x, hi.y, hi.z, 0.f}, l);
      }
      vis.skip_lo = s0;
      vis.skip_hi = s1;
      split_search<KnnVisitor2<KCAP, EXACT>, 32>(c, vis, gp(c.keys)[min(i, c.n - 1)], L);
    }
    vis.merge_halves();
#ifdef DDLO_COV_PROF
    {
      const float kd = wave_max(vis.active && lane_id() < 32 ? vis.kth_dist() : 0.f);
      const unsigned long long cp_t1 = __builtin_amdgcn_s_memrealtime();
      if (lane_id() == 0 && g < kCovProfGroups) {
        unsigned long long* o2 = g_cov_prof2 + (size_t)g * 4;
        o2[0] = vis.pt_wait;
        o2[1] = vis.pt_proc;
        o2[2] = vis.pt_box;
        o2[3] = vis.st_blocks;
        unsigned long long* o = g_cov_prof + (size_t)g * 4;
        o[0] = cp_t0;
        o[1] = cp_t1;
        o[2] = (unsigned long long)vis.st_scan | ((unsigned long long)vis.st_exact << 32);
        o[3] = (unsigned long long)__float_as_uint(kd) | ((unsigned long long)vis.st_splits << 32) |
               ((unsigned long long)(__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) & 0xffff) << 40);
      }
    }
#endif
    if (!vis.active || lane_id() >= 32) continue;
    const bool kth_tie = vis.td == vis.kth_dist(), inner = vis.inner_tie();
    cov_from_keys<KCAP>(c, vis.K, k, method, cov6 + 6 * (size_t)i);
    if (ties.list && (kth_tie || inner)) {   // rare: a tie whose order matters is re-run (nftree.hip)
      bool push = true;
      if constexpr (KCAP <= 16) {   // (k = 20: a second covariance spills at the 3-wave budget; re-run them all)
        const int j = kth_tie ? -1 : vis.single_pair();
        if (j >= 0) push = !cov_order_free<KCAP>(c, vis.K, k, method, j, cov6 + 6 * (size_t)i);
      }
      if (push) ties.push(i);
    }
  }
}
template __global__ void k_covariances2<10, true, 3>(CloudDev, int, int, double*, TieList);
template __global__ void k_covariances2<10, true, 4>(CloudDev, int, int, double*, TieList);
template __global__ void k_covariances2<20, true, 3>(CloudDev, int, int, double*, TieList);
template __global__ void k_covariances2<20, true, 2>(CloudDev, int, int, double*, TieList);

// kNN of external queries (any order) against a cloud; outputs original indices.
template <int KCAP, bool EXACT>
__global__ __launch_bounds__(256) void k_knn_query(CloudDev c, const float4* __restrict__ q, int nq, int k,
                                                   int* __restrict__ out_idx, float* __restrict__ out_d, TieList ties) {
  constexpr bool KLDS = KCAP >= 32;   // a register list of 32 keys spilled here (156 VGPRs)
  __shared__ WaveLds lds[4];
  __shared__ unsigned long long klist[KLDS ? 4 * 64 * KCAP : 1];
  WaveLds* L = &lds[threadIdx.x >> 6];
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves_total = (gridDim.x * blockDim.x) >> 6;
  const int ngroups = (nq + 63) >> 6;
  for (int g = wave; g < ngroups; g += nwaves_total) {
    const int i = g * 64 + lane_id();
    KnnVisitor<KCAP, EXACT, KLDS> vis;
    if constexpr (KLDS) vis.K.p = klist + (size_t)(threadIdx.x >> 6) * 64 * KCAP + lane_id();
    vis.init(k);
    vis.nfull = k <= kLeafSize ? c.n / kLeafSize : 0;   // a full leaf holds >= k points only if k <= 32
    vis.active = i < nq;
    const float4 p = ldg4(q, min(i, nq - 1));
    vis.qx = p.x;
    vis.qy = p.y;
    vis.qz = p.z;
    // seed around the Morton position of the first lane's query
    const float sx = uniform_f(p.x), sy = uniform_f(p.y), sz = uniform_f(p.z);
    const int pos = wave_lower_bound(c.keys, c.n, morton_key(sx, sy, sz, c.quant));
    const int leaf = min(pos, c.n - 1) / kLeafSize;
    knn_search(c, vis, leaf - 1, leaf + 1, L);
    if (!vis.active) continue;
    if (ties.list && (vis.outside_min() == vis.kth_dist() || vis.inner_tie())) ties.push(i);
#pragma unroll
    for (int s = 0; s < KCAP; ++s) {
      if (s < k) {
        const int j = vis.idx(s);
        out_idx[(size_t)i * k + s] = j >= 0 ? c.perm[j] : -1;
        out_d[(size_t)i * k + s] = vis.dist(s);
      }
    }
  }
}


template __global__ void k_covariances<10, true>(CloudDev, int, int, double*, const unsigned char*, TieList);
template __global__ void k_covariances<20, true>(CloudDev, int, int, double*, const unsigned char*, TieList);
template __global__ void k_covariances<16, false>(CloudDev, int, int, double*, const unsigned char*, TieList);
template __global__ void k_covariances<32, false>(CloudDev, int, int, double*, const unsigned char*, TieList);
template __global__ void k_covariances<64, false>(CloudDev, int, int, double*, const unsigned char*, TieList);
template __global__ void k_knn_query<1, true>(CloudDev, const float4*, int, int, int*, float*, TieList);
template __global__ void k_knn_query<10, true>(CloudDev, const float4*, int, int, int*, float*, TieList);
template __global__ void k_knn_query<20, true>(CloudDev, const float4*, int, int, int*, float*, TieList);
template __global__ void k_knn_query<16, false>(CloudDev, const float4*, int, int, int*, float*, TieList);
template __global__ void k_knn_query<32, false>(CloudDev, const float4*, int, int, int*, float*, TieList);
template __global__ void k_knn_query<64, false>(CloudDev, const float4*, int, int, int*, float*, TieList);

// covariance import/export between original order (host layout) and sorted sym6
__global__ __launch_bounds__(256) void k_cov_import(const double* __restrict__ in, int layout, int n,
                                                    const int* __restrict__ inv_perm, double* __restrict__ cov6) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // original index
  if (i >= n) return;
  double* o = cov6 + 6 * (size_t)inv_perm[i];
  if (layout == 0) {  // MAT4D row-major
    const double* m = in + 16 * (size_t)i;
    o[0] = m[0]; o[1] = m[1]; o[2] = m[2]; o[3] = m[5]; o[4] = m[6]; o[5] = m[10];
  } else {
    const double* m = in + 6 * (size_t)i;
    for (int e = 0; e < 6; ++e) o[e] = m[e];
  }
}
__global__ __launch_bounds__(256) void k_cov_export(const double* __restrict__ cov6, int layout, int n,
                                                    const int* __restrict__ perm, double* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;  // sorted index
  if (s >= n) return;
  const double* c = cov6 + 6 * (size_t)s;
  const int i = perm[s];
  if (layout == 0) {
    double* m = out + 16 * (size_t)i;
    m[0] = c[0]; m[1] = c[1]; m[2] = c[2]; m[3] = 0;
    m[4] = c[1]; m[5] = c[3]; m[6] = c[4]; m[7] = 0;
    m[8] = c[2]; m[9] = c[4]; m[10] = c[5]; m[11] = 0;
    m[12] = 0; m[13] = 0; m[14] = 0; m[15] = 0;
  } else {
    double* m = out + 6 * (size_t)i;
    for (int e = 0; e < 6; ++e) m[e] = c[e];
  }
}

// registerInputSource keeps source_covs_ (nano_gicp_impl.hpp:122-130): the
// covariance of original index o moves from the old cloud's sorted position
// to the new one's
__global__ __launch_bounds__(256) void k_cov_remap(const double* __restrict__ old_cov6,
                                                   const int* __restrict__ old_inv_perm,
                                                   const int* __restrict__ new_perm, int n, double* __restrict__ cov6) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;   // new sorted index
  if (s >= n) return;
  const double* src = old_cov6 + 6 * (size_t)old_inv_perm[new_perm[s]];
  double* o = cov6 + 6 * (size_t)s;
  for (int e = 0; e < 6; ++e) o[e] = src[e];
}

// ============================================================================
// K3: fused correspondence search + Mahalanobis + normal-equation moments
// ============================================================================
struct Contrib {
  double M[6];   // Mahalanobis (xx xy xz yy yz zz)
  double q[3];   // transformed source point (double)
  double qq[6];  // q_k q_l (00 01 02 11 12 22)
  double v[3];   // M e
  double y;      // e^T M e
  double c;      // 1 if matched
};

template <int S>
__device__ __forceinline__ double moment_val(const Contrib& C) {
  if constexpr (S < 6) {
    return C.M[S];
  } else if constexpr (S < 24) {
    return C.q[(S - 6) / 6] * C.M[(S - 6) % 6];
  } else if constexpr (S < 60) {
    return C.qq[(S - 24) / 6] * C.M[(S - 24) % 6];
  } else if constexpr (S < 72) {
    constexpr int m = (S - 60) / 4, kk = (S - 60) % 4;
    if constexpr (kk == 3)
      return C.v[m];
    else
      return C.v[m] * C.q[kk];
  } else if constexpr (S == 72) {
    return C.y;
  } else if constexpr (S == 73) {
    return C.c;
  } else {
    return 0.0;
  }
}

// In-register transpose reduction step L (L = 1..5): the lane whose bit
// (6 - L) is 0 keeps the lower-half slot a, the other keeps b; each receives
// its partner's copy of the kept slot.  Steps 1 and 2 use the gfx950
// v_permlane32_swap / v_permlane16_swap (no LDS, no selects), steps 3..5 DPP
// row_mirror / row_half_mirror / quad_perm pairings.
__device__ __forceinline__ double dpp_f64(double x, int ctrl_sel) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  int rlo, rhi;
  switch (ctrl_sel) {
    case 0:  // row_mirror: l <-> 15 - l (bit 3 differs)
      rlo = __builtin_amdgcn_update_dpp(0, lo, 0x140, 0xf, 0xf, false);
      rhi = __builtin_amdgcn_update_dpp(0, hi, 0x140, 0xf, 0xf, false);
      break;
    case 1:  // row_half_mirror: l <-> 7 - l (bit 2 differs)
      rlo = __builtin_amdgcn_update_dpp(0, lo, 0x141, 0xf, 0xf, false);
      rhi = __builtin_amdgcn_update_dpp(0, hi, 0x141, 0xf, 0xf, false);
      break;
    case 2:  // quad_perm [2,3,0,1]: xor 2
      rlo = __builtin_amdgcn_update_dpp(0, lo, 0x4e, 0xf, 0xf, false);
      rhi = __builtin_amdgcn_update_dpp(0, hi, 0x4e, 0xf, 0xf, false);
      break;
    default:  // quad_perm [1,0,3,2]: xor 1
      rlo = __builtin_amdgcn_update_dpp(0, lo, 0xb1, 0xf, 0xf, false);
      rhi = __builtin_amdgcn_update_dpp(0, hi, 0xb1, 0xf, 0xf, false);
      break;
  }
  return __hiloint2double(rhi, rlo);
}

template <int L>
__device__ __forceinline__ double xchg(double a, double b) {
#ifdef DDLO_SHFL_REDUCE
  const int bit = 1 << (6 - L);
  const bool hi = (lane_id() & bit) != 0;
  const double keep = hi ? b : a;
  const double send = hi ? a : b;
  return keep + __shfl_xor(send, bit);
#else
  if constexpr (L == 1 || L == 2) {
    const unsigned alo = __double2loint(a), ahi = __double2hiint(a);
    const unsigned blo = __double2loint(b), bhi = __double2hiint(b);
    unsigned x0, x1, y0, y1;
    if constexpr (L == 1) {
      const auto rl = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
      const auto rh = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
      x0 = rl[0]; y0 = rl[1]; x1 = rh[0]; y1 = rh[1];
    } else {
      const auto rl = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
      const auto rh = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
      x0 = rl[0]; y0 = rl[1]; x1 = rh[0]; y1 = rh[1];
    }
    return __hiloint2double(x1, x0) + __hiloint2double(y1, y0);
  } else {
    const int bit = 1 << (6 - L);
    const bool hi = (lane_id() & bit) != 0;
    const double keep = hi ? b : a;
    const double send = hi ? a : b;
    return keep + dpp_f64(send, L - 3);
  }
#endif
}

template <int L, int S>
__device__ __forceinline__ double treduce(const Contrib& C) {
  if constexpr (L == 0) {
    return moment_val<S>(C);
  } else {
    constexpr int half = kMomentSlots >> L;
    const double a = treduce<L - 1, S>(C);
    const double b = treduce<L - 1, S + half>(C);
    return xchg<L>(a, b);
  }
}

__device__ __forceinline__ double final_pair(double x) {
#ifdef DDLO_SHFL_REDUCE
  return x + __shfl_xor(x, 1);
#else
  return x + dpp_f64(x, 3);
#endif
}

// slot base of the 3 moments a lane owns after the 5 pairing steps
__device__ __forceinline__ int moment_base(int lane) {
  return 48 * ((lane >> 5) & 1) + 24 * ((lane >> 4) & 1) + 12 * ((lane >> 3) & 1) + 6 * ((lane >> 2) & 1) +
         3 * ((lane >> 1) & 1);
}

__device__ __forceinline__ void load_sym6(const __attribute__((address_space(1))) double* p, double c[6]) {
  const auto q = (const __attribute__((address_space(1))) d2v*)p;
  const d2v a = q[0];
  const d2v b = q[1];
  const d2v d = q[2];
  c[0] = a.x; c[1] = a.y; c[2] = b.x; c[3] = b.y; c[4] = d.x; c[5] = d.y;
}

constexpr int kLinWaves = 4;      // waves per block (search and moment kernels)
constexpr int kSearchQ = 16;        // queries per wavefront in the correspondence search
constexpr int kSeedW = 8;           // Morton-window seed points per slice lane

// job_src (optional): the host's pinned AlignJob.  The block copies it to the
// device job (8-byte words) and initialises from its LDS copy, so an align
// needs no separate host-to-device copy before its first kernel.
__global__ __launch_bounds__(256) void k_align_init(AlignJob* __restrict__ job_dev,
                                                    const AlignJob* __restrict__ job_src) {
  static_assert(sizeof(AlignJob) % 8 == 0, "AlignJob is copied in 8-byte words");
  static_assert(offsetof(AlignJob, guess_R) % 8 == 0 && offsetof(AlignJob, guess_t) == offsetof(AlignJob, guess_R) + 72 &&
                    offsetof(AlignJob, job_full) == offsetof(AlignJob, guess_R) + 96 &&
                    offsetof(AlignJob, ticket) == offsetof(AlignJob, guess_R) + 104,
                "guess_R, guess_t, job_full, ticket: 14 consecutive 8-byte words");
  constexpr int kHdr0 = (int)(offsetof(AlignJob, guess_R) / 8), kHdrN = 14, kHdrFull = 12;
  __shared__ unsigned long long job_lds[sizeof(AlignJob) / 8];
  __shared__ int full_s;
  const AlignJob* job = job_dev;
  double gR[9], gt[3];
  // The device job's words this kernel needs, loaded before the host job's
  // header arrives (values only: they are used, and dereferenced, only when
  // the header says the device job is still the one of the last align, i.e.
  // job_full = 0; the device job buffer itself lives as long as the ctx).
  AlignState* const st_dev = job_dev->state;
  unsigned* const ctr_dev = job_dev->task_ctr;
  unsigned* const fb_dev = job_dev->fb_count;
  const int grid_dev = job_dev->grid_on;
  const int maxit_dev = job_dev->max_iterations;
  const int rec0_dev = job_dev->reuse && job_dev->reuse_rec0;
  bool full = true;
  if (job_src) {
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(job_src);
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(job_dev);
    // system scope: read past every GPU cache (the host rewrites this buffer per align).
    // First the guess, the full-copy flag and the ticket (one round trip); the rest of the
    // job only when the host changed more than the guess since the last align.
    if ((int)threadIdx.x < kHdrN) {
      const unsigned long long v = __hip_atomic_load(src + kHdr0 + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      job_lds[kHdr0 + threadIdx.x] = v;
      dst[kHdr0 + threadIdx.x] = v;
      if (threadIdx.x == kHdrFull) full_s = v != 0ull;
    }
    __syncthreads();
    full = full_s != 0;
    if (full) {
      for (int w = threadIdx.x; w < (int)(sizeof(AlignJob) / 8); w += blockDim.x) {
        if (w >= kHdr0 && w < kHdr0 + kHdrN) continue;
        const unsigned long long v = __hip_atomic_load(src + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        job_lds[w] = v;
        dst[w] = v;
      }
      __syncthreads();
      job = reinterpret_cast<const AlignJob*>(job_lds);
    }
    const AlignJob* jh = reinterpret_cast<const AlignJob*>(job_lds);
    for (int i = 0; i < 9; ++i) gR[i] = jh->guess_R[i];
    for (int i = 0; i < 3; ++i) gt[i] = jh->guess_t[i];
  } else {
    for (int i = 0; i < 9; ++i) gR[i] = job->guess_R[i];
    for (int i = 0; i < 3; ++i) gt[i] = job->guess_t[i];
  }
  AlignState* st = full ? job->state : st_dev;
  unsigned* const task_ctr = full ? job->task_ctr : ctr_dev;
  const int grid_on = full ? job->grid_on : grid_dev;
  unsigned* const fb_count = full ? job->fb_count : fb_dev;
  const int max_iterations = full ? job->max_iterations : maxit_dev;
  const int rec0 = full ? (job->reuse && job->reuse_rec0) : rec0_dev;
  if (threadIdx.x <= kTaskCounters) task_ctr[threadIdx.x * kCtrStride] = 0u;   // + the moment kernel's arrival counter
  if (grid_on && threadIdx.x <= kFbSegs) fb_count[threadIdx.x * 32] = 0u;   // the lookup's walk list (+ total)
  // source radius from the top-level boxes (<= 64 of them); an unchanged job
  // (same source cloud) keeps the last align's st->src_radius
  if (full && threadIdx.x < 64) {
    const CloudDev& c = job->src;
    const int top = c.nlevels - 1;
    const int off = lvl_off(c, top), cnt = lvl_cnt(c, top);
    float r = 0.f;
    if ((int)threadIdx.x < cnt) {
      const float4 lo = c.box_lo[off + threadIdx.x], hi = c.box_hi[off + threadIdx.x];
      const float mx = fmaxf(fabsf(lo.x), fabsf(hi.x)), my = fmaxf(fabsf(lo.y), fabsf(hi.y)),
                  mz = fmaxf(fabsf(lo.z), fabsf(hi.z));
      r = sqrtf(mx * mx + my * my + mz * mz) * 1.0001f;
    }
    for (int m = 32; m >= 1; m >>= 1) r = fmaxf(r, __shfl_xor(r, m));
    if (threadIdx.x == 0) st->src_radius = r;
  }
  if (threadIdx.x == 0) {
    st->rec = rec0;
    st->any_rec = 0;
    for (int i = 0; i < 9; ++i) st->R[i] = gR[i];
    for (int i = 0; i < 3; ++i) st->t[i] = gt[i];
    st->lambda = -1.0;
    st->iter = 0;
    st->done = max_iterations <= 0 ? 1 : 0;
    st->converged = 0;
    st->nr_iterations = 0;
    st->lm_failed = 0;
    st->lm_trials = 0;
    st->num_corr = 0;
    st->have_prev = 0;
    st->final_cost = 0.0;
    st->tie_pending = 0;
    st->ties_resolved = 0;
    st->tie_err = 0;
  }
}

// K3g: candidate-cell lookup (cellgrid.hip), one query per lane, before the
// walk.  The fp32 query transform of update_correspondences
// (nano_gicp_impl.hpp:240,253; k_nn_seed's operations), the query's cell, and
// the (squared distance, sorted position) minimum over the cell's list: the
// key the full search returns, because every point that can be the fp32
// nearest point of a query of the cell, or tie with it, is on the list.  The
// tie test of k_moments gets sec = the key's distance when a second list
// point has it (nanoflann's order then re-runs the query), else all ones (no
// test).  A query without a list (its cell was not built, or its list
// exceeded the cap) marks its 16-query sub-group for the walk (fb_mask bit,
// fb_list entry); the walk then searches only those queries.
__global__ __launch_bounds__(256) void k_cell_lookup(const AlignJob* __restrict__ job) {
  constexpr int Q = kTaskQ;   // queries per wavefront; 64 / Q lanes (slices) scan each list
  AlignState* st = job->state;
  if (__builtin_amdgcn_readfirstlane(st->done)) return;
  const CloudDev src = job->src;
  const CellGridDev G = job->grid;
  const float cap2 = job->cap2;
  const int lane = lane_id();
  const int qi = lane % Q, sl = lane / Q;
  const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int nwaves = (int)((gridDim.x * blockDim.x) >> 6);
  const int ngroups = (src.n + Q - 1) / Q;
  const int own_axis = job->own_axis;
  const float own_lo = job->own_lo, own_hi = job->own_hi;
  const int own_mod = job->own_mod, own_rem = job->own_rem;
  const int tie_detect = job->tie_detect;
  float Rf[9], tf[3];
  for (int e = 0; e < 9; ++e) Rf[e] = (float)st->R[e];
  for (int e = 0; e < 3; ++e) tf[e] = (float)st->t[e];
  for (int g = wave; g < ngroups; g += nwaves) {
    const int i = g * Q + qi;
    const bool inrange = i < src.n;
    const float4 a = ldg4(src.pts, inrange ? i : src.n - 1);
    const float qx = (Rf[0] * a.x + Rf[1] * a.y) + (Rf[2] * a.z + tf[0]);
    const float qy = (Rf[3] * a.x + Rf[4] * a.y) + (Rf[5] * a.z + tf[1]);
    const float qz = (Rf[6] * a.x + Rf[7] * a.y) + (Rf[8] * a.z + tf[2]);
    const float qa = own_axis == 0 ? qx : own_axis == 1 ? qy : qz;
    const bool owned = inrange && (own_axis < 0 || (qa >= own_lo && qa < own_hi)) &&
                       (own_mod == 0 || (g % own_mod) == own_rem);
    bool walk = false;
    unsigned off = 0, cnt = 0;
    if (owned) {
      const float tx = (qx - G.ox) * G.inv_s, ty = (qy - G.oy) * G.inv_s, tz = (qz - G.oz) * G.inv_s;
      if (!(tx >= 0.f && tx < (float)G.nx && ty >= 0.f && ty < (float)G.ny && tz >= 0.f && tz < (float)G.nz)) {
        walk = !G.outside_nomatch;   // beyond every target point's reach (or outside the built box)
      } else {
        walk = cg_cell_list(G, tx, ty, tz, off, cnt) == 2;
      }
    }
    // this slice's part of the list: the (distance, position) minimum and the
    // smallest distance of its other points
    unsigned long long bk = ~0ull;
    float d2 = INFINITY;
    constexpr int kU = 4;   // loads in flight per lane
    for (unsigned k = sl; k < cnt; k += kU * (64 / Q)) {
      float4 pp[kU];
#pragma unroll
      for (int j = 0; j < kU; ++j) pp[j] = ldg4(G.ent, off + min(k + j * (64 / Q), cnt - 1));
#pragma unroll
      for (int j = 0; j < kU; ++j) {
        const float4 p = pp[j];
        if (k + j * (64 / Q) < cnt) {
          const float dd = dist2(qx, qy, qz, p.x, p.y, p.z);
          const unsigned long long kk = dkey(dd, __float_as_int(p.w));
          if (kk < bk) {
            if (bk != ~0ull) d2 = fminf(d2, __uint_as_float((unsigned)(bk >> 32)));
            bk = kk;
          } else {
            d2 = fminf(d2, dd);
          }
        }
      }
    }
    // merge the slices: the loser's distance joins the others'
    static_assert(Q == 16, "slice merge over lanes l ^ 16, l ^ 32");
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const unsigned long long ob = h == 0 ? xor_min64<16>(bk) : xor_min64<32>(bk);   // min of the pair
      const unsigned long long other = h == 0 ? __shfl_xor(bk, 16) : __shfl_xor(bk, 32);
      const float od2 = h == 0 ? __shfl_xor(d2, 16) : __shfl_xor(d2, 32);
      const unsigned long long lose = bk < other ? other : bk;
      d2 = fminf(d2, od2);
      if (lose != ~0ull) d2 = fminf(d2, __uint_as_float((unsigned)(lose >> 32)));
      bk = ob;
    }
    if (sl == 0 && inrange && !walk) {
      job->qstate[i] = make_float4(qx, qy, qz, -1.f);
      const unsigned long long key = owned ? umin64(bk, dkey(cap2, -1)) : dkey(INFINITY, -1);
      job->key[i] = key;
      if (tie_detect) {
        const float kd = __uint_as_float((unsigned)(key >> 32));
        const bool tied = owned && (unsigned)key != 0xffffffffu && d2 == kd;
        job->sec[i] = tied ? (unsigned)(key >> 32) : 0xffffffffu;
      }
      if (job->tie_scan == 3) job->key2[i] = mirror_key(key);
    }
    // a sub-group with a query for the walk
    const unsigned m16 = (unsigned)__ballot(walk && sl == 0) & 0xffffu;
    if (m16 && lane == 0) {
      const int seg = g & (kFbSegs - 1);
      const int slot = (int)atomicAdd(job->fb_count + seg * 32, 1u);
      job->fb_list[seg * job->fb_seg_cap + slot] = g;
      job->fb_mask[g] = (unsigned short)m16;
    }
  }
}

// K3a: exact bounded 1-NN correspondence search, Q queries per wavefront.
// Pass 1: bound = distance to the previous correspondence at the new pose
// when there is one (tight), else an optimistic radius kOptR.  Pass 2
// (exact completion): queries whose pass-1 radius was clipped to kOptR and
// found nothing search again with the full max_corr bound.  Writes corr/sqd
// (update_correspondences, nano_gicp_impl.hpp:249-258).
// K3a: seeds of the exact bounded 1-NN correspondence search (nn_tasks.hpp),
// Q = 16 queries (a sub-group) per wavefront: the fp32 query transform,
// then an exact upper bound — the triangle bound from the previous
// correspondence for a small pose step (no load), the Morton window around
// the previous match after a large step, else the Morton window around the
// query's own key — then group sharing.  Writes the per-query search state
// (qstate) and the seed key, and lists the sub-groups whose union box is
// wider than hard_extent, so that k_nn_collect starts them first.
// FUSED: the same wavefront then walks its sub-group (k_nn_collect's work,
// from the seed in registers): one launch and one query-state round trip
// less per outer iteration; no hard list (walking hard sub-groups first
// measured no gain).
template <int MINW, bool FUSED>
__global__ __launch_bounds__(256, MINW) void k_nn_seed(const AlignJob* __restrict__ job) {
  constexpr int Q = kTaskQ;
  AlignState* st = job->state;
  if (__builtin_amdgcn_readfirstlane(st->done)) return;
  const CloudDev src = job->src;
  const CloudDev tgt = job->tgt;
  const auto corr = gpw(job->corr);
  const auto sqd = gpw(job->sqd);
#ifdef DDLO_SEARCH_STATS
  unsigned int* const stats = job->stats;
#else
  // per-sub-group counters only in the developer build (make statsprof): the
  // production kernel then fits 128 VGPRs (4 waves/SIMD, no hot-loop spills)
  unsigned int* const stats = nullptr;
#endif
  const float cap2 = job->cap2;
  const int have_prev = st->have_prev;
  const int prev_window = job->prev_window;
  const double tri_mv = job->tri_mv_d;
  // walk-radius inflation of this search, wave-uniform (scalar registers for the whole kernel)
  const double gap_sel = have_prev ? job->reuse_gap_d : job->reuse_gap0_d;
  const long long gap_bits = __double_as_longlong(gap_sel);
  const double gap_u = __longlong_as_double(
      ((long long)__builtin_amdgcn_readfirstlane((int)(gap_bits >> 32)) << 32) |
      (unsigned)__builtin_amdgcn_readfirstlane((int)gap_bits));
  const int own_axis = job->own_axis;
  const float own_lo = job->own_lo, own_hi = job->own_hi;
  const int own_mod = job->own_mod, own_rem = job->own_rem;
  const int lane = lane_id();
  const int qi = lane % Q;
  const int wib = threadIdx.x >> 6;
  float4* const qstate = job->qstate;
  unsigned long long* const keyout = job->key;
  const int wave = (int)blockIdx.x * kLinWaves + wib;
  const int nwaves_total = gridDim.x * kLinWaves;
  const int ngroups = (src.n + Q - 1) / Q;
  const int reuse = job->reuse;
  const bool check_ref = reuse && have_prev && st->any_rec;   // references exist only after a recording iteration
  const int rec = st->rec;   // this search records references
  // fused walk: dynamic LDS = [kLinWaves x TaskLds][upper-level box cache]
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  TaskLds* const TL = reinterpret_cast<TaskLds*>(dsm) + __builtin_amdgcn_readfirstlane(wib);   // scalar base
  f4v* const upper = reinterpret_cast<f4v*>(dsm + kLinWaves * kTaskLdsBytes);
  // candidate cells (k_cell_lookup): only the listed sub-groups, only their
  // unanswered queries; the answered ones keep the lookup's outputs.  Their
  // tasks are scanned inline (task_cap_r = 0: no k_nn_scan launch).
  const int grid_on = job->grid_on;
  int seg_end[kFbSegs];
  int nitems = ngroups;
  if (grid_on) {
    nitems = 0;
#pragma unroll
    for (int sg = 0; sg < kFbSegs; ++sg) {
      nitems += (int)job->fb_count[sg * 32];
      seg_end[sg] = nitems;
    }
    if ((int)blockIdx.x * kLinWaves >= nitems) return;   // the whole block (uniform): before the LDS prologue
  }
  if constexpr (FUSED) {
    fill_upper(tgt, upper);
    __syncthreads();
  }
  for (int item = wave; item < nitems; item += nwaves_total) {
    int g = item;
    unsigned gmask = 0xffffu;
    if (grid_on) {
      int sg = 0, s0 = 0;
#pragma unroll
      for (int t = 0; t < kFbSegs - 1; ++t)
        if (item >= seg_end[t]) {
          sg = t + 1;
          s0 = seg_end[t];
        }
      g = job->fb_list[sg * job->fb_seg_cap + (item - s0)];
      gmask = job->fb_mask[g];
    }
    const bool mine = (gmask >> qi) & 1u;   // this search writes the query's outputs
    const unsigned long long tm0 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
    const int i = g * Q + qi;
    const bool inrange = i < src.n && mine;
    const int ic = i < src.n ? i : src.n - 1;
    // every independent per-query load of the prologue in one round trip
    const float4 a = ldg4(src.pts, ic);
    const int jprev = have_prev ? corr[ic] : -1;
    const float sqprev = have_prev ? sqd[ic] : 0.f;
    const float4 rf = check_ref ? ldg4(job->ref, ic) : make_float4(0.f, 0.f, 0.f, -1.f);
    const float4 rp = check_ref ? ldg4(job->ref_p, ic) : make_float4(0.f, 0.f, 0.f, 0.f);
    // the pose is read per sub-group, so that it is not held in 12 VGPRs
    // (the fp64 -> fp32 conversions are vector ops) across the walk
    float Rf[9], tf[3];
    for (int e = 0; e < 9; ++e) Rf[e] = (float)st->R[e];
    for (int e = 0; e < 3; ++e) tf[e] = (float)st->t[e];
    // fp32 query transform, Eigen lazy-product order (see oracle/cpu_ref.cpp)
    const float qx = (Rf[0] * a.x + Rf[1] * a.y) + (Rf[2] * a.z + tf[0]);
    const float qy = (Rf[3] * a.x + Rf[4] * a.y) + (Rf[5] * a.z + tf[1]);
    const float qz = (Rf[6] * a.x + Rf[7] * a.y) + (Rf[8] * a.z + tf[2]);
    // spatial sharding: search only the queries this rank owns
    const float qa = own_axis == 0 ? qx : own_axis == 1 ? qy : qz;
    static_assert(Q == 16, "interleaved ownership is per 16-point group: i >> 4 == g");
    const bool owned = inrange && (own_axis < 0 || (qa >= own_lo && qa < own_hi)) &&
                       (own_mod == 0 || (g % own_mod) == own_rem);   // scalar: g is wave-uniform
    // Verified reuse (AlignJob::ref): every target point other than p1 was
    // at fp32 squared distance >= B^2 from q_ref, so (relative 1e-6 covers
    // the fp32 rounding of a squared distance) its true distance from q is
    // >= sqrt(B^2 / (1 + 1e-6)) - eps, eps = |q - q_ref|, and its fp32
    // squared distance >= lb2.  p1 at dn < lb2 is then the exact minimum
    // (no tie possible); with no p1, lb2 > cap2 means no point within the
    // bound.  The key is what the full search returns: min((cap2, none),
    // (dn, p1)).
    bool passed = false;
    unsigned long long pass_key = dkey(cap2, -1);
    int rj = -1;
    float dn = INFINITY;
    if (owned && rf.w >= 0.f) {
      rj = __float_as_int(rp.w);
      const double ex = (double)qx - rf.x, ey = (double)qy - rf.y, ez = (double)qz - rf.z;
      const double eps = sqrt(ex * ex + ey * ey + ez * ez) * (1.0 + 1e-9) + 1e-12;
      const double b = sqrt((double)rf.w / (1.0 + 1e-6));
      const double lb2 = b > eps ? (b - eps) * (b - eps) * (1.0 - 1e-6) : -1.0;
      if (rj >= 0) {
        dn = dist2(qx, qy, qz, rp.x, rp.y, rp.z);
        if ((double)dn < lb2) {
          passed = true;
          pass_key = umin64(pass_key, dkey(dn, rj));
        }
      } else if (lb2 > job->cap2_d) {
        passed = true;
      }
    }
    const bool active = owned && !passed;
    if (!__any(active)) {
      if (inrange && lane < Q) {
        keyout[i] = passed ? pass_key : dkey(INFINITY, -1);
        qstate[i] = make_float4(qx, qy, qz, -1.f);
        if (job->tie_detect) job->sec[i] = 0xffffffffu;   // not searched (proven strict or not owned): no tie test
        if (job->tie_scan == 3) job->key2[i] = mirror_key(passed ? pass_key : dkey(INFINITY, -1));
      }
      if (lane == 0) {
        job->hard_flag[g] = 2;   // nothing to search: k_nn_collect skips the sub-group
        job->grp_blocks[g] = 0;
      }
      if (stats) {
        const unsigned npass = (unsigned)__popcll(__ballot(passed && lane < Q));
        if (lane == 0) {
          unsigned int* o = stats + (size_t)g * kStatFields;
          for (int f = 0; f < kStatFields; ++f) o[f] = 0;
          o[6] = npass << 8;
          o[7] = FUSED ? 1 : 0;
        }
      }
      continue;
    }
    NNVisitor<Q> vis;
    vis.qx = qx;
    vis.qy = qy;
    vis.qz = qz;
    vis.active = active;
    vis.best = active ? cap2 : -1.f;
    vis.bestj = -1;
    vis.skip_lo = 1;
    vis.skip_hi = 0;
    bool seeded = false;
    bool large_step = false;   // previous match exists but the pose moved >= 2 cm since
    bool rewindow = false;     // mode 2: previous match's distance AND the Morton window at the new position
    // coordinates of the point behind vis.bestj (every seed step carries them)
    float bpx = 0.f, bpy = 0.f, bpz = 0.f;
    if (have_prev && active) {
      const int j = jprev;
      if (j >= 0) {
        // NN(q) <= |q - p_prev| <= sqrt(sqd_prev) + |q - q_prev| (triangle
        // inequality; fp64 with an upward margin covers fp32 rounding), so
        // the bound needs no load of the previous match.
        // previous linearization pose (for the triangle-inequality bound)
        float Rp[9], tp[3];
        for (int e = 0; e < 9; ++e) Rp[e] = (float)st->last_lin_R[e];
        for (int e = 0; e < 3; ++e) tp[e] = (float)st->last_lin_t[e];
        const float qpx = (Rp[0] * a.x + Rp[1] * a.y) + (Rp[2] * a.z + tp[0]);
        const float qpy = (Rp[3] * a.x + Rp[4] * a.y) + (Rp[5] * a.z + tp[1]);
        const float qpz = (Rp[6] * a.x + Rp[7] * a.y) + (Rp[8] * a.z + tp[2]);
        const double ddx = (double)qx - qpx, ddy = (double)qy - qpy, ddz = (double)qz - qpz;
        const double mv = sqrt(ddx * ddx + ddy * ddy + ddz * ddz);
        if (mv < tri_mv) {
          const double r = sqrt((double)sqprev) + mv;
          const double b2 = r * r * (1.0 + 1e-5) + 1e-12;
          if (b2 < job->cap2_d) {
            vis.best = __uint_as_float(__float_as_uint((float)b2) + 1);  // round up
            seeded = true;
          }
        } else if (prev_window == 1) {
          large_step = true;   // exact distances to the Morton window around p_prev (below)
        } else {  // large pose step: the exact distance to the previous match (+ mode 2: the Morton window below)
          rewindow = prev_window == 2;
          const float4 p = ldg4(tgt.pts, j);
          const float d = dist2(qx, qy, qz, p.x, p.y, p.z);
          if (d < cap2) {
            vis.best = d;
            vis.bestj = j;
            bpx = p.x;
            bpy = p.y;
            bpz = p.z;
            seeded = true;
          }
        }
      }
    }
    // the reference's match at the new position is a real candidate
    if (active && rj >= 0 && dn < vis.best) {
      vis.best = dn;
      vis.bestj = rj;
      bpx = rp.x;
      bpy = rp.y;
      bpz = rp.z;
      seeded = true;
    }
    // Exact seeding for queries without a usable previous correspondence:
    // the real target points around the query's Morton position give an
    // upper bound, so the single search below stays exact.  After a large
    // pose step the window is centred on the previous match instead (its
    // sorted position IS a Morton position next to the new nearest point,
    // and no key search is needed); the window contains the previous match.
    const bool need_seed = active && ((!seeded && !large_step) || rewindow);
    const bool use_window = need_seed || large_step;
    if (__any(use_window)) {
      // Morton window of kSeedW points per slice lane (64/Q * kSeedW per query)
      int pos = large_step ? jprev : 0;
      if (__any(need_seed)) {
        const unsigned long long qk = morton_key(qx, qy, qz, tgt.quant);
        int dlo, dhi, sp;
        const bool found = seed_pos(tgt.dir, qk, sp, dlo, dhi);   // directory + fine directory: <= 2 loads
        if (__any(!found)) {   // a bucket of >= 2^16 keys: searched
          const bool srch = need_seed && !found;
          sp = group_lower_bound<Q>(tgt.keys, tgt.n, qk, srch ? dlo : sp, srch ? dhi : sp);
        }
        if (need_seed) pos = sp;
      }
      const int s = lane / Q;
      const int w0 = pos - (64 / Q) * kSeedW / 2 + s * kSeedW;
      unsigned long long bk = dkey(vis.best, vis.bestj);
      float4 p[kSeedW];
#pragma unroll
      for (int k = 0; k < kSeedW; ++k) p[k] = ldg4(tgt.pts, min(max(w0 + k, 0), tgt.n - 1));
      // the winner's coordinates travel with its key (group sharing below needs no load)
      float cx = bpx, cy = bpy, cz = bpz;
      if (use_window) {
#pragma unroll
        for (int k = 0; k < kSeedW; ++k) {
          const int cand = min(max(w0 + k, 0), tgt.n - 1);
          const unsigned long long kk = dkey(dist2(qx, qy, qz, p[k].x, p[k].y, p[k].z), cand);
          if (kk < bk) {
            bk = kk;
            cx = p[k].x;
            cy = p[k].y;
            cz = p[k].z;
          }
        }
      }
      static_assert(Q == 16, "slice merge over lanes l ^ 16, l ^ 32");
      xor_min64_xyz<16>(bk, cx, cy, cz);
      xor_min64_xyz<32>(bk, cx, cy, cz);
      if (use_window) {
        const float bd = __uint_as_float((unsigned)(bk >> 32));
        if (bd < cap2) {
          vis.best = bd;
          vis.bestj = (int)(unsigned)bk;
          bpx = cx;
          bpy = cy;
          bpz = cz;
        }
      }
    }
    // Probe seeds: a sub-group whose Morton windows found nothing near (its
    // queries sit off every surface near their own Morton positions, e.g.
    // 0.4-0.5 m off a wall under the guess pose, and keep a bound near the
    // cap) takes the Morton windows of 8 points around its centre, offset by
    // probe_d along +-x, +-y, +-z and the two xy diagonals: 8 points each,
    // staged in LDS, every query their exact distances (real candidates, so
    // exactness is kept; group sharing below spreads them).
    if constexpr (FUSED) {
      const float pt2 = job->probe2;
      if (pt2 > 0.f && pt2 < 0.5f * cap2 && __any(need_seed && vis.best > pt2)) {   // radius < 0.71 x the cap
        // centre: the first active query (the sub-group is Morton-compact)
        const unsigned long long am = __ballot(active);
        const int c0 = am ? __builtin_ctzll(am) : 0;
        const float cx = readlane_f(qx, c0), cy = readlane_f(qy, c0), cz = readlane_f(qz, c0);
        const float d = job->probe_d, dd = d * 0.70710678f;
        const int pr = lane & 7;
        const float ox = pr == 0 ? d : pr == 1 ? -d : pr == 6 ? dd : pr == 7 ? -dd : 0.f;
        const float oy = pr == 2 ? d : pr == 3 ? -d : pr == 6 ? dd : pr == 7 ? -dd : 0.f;
        const float oz = pr == 4 ? d : pr == 5 ? -d : 0.f;
        const unsigned long long pk = morton_key(cx + ox, cy + oy, cz + oz, tgt.quant);
        int plo, phi, plb;
        const bool pfound = seed_pos(tgt.dir, pk, plb, plo, phi);
        if (__any(!pfound)) plb = group_lower_bound<8>(tgt.keys, tgt.n, pk, pfound ? plb : plo, pfound ? plb : phi);
        const int cand = min(max(plb - 4 + (lane >> 3), 0), tgt.n - 1);
        const float4 p = ldg4(tgt.pts, cand);
        f4v* const CP = TL->sb_lo;   // 64 staged candidates (the walk's box stage, free until the walk)
        CP[lane] = f4v{p.x, p.y, p.z, __int_as_float(cand)};
        __builtin_amdgcn_wave_barrier();
        unsigned long long bk = dkey(vis.best, vis.bestj);
        float ux = bpx, uy = bpy, uz = bpz;
        const int s4 = lane / Q;
#pragma unroll 4
        for (int k = 0; k < 64 / (64 / Q); ++k) {
          const f4v c = CP[s4 * (64 / (64 / Q)) + k];
          const unsigned long long kk = dkey(dist2(qx, qy, qz, c.x, c.y, c.z), __float_as_int(c.w));
          if (kk < bk) {
            bk = kk;
            ux = c.x;
            uy = c.y;
            uz = c.z;
          }
        }
        xor_min64_xyz<16>(bk, ux, uy, uz);
        xor_min64_xyz<32>(bk, ux, uy, uz);
        __builtin_amdgcn_wave_barrier();
        if (active && bk < dkey(vis.best, vis.bestj)) {
          vis.best = __uint_as_float((unsigned)(bk >> 32));
          vis.bestj = (int)(unsigned)bk;
          bpx = ux;
          bpy = uy;
          bpz = uz;
          seeded = true;
        }
      }
    }
    // Group sharing: every query also takes the exact distance to the other
    // queries' candidate points (Morton-adjacent queries are spatially
    // adjacent, so a neighbour's candidate is often far closer than the
    // query's own).  Valid (distance, position) pairs only: exactness kept.
    {
      const unsigned long long donors = __ballot(lane < Q && active && vis.bestj >= 0);
      if (donors && __any(active)) {
        // lane (query qi, slice s) takes donors 4s .. 4s + 3 (read from their
        // slice-0 lanes), then the four slices merge: 4 distance steps per
        // lane instead of one per donor
        unsigned long long bk = dkey(vis.best, vis.bestj);
        const int s = lane / Q;
#pragma unroll 1
        for (int t = 0; t < 4; ++t) {
          const int d = s * 4 + t;
          const float sx = __shfl(bpx, d), sy = __shfl(bpy, d), sz = __shfl(bpz, d);
          const int sj = __shfl(vis.bestj, d);
          if ((donors >> d) & 1ull) bk = umin64(bk, dkey(dist2(qx, qy, qz, sx, sy, sz), sj));
        }
        bk = xor_min64<16>(bk);
        bk = xor_min64<32>(bk);
        if (active) {
          vis.best = __uint_as_float((unsigned)(bk >> 32));
          vis.bestj = (int)(unsigned)bk;
        }
      }
    }
    // walk radius: the seed bound, widened by the reuse gap so that the
    // reference recorded from this search has B well above d1
    float wr = vis.best;
    const double gap = gap_u;
    if (rec && active && gap > 0.0) {
      const double r = sqrt((double)vis.best) + gap;
      wr = __uint_as_float(__float_as_uint((float)(r * r)) + 1);   // rounded up
    }
    // FUSED: the query state and key are stored after the walk -- a store
    // ahead of the walk's first box loads would be waited for with them
    // (vmcnt counts loads and stores in issue order)
    if (!FUSED && inrange && lane < Q) {
      qstate[i] = make_float4(qx, qy, qz, active ? wr : -1.f);
      keyout[i] = active ? dkey(vis.best, vis.bestj) : passed ? pass_key : dkey(INFINITY, -1);
      if (job->tie_scan == 3) job->key2[i] = mirror_key(keyout[i]);
    }
    if constexpr (FUSED) {
      // the walk of k_nn_collect, from the seed in registers
      const unsigned long long k0 = dkey(vis.best, vis.bestj);
      TaskList tl;
      tl.tasks = job->tasks;
      tl.ctr = job->task_ctr;
      tl.cap_r = job->task_cap_r;
      TaskCollector col;
      col.L = TL;
      col.U = upper;
      col.nup = upper_count(tgt);
      col.qx = qx;
      col.qy = qy;
      col.qz = qz;
      col.active = active;
      col.bk = k0;
      col.wr = active ? wr : -1.f;
      col.sg = g;
      col.pf_ratio = job->pf_ratio;
      const unsigned tm1 = stats ? (unsigned)__builtin_amdgcn_s_memtime() : 0u;
      col.run(tgt, tl, gp(src.keys)[ic], job->split_extent);
      if (inrange && lane < Q) {
        qstate[i] = make_float4(qx, qy, qz, active ? wr : -1.f);
        const unsigned long long k_out = active ? col.bk : passed ? pass_key : dkey(INFINITY, -1);
        keyout[i] = k_out;   // col.bk: the seed, lowered by inline scans
        if (job->tie_scan == 3) job->key2[i] = mirror_key(k_out);
      }
      // the examined points' second distance: the reuse bound (rec) and the
      // tie test of k_moments (sec == the key's distance); k_nn_scan lowers it
      if ((rec || job->tie_detect) && inrange && lane < Q)
        job->sec[i] = active ? __float_as_uint(col.sec) : 0xffffffffu;   // all ones: not searched, no tie test
      if (stats) {
        const unsigned npass = (unsigned)__popcll(__ballot(passed && lane < Q));
        if (lane == 0) {
          unsigned int* o = stats + (size_t)g * kStatFields;
          o[0] = col.st_blocks;
          o[1] = min((tm1 - (unsigned)tm0) >> 4, 65535u);
          o[2] = col.st_tasks | (min(col.st_iters, 65535u) << 16);
          o[3] = col.st_inline;
          o[4] = (unsigned)__builtin_amdgcn_s_memtime() - (unsigned)tm0;
          o[5] = min((col.tm_walk - (unsigned)tm0) >> 4, 65535u);
          o[6] = npass << 8;
          o[7] = 1;
        }
      }
    } else {
      // hard sub-group: a wide union box (a query far from every target point
      // drags many blocks into the walk) -> listed, walked first
      const WaveBox whole = make_wave_box(active, qx, qy, qz, active ? wr : -1.f);
      // hard: the previous outer iteration walked many blocks for this
      // sub-group (same source points, a nearby pose), else -- first
      // iteration -- a wide union box
      const bool hard = have_prev ? job->grp_blocks[g] > job->hard_blocks : box_extent(whole) > job->hard_extent;
      if (lane == 0) {
        int slot = -1;
        if (hard) {
          slot = (int)atomicAdd(job->task_ctr + kTaskRegions * kCtrStride, 1u);
          if (slot < kHardMax) job->hard_list[slot] = g;
        }
        job->hard_flag[g] = (unsigned char)(hard && slot < kHardMax);
      }
      if (stats) {
        const unsigned npass = (unsigned)__popcll(__ballot(passed && lane < Q));
        if (lane == 0) {
          unsigned int* o = stats + (size_t)g * kStatFields;
          o[1] = min(((unsigned)__builtin_amdgcn_s_memtime() - (unsigned)tm0) >> 4, 65535u);
          o[6] = (unsigned)hard | (npass << 8);   // queries proven by their reuse reference
        }
      }
    }
  }
}

// K3b: task collect, one wavefront per sub-group (nn_tasks.hpp): the
// query states and seed keys of k_nn_seed, the LDS-cached walk of the upper
// levels with the union box of the 16 balls, the exact (leaf, query) box
// tests, tasks appended to the list.  Waves 0 .. kHardMax-1 take the hard
// sub-groups listed by the seed kernel (dispatched first, so the longest
// walks start first); the other waves take the remaining sub-groups in
// order.
template <int MINW>
__global__ __launch_bounds__(256, MINW) void k_nn_collect(const AlignJob* __restrict__ job) {
  constexpr int Q = kTaskQ;
  const AlignState* st = job->state;
  if (__builtin_amdgcn_readfirstlane(st->done)) return;
  const CloudDev src = job->src;
  const CloudDev tgt = job->tgt;
  unsigned int* const stats = job->stats;
  const int lane = lane_id();
  const int qi = lane % Q;
  const int wib = threadIdx.x >> 6;
  // dynamic LDS: [kLinWaves x TaskLds][upper-level box cache]
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  TaskLds* TL = reinterpret_cast<TaskLds*>(dsm) + wib;
  f4v* upper = reinterpret_cast<f4v*>(dsm + kLinWaves * kTaskLdsBytes);
  TaskList tl;
  tl.tasks = job->tasks;
  tl.ctr = job->task_ctr;
  tl.cap_r = job->task_cap_r;
  unsigned long long* const keyout = job->key;
  const int ngroups = (src.n + Q - 1) / Q;
  const int wave = (int)blockIdx.x * kLinWaves + wib;
  int g;
  if (wave < kHardMax) {
    const int nhard = min((int)__builtin_amdgcn_readfirstlane(job->task_ctr[kTaskRegions * kCtrStride]), kHardMax);
    if (__builtin_amdgcn_readfirstlane((int)(blockIdx.x * kLinWaves)) >= nhard) return;   // whole block idle
    g = wave < nhard ? job->hard_list[wave] : -1;
  } else {
    g = wave - kHardMax;
    if (g >= ngroups || job->hard_flag[g]) g = -1;
  }
  g = __builtin_amdgcn_readfirstlane(g);
  if (wave >= kHardMax) {
    // no sub-group of this block has work: skip the box cache fill (every
    // wave reads the block's kLinWaves flags itself: block-uniform, no barrier)
    const int gk = (int)blockIdx.x * kLinWaves + lane - kHardMax;
    if (!__any(lane < kLinWaves && gk < ngroups && !job->hard_flag[gk])) return;
  }
  fill_upper(tgt, upper);
  __syncthreads();
  if (g < 0) return;
  const unsigned long long tm0 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
  const int i = g * Q + qi;
  const bool inrange = i < src.n;
  const int ic = inrange ? i : src.n - 1;
  const float4 q = ldg4(job->qstate, ic);
  const unsigned long long k0 = gp(keyout)[ic];
  const unsigned long long skey = gp(src.keys)[ic];
  TaskCollector col;
  col.L = TL;
  col.U = upper;
  col.nup = upper_count(tgt);
  col.qx = q.x;
  col.qy = q.y;
  col.qz = q.z;
  col.active = inrange && q.w >= 0.f;
  col.bk = k0;
  col.wr = q.w;
  col.sg = g;
  col.pf_ratio = job->pf_ratio;
  col.run(tgt, tl, skey, job->split_extent);
  if (inrange && lane < Q && col.bk != k0) {
    keyout[i] = col.bk;   // lowered by inline scans
    if (job->tie_scan == 3) job->key2[i] = mirror_key(col.bk);
  }
  if ((st->rec || job->tie_detect) && inrange && lane < Q)   // k_nn_scan lowers it further; all ones: not searched
    job->sec[i] = col.active ? __float_as_uint(col.sec) : 0xffffffffu;
  if (lane == 0) job->grp_blocks[g] = (unsigned short)min(col.st_blocks, 65535u);
  if (stats && lane == 0) {
    const unsigned long long tm1 = __builtin_amdgcn_s_memtime();
    unsigned int* o = stats + (size_t)g * kStatFields;
    o[0] = col.st_blocks;
    o[2] = col.st_tasks | (min(col.st_iters, 65535u) << 16);
    o[3] = col.st_inline;
    o[4] = (unsigned)(tm1 - tm0);
    o[5] = min((col.tm_walk - (unsigned)tm0) >> 4, 65535u);
    o[7] = 1;
  }
}

// K3c: leaf scans of the task list.  The waves of region r split its tasks
// into contiguous chunks (XCD-aware, see below).  A wave loads up to 64
// task words at once and stages batches of kScanBatch tasks in LDS with
// LDS-DMA — per task the leaf's 32 SoA points (384 B) and the sub-group's 16
// query states (256 B) — double-buffered: batch k + 1 is in flight while
// batch k is scanned from LDS (lane = query qi x quarter s of the leaf).  A
// sub-group's tasks sit next to each other in the list (one collect flush),
// so the per-query minimum is kept in registers across a run of the same
// sub-group and merged into the result with one 64-bit atomicMin per query.
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}

constexpr int kScanBatch = 8;                         // tasks per LDS batch (two batches in flight)
constexpr int kScanTaskBytes = 3 * kLeafSize * 4 + kTaskQ * 16;   // 384 B points + 256 B queries
constexpr int kScanWaves = 4;                         // waves per block

template <int MINW, int BATCH = kScanBatch>
__global__ __launch_bounds__(64 * kScanWaves, MINW) void k_nn_scan(const AlignJob* __restrict__ job) {
  const AlignState* st = job->state;
  if (__builtin_amdgcn_readfirstlane(st->done)) return;
  const CloudDev tgt = job->tgt;
  const float4* const qstate = job->qstate;
  unsigned long long* const key = job->key;
  const int cap_r = job->task_cap_r;
  const int lane = lane_id();
  const int qi = lane & 15, s = lane >> 4;
  constexpr int kBatchBytes = BATCH * kScanTaskBytes;   // 8 tasks: 5 KB = 5 LDS-DMA wave-instructions
  constexpr int kDma = (kBatchBytes + 1023) / 1024;     // LDS-DMA wave-instructions per batch
  static_assert(kDma <= 15, "vmcnt immediate");
  __shared__ __attribute__((aligned(16))) unsigned char lds_all[kScanWaves][2][kBatchBytes];
  unsigned char* const L0 = lds_all[threadIdx.x >> 6][0];
  unsigned char* const L1 = lds_all[threadIdx.x >> 6][1];
  const int nwaves = (int)((gridDim.x * blockDim.x) >> 6);
  const int wpr = nwaves / kTaskRegions;   // the grid is a multiple of 8 * kTaskRegions waves
  // (region, chunk) of this wave.  A region's tasks were appended roughly in
  // sub-group (= Morton) order, so chunk c of every region covers about the
  // same c-th slice of the scene; blocks b and b + 8 share an XCD and its
  // L2, so XCD x = b % 8 gets chunks [x wpr / 8, (x + 1) wpr / 8) of all
  // regions: one spatial eighth of the target per L2.  Speed only: any
  // bijection of waves onto (region, chunk) is exact.
  int r, c;
  if (job->xcd_scan && wpr % 8 == 0) {
    const int x = blockIdx.x % 8, u = (int)(blockIdx.x / 8) * kScanWaves + (int)(threadIdx.x >> 6);
    r = u % kTaskRegions;
    c = x * (wpr / 8) + u / kTaskRegions;
  } else {
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    r = wave % kTaskRegions;
    c = wave / kTaskRegions;
  }
  const int n = min((int)__builtin_amdgcn_readfirstlane(job->task_ctr[r * kCtrStride]), cap_r);
  const int chunk = (n + wpr - 1) / wpr;
  const int lo = c * chunk, hi = min(n, lo + chunk);
  const unsigned long long* rt = job->tasks + (size_t)r * cap_r;
  unsigned* const sec = job->sec;
  const bool rec = st->rec != 0;     // this search records reuse references
  // the second distance of the examined points is tracked for the reuse
  // bound (rec) and for k_moments' tie test (tie_detect): every point at the
  // final nearest distance is examined (its leaf is within the walk radius),
  // so the query is tied iff another examined point has that distance
  const bool reuse = rec || (job->tie_scan == 1 || job->tie_scan == 2);
  const bool lane_sd = rec || job->tie_scan == 1;   // second distance over every point of a slice
  // tie_scan 3 (not recording): the Morton-order scan plus equal-distance
  // flags at its merges (slices, tasks of a run) and the mirrored key pushed
  // beside the key (runs): no atomic return is waited for
  // tie_scan 4: the same, but the runs' ties come from the key's atomicMin
  // return (consumed at the next run's merge) and a run's own merges instead
  // of a mirrored key: one atomic per run, no key2 traffic
  const bool tie3 = !rec && (job->tie_scan == 3 || job->tie_scan == 4);
  const bool mirror = job->tie_scan == 3;
  const bool tie_xor = !(job->tie_ab & 2);
  unsigned long long* const key2 = job->key2;
  unsigned td = 0xffffffffu;   // smallest distance (bits) met twice at a slice merge of this run (any slice lane)
  unsigned long long accm = ~0ull;   // the run's minimum of mirrored keys (its tasks' bests, highest position first)
  int run_sg = -1;
  unsigned long long acc = ~0ull;   // lane's query minimum over the current run
  float acc2 = INFINITY;            // smallest distance of the run's other points (reuse)
  float run_bound = -1.f;
  // A run's merge into the result: the key's atomicMin, then (reuse) the
  // smallest distance of every examined point except the final best — the
  // run's other points and whichever of (old key, run minimum) lost.  The
  // second push needs the atomicMin's return value: it is issued at the
  // NEXT run's merge, so the return trip overlaps the scan of that run.
  bool pend = false;
  size_t pend_q = 0;
  unsigned long long pend_acc = 0ull, pend_old = 0ull;
  float pend_acc2 = 0.f, pend_bound = 0.f;
  auto resolve = [&]() {
    if (pend) {
      float push = pend_acc2;
      if (pend_old != pend_acc) {
        const unsigned long long lost = pend_old < pend_acc ? pend_acc : pend_old;
        if (key_real(lost)) push = fminf(push, key_dist(lost));
      }
      // rec: everything below the walk radius (B^2 = min(sec, radius));
      // tie test only: a push can matter only if it equals the query's
      // current minimum (the final one is <= it), so almost none is issued
      if (rec ? push <= pend_bound : push == key_dist(umin64(pend_old, pend_acc)))
        atomicMin(sec + pend_q, __float_as_uint(push));
      pend = false;
    }
  };
  // tie_scan 4 (the same pending slot, reuse is off): the previous run's key
  // atomicMin return at the same distance and another position is a tie
  auto resolve4 = [&]() {
    if (pend) {
      if (key_real(pend_old) && pend_old != pend_acc && (pend_old >> 32) == (pend_acc >> 32))
        atomicMin(sec + pend_q, (unsigned)(pend_acc >> 32));
      pend = false;
    }
  };
  auto flush_run = [&]() {
    if (tie3 && !mirror) resolve4();
    if (run_sg >= 0 && lane < 16 && (unsigned)(acc >> 32) <= __float_as_uint(run_bound)) {
      const size_t qidx = (size_t)run_sg * kTaskQ + qi;
      if (reuse) {
        resolve();
        pend_old = atomicMin(key + qidx, acc);
        pend = true;
        pend_q = qidx;
        pend_acc = acc;
        pend_acc2 = acc2;
        pend_bound = run_bound;
      } else if (tie3 && !mirror) {
        pend_old = atomicMin(key + qidx, acc);
        pend = true;
        pend_q = qidx;
        pend_acc = acc;
      } else {
        atomicMin(key + qidx, acc);
        if (tie3 && !(job->tie_ab & 1)) atomicMin(key2 + qidx, accm);   // with key: two of the run's tasks at the distance = a tie
      }
    }
    if (tie3 && run_sg >= 0) {   // the run's tie distances of the query's four slice lanes -> its lane qi
      unsigned t = min(td, (unsigned)__shfl_xor((int)td, 16));
      t = min(t, (unsigned)__shfl_xor((int)t, 32));
      if (lane < 16 && t <= __float_as_uint(run_bound))   // rare: a real equal-distance pair
        atomicMin(sec + (size_t)run_sg * kTaskQ + qi, t);   // k_moments: tied iff it is the final distance
    }
  };
  for (int wbase = lo; wbase < hi; wbase += 64) {
    const int wcnt = min(64, hi - wbase);
    const unsigned long long tl = lane < wcnt ? rt[wbase + lane] : 0ull;   // up to 64 task words at once
    // LDS-DMA tasks [b0, b0 + kScanBatch) of the window: 16 B per lane per
    // instruction, 1 KB per wave-instruction (past the window: the last task
    // again, never read)
    auto issue = [&](int b0, unsigned char* buf) {
#pragma unroll
      for (int i = 0; i < kDma; ++i) {
        const int o = i * 1024 + lane * 16;
        const int k = min(b0 + o / kScanTaskBytes, wcnt - 1), w = o % kScanTaskBytes;
        const unsigned long long tk = __shfl(tl, k);   // every lane takes part in the permute
        const char* src = w < 3 * kLeafSize * 4
                              ? (const char*)(tgt.soa + (size_t)(tk >> 40) * (3 * kLeafSize)) + w
                              : (const char*)(qstate + (size_t)((tk >> 16) & 0xffffffull) * kTaskQ) + (w - 3 * kLeafSize * 4);
        if (kBatchBytes % 1024 == 0 || o < kBatchBytes)   // a partial last instruction: lanes past the batch idle
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                           (__attribute__((address_space(3))) void*)(buf + i * 1024), 16, 0, 0);
      }
    };
    issue(0, L0);
    for (int b0 = 0; b0 < wcnt; b0 += BATCH) {
      unsigned char* const cur = ((b0 / BATCH) & 1) ? L1 : L0;
      if (b0 + BATCH < wcnt) {
        issue(b0 + BATCH, ((b0 / BATCH) & 1) ? L0 : L1);
        __builtin_amdgcn_s_waitcnt(0x0F70 | kDma);  // vmcnt(kDma): all but the batch just issued -> the current batch landed
      } else {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      }
      __builtin_amdgcn_wave_barrier();
      const int nb = min(BATCH, wcnt - b0);
      for (int k = 0; k < nb; ++k) {
        const unsigned long long t = readlane_u64(tl, b0 + k);
        const int sg = (int)((t >> 16) & 0xffffffull);
        if (sg != run_sg) {   // uniform: a new sub-group's run starts
          flush_run();
          run_sg = sg;
          acc = ~0ull;
          acc2 = INFINITY;
          run_bound = -1.f;
          td = 0xffffffffu;
          accm = ~0ull;
        }
        const unsigned char* T = cur + k * kScanTaskBytes;
        const f4v x0 = *(const f4v*)(T + s * 32), x1 = *(const f4v*)(T + s * 32 + 16);
        const f4v y0 = *(const f4v*)(T + 128 + s * 32), y1 = *(const f4v*)(T + 128 + s * 32 + 16);
        const f4v z0 = *(const f4v*)(T + 256 + s * 32), z1 = *(const f4v*)(T + 256 + s * 32 + 16);
        const f4v q = *(const f4v*)(T + 384 + qi * 16);
        const float X[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const float Y[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
        const float Z[8] = {z0.x, z0.y, z0.z, z0.w, z1.x, z1.y, z1.z, z1.w};
        // same IEEE ops as dist2(), two points per packed instruction; the
        // lane's points come in increasing position, so strict < keeps the
        // lowest position among equal distances
        const f2v qx2 = {q.x, q.x}, qy2 = {q.y, q.y}, qz2 = {q.z, q.z};
        f2v d[4];
#pragma unroll
        for (int h = 0; h < 8; h += 2) {
          const f2v dx = qx2 - f2v{X[h], X[h + 1]};
          const f2v dy = qy2 - f2v{Y[h], Y[h + 1]};
          const f2v dz = qz2 - f2v{Z[h], Z[h + 1]};
          d[h / 2] = (dx * dx + dy * dy) + dz * dz;
        }
        const bool on = ((t >> qi) & 1ull) != 0ull;
        const int pos0 = (int)(t >> 40) * kLeafSize + s * 8;
        if (reuse) {   // recording search / tie test: the leaf's best key and a second distance (uniform branch)
          float bd = INFINITY, sd = INFINITY;
          int bh = 0;
          if (lane_sd) {   // every examined point: the reuse bound (and the full tie test)
#pragma unroll
            for (int h = 0; h < 8; ++h) {
              const float dh = (h & 1) ? d[h / 2].y : d[h / 2].x;
              if (dh < bd) { sd = bd; bd = dh; bh = h; } else { sd = fminf(sd, dh); }
            }
          } else {   // tie test only: the slices' losing bests; a tie inside the winner's 8-point slice is
                     // k_moments' own check
#pragma unroll
            for (int h = 0; h < 8; ++h) {
              const float dh = (h & 1) ? d[h / 2].y : d[h / 2].x;
              if (dh < bd) { bd = dh; bh = h; }
            }
          }
          unsigned long long bk = dkey(bd, pos0 + bh);
          xor_top2<16>(bk, sd);
          xor_top2<32>(bk, sd);
          if (on) fold_top2(acc, acc2, bk, sd);
        } else {
          float bd = INFINITY;
          int bh = 0;
#pragma unroll
          for (int h = 0; h < 8; ++h) {
            const float dh = (h & 1) ? d[h / 2].y : d[h / 2].x;
            if (dh < bd) { bd = dh; bh = h; }
          }
          unsigned long long bk = dkey(bd, pos0 + bh);
          if (tie3) {   // equal distances meeting at a merge: a tie (two points of one slice: k_moments' check)
            unsigned tt = 0xffffffffu;
            if (tie_xor) {
              bk = xor_min64_eq<16>(bk, tt);
              bk = xor_min64_eq<32>(bk, tt);
            } else {
              bk = xor_min64<16>(bk);
              bk = xor_min64<32>(bk);
            }
            if (on) {
              td = min(td, tt);
              // two of the run's tasks at one distance (tie_scan 4; a leaf met twice in a run is one key)
              if (!mirror && acc != bk && (acc >> 32) == (bk >> 32)) td = min(td, (unsigned)(bk >> 32));
              acc = umin64(acc, bk);
              if (mirror) accm = umin64(accm, mirror_key(bk));   // (a leaf met twice in a run is one key: no false tie)
            }
          } else {
            bk = xor_min64<16>(bk);
            bk = xor_min64<32>(bk);
            if (on) acc = umin64(acc, bk);
          }
        }
        if (on) run_bound = q.w;
      }
      __builtin_amdgcn_wave_barrier();   // reads of `cur` done before it is refilled
    }
  }
  flush_run();
  if (tie3 && !mirror) resolve4();
  else resolve();
}

// K3b: Mahalanobis + normal-equation moments of the matched pairs
// (update_correspondences :265-273 + linearize :292-328), 64 points per
// wavefront, in-register transpose reduction, one slab row per block.
constexpr int kMomWaves = 8;    // waves per moment block (512 threads: 256 blocks fill the chip at 131k points)

// (A last-block-done fusion of k_lm_step into this kernel measured slower:
// 27.3 us against 9 + 13.5 us — every block's agent-scope release writes
// back its XCD's L2 before the completion counter.)
template <bool PREMOM>
__device__ __forceinline__ void lm_step_body(const AlignJob* __restrict__ job, AlignState* __restrict__ st,
                                             const double* __restrict__ slab, int nblocks,
                                             const double* __restrict__ premom);

// Exact ties of update_correspondences' 1-NN (nano_gicp_impl.hpp:255): the
// reference keeps the equidistant point nanoflann's walk meets first
// (KNNResultSet adds only below the worst distance, nanoflann_impl.hpp:1509),
// the search here the lower Morton position.  The lanes in `tied` are re-run,
// one at a time by the whole wavefront, through the target's nanoflann tree
// (nf_search_wave, k = 1), from the same fp32 query; the result must have the
// same distance.  Without a tree the align is flagged (tie_pending): the host
// builds it and runs the align again.  Not inlined: the rare path keeps its
// registers out of the moment loop.
__device__ __forceinline__ void resolve_tied_corr(const AlignJob* __restrict__ job, AlignState* st, const CloudDev& tgt,
                                               bool tied, int i, float kd, int& j, NfWaveStack* S,
                                               bool q_in_regs = false, float qx = 0.f, float qy = 0.f, float qz = 0.f) {
  unsigned long long tm = __ballot(tied);
  const int lane = lane_id();
  const NfTreeDev t = job->tgt_nf;
  if (t.nodes == nullptr) {
    if (lane == __builtin_ctzll(tm)) st->tie_pending = 1;
    return;
  }
  if (*job->tgt_nf_status) {   // the tree build failed: keep the Morton-order answers, report
    if (lane == __builtin_ctzll(tm)) atomicOr(&st->tie_err, 2);
    return;
  }
  int nres = 0;
  while (tm) {
    const int l = __builtin_ctzll(tm);
    tm &= tm - 1;
    const int il = __builtin_amdgcn_readlane(i, l);
    const float dl = __uint_as_float((unsigned)__builtin_amdgcn_readlane((int)__float_as_uint(kd), l));
    // the search's fp32 query (trans_f * a_i, :240,253)
    const float4 q = q_in_regs ? make_float4(readlane_f(qx, l), readlane_f(qy, l), readlane_f(qz, l), 0.f)
                               : ldg4(job->qstate, il);
    float rd;
    int rix;
    int err = 0, jn = -1;
    const bool ok = nf_search_wave(t, q.x, q.y, q.z, 1, S, &rd, &rix);
    // lane 0 holds the (k = 1) result
    rd = __uint_as_float((unsigned)__builtin_amdgcn_readfirstlane((int)__float_as_uint(rd)));
    rix = __builtin_amdgcn_readfirstlane(rix);
    if (!ok) err = 1;
    else if (__float_as_uint(rd) != __float_as_uint(dl) || rix < 0 || rix >= t.n) err = 16;
    else if ((jn = tgt.inv_perm[rix]) < 0) err = 32;
    if (lane == l) {
      if (jn >= 0) j = jn;
      else atomicOr(&st->tie_err, err);
    }
    ++nres;
  }
  if (lane == 0) atomicAdd(&st->ties_resolved, nres);
}

// FUSE_LM: the LM step runs in the last block to finish (one block per CU:
// 256 blocks), handed off without a release fence -- each block stores its
// slab row write-through (sc1), drains it (vmcnt(0)), and one lane adds to
// an arrival counter (memory-side atomic); the block that arrives last takes
// one agent-scope acquire and reads the slab with plain loads
// (MI355X_MICROARCH.md "visibility", the split-K form of Guideline 16).
// LOOKUP (candidate cells without any fallback cell): the correspondence
// lookup of k_cell_lookup is done here, one query per lane, and the match's
// coordinates come from its list entry -- no lookup kernel, no key / sec
// round trip.  Same keys, ties and moments as k_cell_lookup + k_moments.
// Fused lookup: list entries loaded per round (clamped loads, no branch).
// 16 measured 2-4 % faster on cfg 3 than 8 (the waves are 2 per SIMD, so the
// registers are free); 12, 32, exec-masked loads, two rounds in flight (8 or
// 12 per round) and a flat wavefront-wide scan of all 64 lists (LDS atomic
// min per owner) all slower: the lookup is bound by the memory system's
// throughput of scattered lines, not by the rounds' latency
// (tools/mom_timeline.py; -DDDLO_LOOKUP_U for A/B builds).
#ifndef DDLO_LOOKUP_U
#define DDLO_LOOKUP_U 16
#endif
constexpr int kLookupU = DDLO_LOOKUP_U;

// developer build (-DDDLO_MOM_PROF): a wave timeline of the fused-lookup
// moment kernel, s_memrealtime stamps (100 MHz, one clock for the device)
// printed by every 16th wavefront
#ifdef DDLO_MOM_PROF
#define MOM_PROF(i) if (LOOKUP) mp_t[i] = __builtin_amdgcn_s_memrealtime()
constexpr int kMomProfIters = 8, kMomProfWaves = 2048;
__device__ unsigned long long g_mom_prof[kMomProfIters * kMomProfWaves * 6];   // [iteration][wave][stamp]
#else
#define MOM_PROF(i)
#endif
// Copy the state to the host-mapped slot, then its publication word
// (AlignState::pub: ticket, done, iter) after a system-scope fence, so the
// host that sees the word reads a complete state.  Whole block.
__device__ __forceinline__ void publish_state(const AlignJob* __restrict__ job, const AlignState* __restrict__ st,
                                              AlignState* __restrict__ publish) {
  static_assert(sizeof(AlignState) % 16 == 0, "AlignState is copied in 16-byte words");
  static_assert(offsetof(AlignState, pub) == sizeof(AlignState) - 8, "the publication word is the last 8 bytes");
  __threadfence();   // this block's state stores, then an L1 invalidate before they are read back
  __syncthreads();
  const int4* src = reinterpret_cast<const int4*>(st);
  int4* dst = reinterpret_cast<int4*>(publish);
  for (int w = threadIdx.x; w < (int)(sizeof(AlignState) / 16); w += blockDim.x) dst[w] = src[w];
  const unsigned long long tk = job->ticket;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long w = (tk << 17) | ((unsigned long long)(st->done != 0) << 16) | ((unsigned)st->iter & 0xffffu);
    __hip_atomic_store(&publish->pub, w, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <bool FUSE_LM, bool LOOKUP = false>
__global__ __launch_bounds__(64 * kMomWaves) void k_moments(const AlignJob* __restrict__ job,
                                                            AlignState* __restrict__ st, AlignState* __restrict__ publish) {
#ifdef DDLO_MOM_PROF
  unsigned long long mp_t[6] = {0, 0, 0, 0, 0, 0};
#endif
  MOM_PROF(0);
  // st (= job->state) is a kernel argument and the pose is loaded with the
  // done flag, before the test: the state words are one load from the
  // arguments, not three dependent ones (job -> state -> done -> pose)
  const auto sg = gp(st);
  double R[9], t[3];
  for (int e = 0; e < 9; ++e) R[e] = sg->R[e];
  for (int e = 0; e < 3; ++e) t[e] = sg->t[e];
  const int st_rec = sg->rec, st_any_rec = sg->any_rec;
  if (__builtin_amdgcn_readfirstlane(sg->done)) {
    // a no-op iteration after convergence: the chunk's publication still
    // happens (as k_lm_step's after an early exit), by block 0
    if (FUSE_LM && publish && blockIdx.x == 0) publish_state(job, st, publish);
    return;
  }
  const CloudDev src = job->src;
  const CloudDev tgt = job->tgt;
  const auto src_cov = gp(job->src_cov);
  const auto tgt_cov = gp(job->tgt_cov);
  const auto key = gp((const unsigned long long*)job->key);
  const auto corr = gpw(job->corr);
  const auto sqd = gpw(job->sqd);
  const auto slab = gpw(job->slab);
  const double max_corr2 = job->max_corr2;
  const int rec = st_rec;   // this iteration records reuse references
  const int first_rec_done = st_any_rec;   // an earlier iteration of this align recorded
  const int tie_detect = job->tie_detect;
  const bool slice_check = tie_detect && job->tie_scan >= 2 && !(job->tie_ab & 4);
  const bool tie3m = tie_detect && job->tie_scan == 3 && !rec;   // the mirrored key of a non-recording search
  __shared__ NfWaveStack tie_stk[kMomWaves];   // nanoflann search frames of a tied query (per wave)
  const int lane = lane_id();
  const int wib = threadIdx.x >> 6;
#ifdef DDLO_MOM_PROF
  __builtin_amdgcn_s_waitcnt(0);
#endif
  MOM_PROF(1);
  const int wave = blockIdx.x * kMomWaves + wib;
  const int nwaves_total = gridDim.x * kMomWaves;
  const int ngroups = (src.n + 63) >> 6;
  // the search's task counters are free again: zero them for the next one
  if (blockIdx.x == 0 && threadIdx.x < kTaskCounters) job->task_ctr[threadIdx.x * kCtrStride] = 0u;
  if (blockIdx.x == 0 && job->grid_on && threadIdx.x == 0) {   // the walk list is consumed: its total, then reset
    unsigned t = 0;
    for (int sg = 0; sg < kFbSegs; ++sg) t += job->fb_count[sg * 32];
    job->fb_count[kFbSegs * 32] += t;
    for (int sg = 0; sg < kFbSegs; ++sg) job->fb_count[sg * 32] = 0u;
  }
  double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
  for (int g = wave; g < ngroups; g += nwaves_total) {
    const int i = g * 64 + lane;
    const bool active = i < src.n;
    // the search result key -> correspondences_ / sq_distances_
    // (nano_gicp_impl.hpp:257-258): a match iff a point was found and its
    // squared distance, promoted to double, is below max_corr^2
    int j = -1;
    unsigned kj = 0xffffffffu;
    float kd = INFINITY;
    bool tied = false;
    // the moment operands (a, b, their covariances) are loaded before the tie
    // checks, so those loads overlap them; a re-run query reloads its b
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    double ca[6] = {0, 0, 0, 0, 0, 0}, cb[6] = {0, 0, 0, 0, 0, 0};
    float lqx = 0.f, lqy = 0.f, lqz = 0.f;   // LOOKUP: the fp32 query
    unsigned long long lkey = 0ull;
    unsigned lsec = 0xffffffffu;
    if constexpr (LOOKUP) {
      // k_cell_lookup's arithmetic, one lane per query
      const CellGridDev G = job->grid;
      a = ldg4(src.pts, active ? i : src.n - 1);
      const float Rf0 = (float)R[0], Rf1 = (float)R[1], Rf2 = (float)R[2], Rf3 = (float)R[3], Rf4 = (float)R[4],
                  Rf5 = (float)R[5], Rf6 = (float)R[6], Rf7 = (float)R[7], Rf8 = (float)R[8];
      const float tf0 = (float)t[0], tf1 = (float)t[1], tf2 = (float)t[2];
      lqx = (Rf0 * a.x + Rf1 * a.y) + (Rf2 * a.z + tf0);
      lqy = (Rf3 * a.x + Rf4 * a.y) + (Rf5 * a.z + tf1);
      lqz = (Rf6 * a.x + Rf7 * a.y) + (Rf8 * a.z + tf2);
      const int g16 = i >> 4;
      const float qa = job->own_axis == 0 ? lqx : job->own_axis == 1 ? lqy : lqz;
      const bool owned = active && (job->own_axis < 0 || (qa >= job->own_lo && qa < job->own_hi)) &&
                         (job->own_mod == 0 || (g16 % job->own_mod) == job->own_rem);
      unsigned off = 0, cnt = 0;
      if (owned) {
        const float tx = (lqx - G.ox) * G.inv_s, ty = (lqy - G.oy) * G.inv_s, tz = (lqz - G.oz) * G.inv_s;
        if (tx >= 0.f && tx < (float)G.nx && ty >= 0.f && ty < (float)G.ny && tz >= 0.f && tz < (float)G.nz) {
          cg_cell_list(G, tx, ty, tz, off, cnt);   // (no fallback cell in LOOKUP mode)
        }
      }
      unsigned long long bk = ~0ull;
      float d2 = INFINITY, bx = 0.f, by = 0.f, bz = 0.f;
      const bool track2 = tie_detect;   // the second distance only feeds the tie test
      constexpr int kU = kLookupU;   // loads in flight
      auto consume = [&](const float4 (&pp)[kU], unsigned k) {
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          if (k + u < cnt) {
            const float dd = dist2(lqx, lqy, lqz, pp[u].x, pp[u].y, pp[u].z);
            const unsigned long long kk = dkey(dd, __float_as_int(pp[u].w));
            if (kk < bk) {
              if (track2 && bk != ~0ull) d2 = fminf(d2, __uint_as_float((unsigned)(bk >> 32)));
              bk = kk;
              bx = pp[u].x;
              by = pp[u].y;
              bz = pp[u].z;
            } else if (track2) {
              d2 = fminf(d2, dd);
            }
          }
        }
      };
      auto fetch = [&](float4 (&pp)[kU], unsigned k) {
#pragma unroll
        for (int u = 0; u < kU; ++u) pp[u] = ldg4(G.ent, off + min(k + u, cnt - 1));
      };
      for (unsigned k = 0; k < cnt; k += kU) {
        float4 pp[kU];
        fetch(pp, k);
        consume(pp, k);
      }
      lkey = owned ? umin64(bk, dkey(job->cap2, -1)) : dkey(INFINITY, -1);
      const float lkd = __uint_as_float((unsigned)(lkey >> 32));
      lsec = (owned && (unsigned)lkey != 0xffffffffu && d2 == lkd) ? (unsigned)(lkey >> 32) : 0xffffffffu;
      b = make_float4(bx, by, bz, 0.f);

      MOM_PROF(2);
    }
    if (active) {
      const unsigned long long k = LOOKUP ? lkey : key[i];
      // independent of the key: issued with it
      const unsigned sv = !tie_detect ? 0xffffffffu : LOOKUP ? lsec : job->sec[i];
      const unsigned k2lo = (tie3m && !LOOKUP) ? (unsigned)job->key2[i] : 0u;
      kj = (unsigned)k;
      kd = __uint_as_float((unsigned)(k >> 32));
      j = (kj != 0xffffffffu && (double)kd < max_corr2) ? (int)kj : -1;
      if (j >= 0) {
        if constexpr (!LOOKUP) {   // (LOOKUP: a and b are in registers already)
          a = ldg4(src.pts, i);
          b = ldg4(tgt.pts, j);
        }

        load_sym6(src_cov + 6 * (size_t)i, ca);
        load_sym6(tgt_cov + 6 * (size_t)j, cb);
      }
      // another examined point at the nearest distance: an exact tie.  sec:
      // all ones = not searched (a reuse reference proved the match), else
      // the smallest distance met twice / of a non-best point (never below
      // the key's); tie_scan 3 also: the mirrored key names another point
      const bool searched = tie_detect && j >= 0 && sv != 0xffffffffu;
      tied = searched && sv <= (unsigned)(k >> 32);
      if (tie3m && searched && !LOOKUP) tied = tied || k2lo != ((unsigned)k ^ 0xffffffffu);
      // tie_scan >= 2: the scan compares only the 8-point slices' bests, so a
      // second point at the distance inside the winner's own slice (the 8
      // aligned sorted positions one lane scanned; the same 128-B line as the
      // winner) is checked here, in the scan's fp32 arithmetic
      if (slice_check && searched && !tied) {
        // the search's fp32 query, recomputed (k_nn_seed's transform, same operations)
        const float qx = ((float)R[0] * a.x + (float)R[1] * a.y) + ((float)R[2] * a.z + (float)t[0]);
        const float qy = ((float)R[3] * a.x + (float)R[4] * a.y) + ((float)R[5] * a.z + (float)t[1]);
        const float qz = ((float)R[6] * a.x + (float)R[7] * a.y) + ((float)R[8] * a.z + (float)t[2]);
        const int b0 = j & ~7;
#pragma unroll
        for (int h = 0; h < 8; ++h) {
          const float4 p = ldg4(tgt.pts, b0 + h);
          tied = tied || (b0 + h != j && dist2(qx, qy, qz, p.x, p.y, p.z) == kd);
        }
      }
    }
    // nanoflann's choice among the tied points (wave-uniform, rare)
    if (tie_detect && __any(tied)) {
      const int j0 = j;
      resolve_tied_corr(job, st, tgt, tied, i, kd, j, &tie_stk[wib], LOOKUP, lqx, lqy, lqz);
      if (tied) kj = (unsigned)j;
      if (j != j0) {   // another point of the same distance: its coordinates and covariance
        b = ldg4(tgt.pts, j);
        load_sym6(tgt_cov + 6 * (size_t)j, cb);
      }
    }
    if (active) {
      corr[i] = j;
      sqd[i] = kj != 0xffffffffu ? kd : INFINITY;
      // reuse reference of a query searched in a recording iteration: its
      // position, B^2 = min(smallest distance of an examined non-best point,
      // walk radius) — every unexamined point lies in a leaf farther than the
      // walk radius — and its match.  A reference stays a valid proof for
      // the rest of the align (same target), so other iterations keep it.
      if (rec && !LOOKUP) {   // (LOOKUP: no walk, so no reference is ever checked)
        const float4 qs = ldg4(job->qstate, i);
        if (qs.w >= 0.f) {
          job->ref[i] = make_float4(qs.x, qs.y, qs.z, fminf(__uint_as_float(job->sec[i]), qs.w));
          float4 pp = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
          if (kj != 0xffffffffu) {
            const float4 p = ldg4(tgt.pts, (int)kj);
            pp = make_float4(p.x, p.y, p.z, __int_as_float((int)kj));
          }
          job->ref_p[i] = pp;
        } else if (!first_rec_done) {
          // the align's first recording iteration: a query it did not search
          // (another shard's) must not keep a previous align's reference
          job->ref[i] = make_float4(0.f, 0.f, 0.f, -1.f);
        }
      }
    }
    Contrib C;
    if (j >= 0) {
      const double A[9] = {ca[0], ca[1], ca[2], ca[1], ca[3], ca[4], ca[2], ca[4], ca[5]};
      // RC = R * CA ; S = RC * R^T ; RCR = CB + S
      double RC[9];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) RC[3 * r + cc] = R[3 * r] * A[cc] + R[3 * r + 1] * A[3 + cc] + R[3 * r + 2] * A[6 + cc];
      double S[9];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) S[3 * r + cc] = RC[3 * r] * R[3 * cc] + RC[3 * r + 1] * R[3 * cc + 1] + RC[3 * r + 2] * R[3 * cc + 2];
      const double Cm[9] = {cb[0] + S[0], cb[1] + S[1], cb[2] + S[2], cb[1] + S[3], cb[3] + S[4],
                            cb[4] + S[5], cb[2] + S[6], cb[4] + S[7], cb[5] + S[8]};
      double Mi[9];
      inv3(Cm, Mi);
      C.M[0] = Mi[0]; C.M[1] = 0.5 * (Mi[1] + Mi[3]); C.M[2] = 0.5 * (Mi[2] + Mi[6]);
      C.M[3] = Mi[4]; C.M[4] = 0.5 * (Mi[5] + Mi[7]); C.M[5] = Mi[8];
      const double ax = a.x, ay = a.y, az = a.z;
      C.q[0] = (R[0] * ax + R[1] * ay) + (R[2] * az + t[0]);
      C.q[1] = (R[3] * ax + R[4] * ay) + (R[5] * az + t[1]);
      C.q[2] = (R[6] * ax + R[7] * ay) + (R[8] * az + t[2]);
      const double e0 = (double)b.x - C.q[0], e1 = (double)b.y - C.q[1], e2 = (double)b.z - C.q[2];
      C.v[0] = C.M[0] * e0 + C.M[1] * e1 + C.M[2] * e2;
      C.v[1] = C.M[1] * e0 + C.M[3] * e1 + C.M[4] * e2;
      C.v[2] = C.M[2] * e0 + C.M[4] * e1 + C.M[5] * e2;
      C.y = e0 * C.v[0] + e1 * C.v[1] + e2 * C.v[2];
      C.c = 1.0;
    } else {
      for (int e = 0; e < 6; ++e) C.M[e] = 0.0;
      C.q[0] = C.q[1] = C.q[2] = 0.0;
      C.v[0] = C.v[1] = C.v[2] = 0.0;
      C.y = 0.0;
      C.c = 0.0;
    }
    C.qq[0] = C.q[0] * C.q[0]; C.qq[1] = C.q[0] * C.q[1]; C.qq[2] = C.q[0] * C.q[2];
    C.qq[3] = C.q[1] * C.q[1]; C.qq[4] = C.q[1] * C.q[2]; C.qq[5] = C.q[2] * C.q[2];
    MOM_PROF(3);
    acc0 += final_pair(treduce<5, 0>(C));
    acc1 += final_pair(treduce<5, 1>(C));
    acc2 += final_pair(treduce<5, 2>(C));
  }
  MOM_PROF(4);
  __shared__ double red[kMomWaves][kMomentSlots];
  if ((lane & 1) == 0) {
    const int base = moment_base(lane);
    red[wib][base + 0] = acc0;
    red[wib][base + 1] = acc1;
    red[wib][base + 2] = acc2;
  }
  __syncthreads();
  if (threadIdx.x < kSlabStride) {
    double sum = 0.0;
    if (threadIdx.x < kMoments)
      for (int w = 0; w < kMomWaves; ++w) sum += red[w][threadIdx.x];
    if constexpr (FUSE_LM)
      __hip_atomic_store((__attribute__((address_space(1))) unsigned long long*)(slab + (size_t)blockIdx.x * kSlabStride +
                                                                                 threadIdx.x),
                         (unsigned long long)__double_as_longlong(sum), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      slab[(size_t)blockIdx.x * kSlabStride + threadIdx.x] = sum;
  }
#ifdef DDLO_MOM_PROF
  MOM_PROF(5);
  if (LOOKUP && lane == 0 && wave < kMomProfWaves) {
    unsigned long long* o = g_mom_prof + ((size_t)min(st->iter, kMomProfIters - 1) * kMomProfWaves + wave) * 6;
    for (int e = 0; e < 6; ++e) o[e] = mp_t[e];
  }
#endif
  if constexpr (FUSE_LM) {
    __shared__ int last_s;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave: its sc1 slab stores are done
    __syncthreads();
    unsigned* const arrive = job->task_ctr + kTaskCounters * kCtrStride;
    if (threadIdx.x == 0) last_s = atomicAdd(arrive, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!last_s) return;
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      atomicExch(arrive, 0u);   // re-armed for the next iteration (k_align_init zeroes it per align)
    }
    __syncthreads();
    lm_step_body<false>(job, st, job->slab, job->nblocks, nullptr);
    if (publish) publish_state(job, st, publish);
  }
}
template __global__ void k_moments<false>(const AlignJob*, AlignState*, AlignState*);
template __global__ void k_moments<true>(const AlignJob*, AlignState*, AlignState*);
template __global__ void k_moments<false, true>(const AlignJob*, AlignState*, AlignState*);
template __global__ void k_moments<true, true>(const AlignJob*, AlignState*, AlignState*);

// ---------------------------------------------------------------------------
// K5: slab reduction + LM/GN step on one workgroup.
__device__ void so3_exp_d(const double w[3], double R[9]) {  // gicp/so3.hpp:101-124
  const double theta_sq = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  double imag, real;
  if (theta_sq < 1e-10) {
    const double theta_quad = theta_sq * theta_sq;
    imag = 0.5 - 1.0 / 48.0 * theta_sq + 1.0 / 3840.0 * theta_quad;
    real = 1.0 - 1.0 / 8.0 * theta_sq + 1.0 / 384.0 * theta_quad;
  } else {
    const double theta = sqrt(theta_sq);
    const double half = 0.5 * theta;
    double sh, ch;
    sincos(half, &sh, &ch);   // one argument reduction for both
    imag = sh / theta;
    real = ch;
  }
  const double qw = real, qx = imag * w[0], qy = imag * w[1], qz = imag * w[2];
  const double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
  const double twx = tx * qw, twy = ty * qw, twz = tz * qw;
  const double txx = tx * qx, txy = ty * qx, txz = tz * qx;
  const double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

// Eigen::LDLT<Matrix6d>(H + lambda I).solve(rhs) (restated, see oracle).
// Eigen's pivoted LDLT (ldlt_inplace) is left-looking: step k updates only
// row / column k, so the diagonal entries k..5 its pivot search reads are
// still A's own and the transpositions follow from diag(A) alone.  They are
// found first; the factorization then runs unpivoted on the lower triangle of
// P A P^T, gathered from LDS — the same operations on the same values as
// swapping rows and columns in place (checked bit for bit against that form
// on 2M random, tied and rank-deficient systems), without its select chains.
// H, b: LDS (H's lower triangle is read, as Eigen's Lower LDLT); rhs = -b;
// xs: this thread's 6-double LDS row for the un-permuting scatter.  Every
// register-array index is a compile-time constant (no scratch).
__device__ void ldlt_solve6_perm(const double* H, const double* b, double lambda, double* xs, double x[6]) {
  constexpr int n = 6;
  double v[6];
  int p[6];
#pragma unroll
  for (int i = 0; i < n; ++i) {
    v[i] = fabs(H[7 * i] + lambda);
    p[i] = i;
  }
#pragma unroll
  for (int k = 0; k < n - 1; ++k) {
    // the first largest of v[k..5] (Eigen's maxCoeff keeps the first), swapped to k
    double bv = v[k];
    int bp = p[k], big = k;
#pragma unroll
    for (int i = k + 1; i < n; ++i)
      if (v[i] > bv) { bv = v[i]; bp = p[i]; big = i; }
#pragma unroll
    for (int i = k + 1; i < n; ++i)
      if (big == i) { v[i] = v[k]; p[i] = p[k]; }
    v[k] = bv;
    p[k] = bp;
  }
  double m[36];
#pragma unroll
  for (int i = 0; i < n; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      const int hi = max(p[i], p[j]), lo = min(p[i], p[j]);
      m[i * n + j] = i == j ? H[7 * p[i]] + lambda : H[hi * n + lo];
    }
#pragma unroll
  for (int k = 0; k < n; ++k) {
    if (k > 0) {
      double temp[6];
#pragma unroll
      for (int j = 0; j < k; ++j) temp[j] = m[j * n + j] * m[k * n + j];
      double s = 0;
#pragma unroll
      for (int j = 0; j < k; ++j) s += m[k * n + j] * temp[j];
      m[k * n + k] -= s;
#pragma unroll
      for (int i = k + 1; i < n; ++i) {
        double a = 0;
#pragma unroll
        for (int j = 0; j < k; ++j) a += m[i * n + j] * temp[j];
        m[i * n + k] -= a;
      }
    }
    const double akk = m[k * n + k];
    if (k < n - 1 && fabs(akk) > 0.0) {
#pragma unroll
      for (int i = k + 1; i < n; ++i) m[i * n + k] /= akk;
    }
  }
  double y[6];
#pragma unroll
  for (int i = 0; i < n; ++i) y[i] = -b[p[i]];   // P rhs
#pragma unroll
  for (int i = 0; i < n; ++i)
#pragma unroll
    for (int j = 0; j < i; ++j) y[i] -= m[i * n + j] * y[j];
#pragma unroll
  for (int i = 0; i < n; ++i) y[i] = (fabs(m[i * n + i]) > 2.2250738585072014e-308) ? y[i] / m[i * n + i] : 0.0;
#pragma unroll
  for (int i = n - 1; i >= 0; --i)
#pragma unroll
    for (int j = i + 1; j < n; ++j) y[i] -= m[j * n + i] * y[j];
#pragma unroll
  for (int i = 0; i < n; ++i) xs[p[i]] = y[i];   // P^T y
#pragma unroll
  for (int i = 0; i < n; ++i) x[i] = xs[i];
}

// Moment slots.  W(k,l) = sum M qt_k qt_l (qt = [q;1]), G(m,k) = sum (Me)_m qt_k.
constexpr int mom_ab(int a, int b) {   // symmetric 3 x 3 (a, b) -> 0..5
  return a <= b ? (a == 0 ? b : (a == 1 ? 2 + b : 5)) : (b == 0 ? a : (b == 1 ? 2 + a : 5));
}
constexpr int mom_w(int k, int l, int a, int b) {   // (a, b) entry of W(k, l)
  return (k == 3 && l == 3) ? mom_ab(a, b)
         : k == 3           ? 6 + 6 * l + mom_ab(a, b)
         : l == 3           ? 6 + 6 * k + mom_ab(a, b)
                            : 24 + 6 * mom_ab(k, l) + mom_ab(a, b);
}
constexpr int mom_g(int mm, int k) { return 60 + 4 * mm + k; }
constexpr int kMomY0 = 72, kMomCount = 73;

// The LM step's inputs from the moments, one entry per thread through a
// compile-time table of signed moment slots summed in order:
//   [0, 36)  H = sum J^T M J, [36, 42) b = sum J^T M e, J = [skew(q) | -I]
//            (nano_gicp_impl.hpp:317-324);
//   [42, 186) W12[3k + a][3l + b] = W(k,l)[a][b], [186, 198) g12[3k + r] = G(r, k):
//            the trials' cost decrease y0 - y(delta) = 2 <g12, d> - d^T W12 d over
//            d = vec([Rd - I | td]) (e' = e - D qt for the frozen correspondences).
// Column i of the skew generators S_c has two non-zeros S_c[r][i] = +-1,
// ordered by c, so H_rr(i,j) = sum_{c,d,r,q} S_c[r][i] W(c,d)[r][q] S_d[q][j]
// is a 4-term signed sum (the same products in the same order as the full one).
constexpr int kNeqEntries = 198;
struct NeqTerm {       // packed into three registers: byte t of idx / sgn is term t
  unsigned idx;        // moment slots
  unsigned sgn;        // signs: 1 = +1, 0xff = -1
  unsigned ctl;        // bits 0-7: term count, bit 8: negate the sum
};
struct NeqTable {
  NeqTerm e[kNeqEntries];
};
constexpr void skew_nz_c(int i, int p, int& c, int& r, int& sg) {
  // i=0: S_1[2][0]=-1, S_2[1][0]=+1; i=1: S_0[2][1]=+1, S_2[0][1]=-1; i=2: S_0[1][2]=-1, S_1[0][2]=+1
  constexpr int cc[3][2] = {{1, 2}, {0, 2}, {0, 1}};
  constexpr int rr[3][2] = {{2, 1}, {2, 0}, {1, 0}};
  constexpr int ss[3][2] = {{-1, 1}, {1, -1}, {-1, 1}};
  c = cc[i][p];
  r = rr[i][p];
  sg = ss[i][p];
}
constexpr NeqTable make_neq_table() {
  NeqTable T{};
  auto add = [&](int e, int idx, int sg) {
    const unsigned t = T.e[e].ctl & 0xffu;
    T.e[e].idx |= (unsigned)idx << (8 * t);
    T.e[e].sgn |= (sg < 0 ? 0xffu : 1u) << (8 * t);
    T.e[e].ctl += 1u;
  };
  for (int e = 0; e < 42; ++e) {
    if (e >= 36) {
      const int i = e - 36;
      if (i >= 3) {
        add(e, mom_g(i - 3, 3), -1);   // b_t = -G(:,3)
      } else {                         // b_r(i) = sum_c sum_r S_c[r][i] G(r,c)
        for (int p = 0; p < 2; ++p) {
          int c = 0, r = 0, sg = 0;
          skew_nz_c(i, p, c, r, sg);
          add(e, mom_g(r, c), sg);
        }
      }
      continue;
    }
    const int i = e / 6, j = e % 6;
    if (i < 3 && j < 3) {
      for (int p = 0; p < 2; ++p) {
        int c = 0, r = 0, sr = 0;
        skew_nz_c(i, p, c, r, sr);
        for (int u = 0; u < 2; ++u) {
          int d = 0, q = 0, sq = 0;
          skew_nz_c(j, u, d, q, sq);
          add(e, mom_w(c, d, r, q), sr * sq);
        }
      }
    } else if (i >= 3 && j >= 3) {
      add(e, mom_w(3, 3, i - 3, j - 3), 1);   // H_tt = sum M
    } else {   // H_rt(a, t) = -sum_c sum_r S_c[r][a] W(c,3)[r][t]
      const int a = i < 3 ? i : j, t = i < 3 ? j - 3 : i - 3;
      for (int p = 0; p < 2; ++p) {
        int c = 0, r = 0, sr = 0;
        skew_nz_c(a, p, c, r, sr);
        add(e, mom_w(c, 3, r, t), sr);
      }
      T.e[e].ctl |= 0x100u;
    }
  }
  for (int e = 0; e < 144; ++e) add(42 + e, mom_w(e / 12 / 3, e % 12 / 3, e / 12 % 3, e % 12 % 3), 1);
  for (int e = 0; e < 12; ++e) add(186 + e, mom_g(e % 3, e / 3), 1);
  return T;
}
__constant__ NeqTable kNeq = make_neq_table();
// One table entry: a single slot is taken as is (times +-1, exact); a sum
// starts from 0.0 and adds its terms in order (as the loops it restates).
__device__ __forceinline__ double neq_term(const NeqTerm& E, const double* mom, int t) {
  const double v = mom[(E.idx >> (8 * t)) & 0xffu];
  return ((E.sgn >> (8 * t)) & 0xffu) == 1u ? v : -v;
}
__device__ __forceinline__ double neq_value(const NeqTerm& E, const double* mom) {
  const unsigned n = E.ctl & 0xffu;
  double s = neq_term(E, mom, 0);
  if (n > 1) {
    s = 0.0 + s;
#pragma unroll
    for (int t = 1; t < 4; ++t)
      if (t < (int)n) s += neq_term(E, mom, t);
  }
  return (E.ctl & 0x100u) ? -s : s;
}

constexpr int kLmThreads = 512;
constexpr int kMaxTrials = 64;
constexpr int kMomBlocksMax = 256;                      // moment-kernel blocks (slab rows)
constexpr int kLmParts = 12;                                          // slab row partitions
// (1024 threads, 25 partitions of 11 rows: reduction 5.5k -> 5.8k cycles, no gain)
constexpr int kLmRowsPerPart = (kMomBlocksMax + kLmParts - 1) / kLmParts;  // slab rows per reducer thread

// Fixed-order reduction of the linearize slab (nblocks x kSlabStride) into
// mom[kSlabStride] by one workgroup: thread (p, v2) sums column pair v2 of
// rows p, p + 12, ... with 16-byte loads (kLmParts x 40 threads), then 80
// threads add the 12 partials in order (fixed order => deterministic).
// mom is complete after the caller's next barrier.
__device__ __forceinline__ void reduce_slab(const double* slab_in, int nb, double (*part)[kSlabStride], double* mom) {
  const int tid = threadIdx.x;
  const auto slab = (const __attribute__((address_space(1))) d2v*)gp(slab_in);
  constexpr int kPairs = kSlabStride / 2;
  if (tid < kLmParts * kPairs) {
    // unconditional (clamped) loads into registers, all issued before the
    // in-order adds consume them (one memory latency, not one per batch the
    // scheduler would otherwise interleave with the adds)
    const int v2 = tid % kPairs, p = tid / kPairs;
    d2v x[kLmRowsPerPart];
#pragma unroll
    for (int r = 0; r < kLmRowsPerPart; ++r) x[r] = slab[(size_t)min(p + kLmParts * r, nb - 1) * kPairs + v2];
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int r = 0; r < kLmRowsPerPart; ++r) {
      const bool in = p + kLmParts * r < nb;
      s0 += in ? x[r].x : 0.0;
      s1 += in ? x[r].y : 0.0;
    }
    part[p][2 * v2] = s0;
    part[p][2 * v2 + 1] = s1;
  }
  __syncthreads();
  if (tid < kSlabStride) {
    double s = 0.0;
#pragma unroll
    for (int p = 0; p < kLmParts; ++p) s += part[p][tid];
    mom[tid] = s;
  }
}

// K5a (sharded align only): this rank's reduced moments -> job->mom, which
// the host's all-reduce then sums across ranks before k_lm_step.
__global__ __launch_bounds__(kLmThreads) void k_mom_reduce(const AlignJob* __restrict__ job) {
  AlignState* st = job->state;
  if (__builtin_amdgcn_readfirstlane(st->done)) return;
  __shared__ double part[kLmParts][kSlabStride];
  __shared__ double mom[kSlabStride];
  reduce_slab(job->slab, job->nblocks, part, mom);
  __syncthreads();
  if (threadIdx.x < kSlabStride) gpw(job->mom)[threadIdx.x] = mom[threadIdx.x];
}

// One workgroup: (1) fixed-order reduction of the linearize partials,
// (2) H, b and the cost-decrease form one entry per thread, (3) every LM
// trial in its own thread — the reference's trial sequence is fully
// determined up front (lambda_i = nu_{i-1} lambda_{i-1}, nu doubling:
// lsq_registration_impl.hpp:187-223), so trial i is evaluated with exactly
// the lambda the sequential loop would use, (4) wavefront 0 takes the
// sequential accept/reject decisions as one ballot and stores the new state
// while the other wavefronts store the per-linearize record.  Every state
// and job word is loaded at the start (its latency hides behind the slab).
#ifdef DDLO_LM_PROF   // developer build (make lmprof): per-phase cycle counts of one LM step, printed by thread 0
#define LM_PROF(i) if (threadIdx.x == 0) lm_t[i] = __builtin_amdgcn_s_memtime()
#define LM_PROF_TRIAL(i) if (threadIdx.x == 0) lm_tt[i] = __builtin_amdgcn_s_memtime()
#else
#define LM_PROF(i)
#define LM_PROF_TRIAL(i)
#endif
// st, slab, nblocks: job->state, job->slab, job->nblocks, passed as kernel
// arguments so the slab loads need no job load first; premom (PREMOM): the
// moments already reduced (and summed across shards: job->mom).
template <bool PREMOM>
__device__ __forceinline__ void lm_step_body(const AlignJob* __restrict__ job, AlignState* __restrict__ st,
                                             const double* __restrict__ slab, int nblocks,
                                             const double* __restrict__ premom) {
#ifdef DDLO_LM_PROF
  unsigned long long lm_t[6], lm_tt[4] = {0, 0, 0, 0};
#endif
  LM_PROF(0);
  __shared__ double part[kLmParts][kSlabStride];
  __shared__ double mom[kSlabStride];
  __shared__ double nq[kNeqEntries];   // H (36), b (6), W12 (144), g12 (12)
  double* const Hs = nq;
  double* const bs = nq + 36;
  double* const W12 = nq + 42;
  double* const g12 = nq + 186;
  __shared__ double tr_lambda[kMaxTrials], tr_cm[kMaxTrials], tr_fro[kMaxTrials];
  __shared__ double tr_R[kMaxTrials][9], tr_t[kMaxTrials][3];
  __shared__ double tr_d[kMaxTrials][12], tr_row[kMaxTrials][12], tr_den[kMaxTrials], tr_x[kMaxTrials][6];
  __shared__ double Rt_s[12];
  __shared__ int tr_conv[kMaxTrials];
  const int tid = threadIdx.x;
  // state words, loaded before the slab (their latency overlaps it)
  const int it_pre = st->iter;
  const int trials_pre = st->lm_trials;
  const int rec_pre = st->rec;
  const float src_radius = st->src_radius;
  const double lambda_pre = st->lambda;
  // the pose, held in a register until the slab loads are issued (an LDS
  // store here would wait for it first)
  double rt_v = 0.0;
  if (tid < 12) rt_v = tid < 9 ? st->R[tid] : st->t[tid - 9];
  // job words and this thread's table entry too (misses at their first use would each stall a phase)
  const int optimizer = job->optimizer, lm_max_iterations = job->lm_max_iterations;
  const int fixed_iterations = job->fixed_iterations, max_iterations = job->max_iterations;
  const double lm_init_lambda_factor = job->lm_init_lambda_factor;
  const double rotation_epsilon = job->rotation_epsilon, transformation_epsilon = job->transformation_epsilon;
  const int reuse = job->reuse;
  const float reuse_rec_eps = job->reuse_rec_eps, reuse_rec_conv = job->reuse_rec_conv;
  NeqTerm E{};
  if (tid < kNeqEntries) E = kNeq.e[tid];
  if constexpr (PREMOM) {  // moments already reduced (and summed across shards)
    if (tid < kSlabStride) mom[tid] = gp(premom)[tid];
  } else {
    reduce_slab(slab, nblocks, part, mom);
  }
  if (tid < 12) Rt_s[tid] = rt_v;
  __syncthreads();
  LM_PROF(1);
  if (tid < kNeqEntries) nq[tid] = neq_value(E, mom);
  __syncthreads();
  LM_PROF(2);
  const bool lm = optimizer != 0;
  const int ntr = lm ? min(lm_max_iterations, kMaxTrials) : 1;
  // one trial per thread (one wavefront issues them all: a trial per
  // wavefront with wave-uniform pivots measured 2x slower, the waves then
  // share the SIMDs' fp64 issue)
  if (tid < ntr) {
    const int trial = tid;
    double lambda = 0.0;
    if (lm) {
      lambda = lambda_pre;
      if (lambda < 0.0) {   // the first LM step: lm_init_lambda_factor * max |diag H| (:180-183)
        double mx = 0.0;
        for (int e = 0; e < 6; ++e) mx = fmax(mx, fabs(Hs[7 * e]));
        lambda = lm_init_lambda_factor * mx;
      }
      double nu = 2.0;
      for (int k = 0; k < trial; ++k) {
        lambda = nu * lambda;
        nu = 2 * nu;
      }
    }
    LM_PROF_TRIAL(0);
    double d[6];
    ldlt_solve6_perm(Hs, bs, lambda, tr_x[trial], d);   // GN: lambda 0 (H + 0 = H)
    LM_PROF_TRIAL(1);
    double Rd[9], td[3];
    so3_exp_d(d, Rd);
    LM_PROF_TRIAL(2);
    td[0] = d[3]; td[1] = d[4]; td[2] = d[5];
    double den = 0.0;
    for (int e = 0; e < 6; ++e) den += d[e] * (lambda * d[e] - bs[e]);
    tr_den[trial] = den;
    tr_lambda[trial] = lambda;
    // is_converged's measure max((1 / rot_eps) |Rd - I|, (1 / trans_eps) |td|)
    // (lsq_registration_impl.hpp:128-139); the product rounds monotonically,
    // so scaling each largest |x| gives the same maximum
    double mr = 0.0, mt = 0.0;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) mr = fmax(mr, fabs(Rd[3 * i + j] - (i == j ? 1.0 : 0.0)));
    for (int i = 0; i < 3; ++i) mt = fmax(mt, fabs(td[i]));
    const double cm = fmax(1.0 / rotation_epsilon * mr, 1.0 / transformation_epsilon * mt);
    tr_cm[trial] = cm;
    tr_conv[trial] = fixed_iterations <= 0 && cm < 1;
    double fro = 0.0;
    for (int e = 0; e < 9; ++e) {
      const double dd = Rd[e] - ((e % 4 == 0) ? 1.0 : 0.0);
      fro += dd * dd;
    }
    tr_fro[trial] = fro;
    for (int e = 0; e < 9; ++e) tr_R[trial][e] = Rd[e];
    for (int e = 0; e < 3; ++e) tr_t[trial][e] = td[e];
    // d = vec([Rd - I | td]), d[3k + a] = D[a][k]
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int a = 0; a < 3; ++a) tr_d[trial][3 * k + a] = k < 3 ? Rd[3 * a + k] - (a == k ? 1.0 : 0.0) : td[a];
    LM_PROF_TRIAL(3);
  }
  __syncthreads();
  LM_PROF(3);
  // trial cost decrease, one row of the quadratic form per thread: (trial, row) = (x / 12, x % 12)
  for (int x = tid; lm && x < 12 * ntr; x += (int)blockDim.x) {
    const int tr = x / 12, i = x % 12;
    double srow = 0.0;
#pragma unroll
    for (int j = 0; j < 12; ++j) srow += W12[12 * i + j] * tr_d[tr][j];
    tr_row[tr][i] = tr_d[tr][i] * srow;
  }
  __syncthreads();
  LM_PROF(4);
  if (tid >= 64) {
    // the per-linearize record, stored by the other wavefronts while wavefront 0 decides
    const int u = tid - 64;
    if (u < kSlabStride) st->last_mom[u] = mom[u];
    else if (u < kSlabStride + 9) st->last_lin_R[u - kSlabStride] = Rt_s[u - kSlabStride];
    else if (u < kSlabStride + 12) st->last_lin_t[u - kSlabStride - 9] = Rt_s[u - kSlabStride];
    else if (u < kSlabStride + 18) st->last_b[u - kSlabStride - 12] = bs[u - kSlabStride - 12];
    return;
  }
  // wavefront 0: the trials' gain ratios, then step_lm's sequential decisions
  // (:188-231) as one ballot — the first trial that is accepted (rho >= 0, or
  // NaN) or, rejected, has converged; step_gn always takes its step (:155-173)
  const int lane = tid;
  double rho = 1.0;
  if (lm && lane < ntr) {
    double lin = 0.0, quad = 0.0;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int k = 0; k < 4; ++k) lin += tr_d[lane][3 * k + r] * g12[3 * k + r];
#pragma unroll
    for (int i = 0; i < 12; ++i) quad += tr_row[lane][i];
    rho = (2.0 * lin - quad) / tr_den[lane];
  }
  bool ok = true, accept = true;
  int chosen = 0;
  if (lm) {
    const unsigned long long ball = __ballot(lane < ntr && (!(rho < 0) || tr_conv[lane]));
    ok = ball != 0ull;
    chosen = ok ? (int)__builtin_ctzll(ball) : ntr - 1;
    const double rho_c = __shfl(rho, chosen);
    accept = ok && !(rho_c < 0);
    if (lane == 0) {
      st->lm_trials = trials_pre + (ok ? chosen + 1 : ntr);
      if (accept) {
        const double c = 2 * rho_c - 1;
        st->lambda = tr_lambda[chosen] * fmax(1.0 / 3.0, 1 - c * c * c);
      } else if (ok) {
        st->lambda = tr_lambda[chosen];
      } else {
        st->lambda = tr_lambda[ntr - 1] * 2.0;  // not observable: the align ends
      }
    }
  }
  if (lane == 0) {
    st->nr_iterations = it_pre;
    st->final_cost = mom[kMomY0];
    st->num_corr = (int)mom[kMomCount];
    if (rec_pre) st->any_rec = 1;   // this iteration's search recorded references
    st->iter = it_pre + 1;
    st->have_prev = 1;
    int done = 0;
    if (!ok) {
      st->lm_failed = 1;
      done = 1;
    } else if (tr_conv[chosen]) {
      st->converged = 1;
      done = 1;
    }
    if (it_pre + 1 >= max_iterations) done = 1;
    if (done) st->done = 1;
  }
  // accepted: x0 = delta * x0 (compose, lsq_registration_impl.hpp:193-197,225-228),
  // one entry of (Rn | tn) per lane
  double v = 0.0;
  if (accept) {
    const double* Rd = tr_R[chosen];
    if (lane < 9) {
      const int i = lane / 3, j = lane % 3;
      v = Rd[3 * i + 0] * Rt_s[0 + j] + Rd[3 * i + 1] * Rt_s[3 + j] + Rd[3 * i + 2] * Rt_s[6 + j];
      st->R[lane] = v;
    } else if (lane < 12) {
      const int i = lane - 9;
      v = (Rd[3 * i + 0] * Rt_s[9] + Rd[3 * i + 1] * Rt_s[10] + Rd[3 * i + 2] * Rt_s[11]) + tr_t[chosen][i];
      st->t[i] = v;
    } else if (lane >= 16 && lane < 16 + 36) {
      st->final_hessian[lane - 16] = Hs[lane - 16];
    }
  }
  int rec = reuse;
  if (accept) {
    // how far the step moved a source point: |dR q + dt - q| <= |dR - I|_F |q| + |dt|,
    // |q| <= src_radius + |t|; the next search records references only
    // after a small step (the one after it is expected to be smaller) ...
    const double tn0 = __shfl(v, 9), tn1 = __shfl(v, 10), tn2 = __shfl(v, 11);
    const double* dt = tr_t[chosen];
    const double mv = sqrt(tr_fro[chosen]) * ((double)src_radius + sqrt(tn0 * tn0 + tn1 * tn1 + tn2 * tn2)) +
                      sqrt(dt[0] * dt[0] + dt[1] * dt[1] + dt[2] * dt[2]);
    // ... and, with the reference's convergence test on, only while the step
    // is still far from converging (is_converged's measure > reuse_rec_conv):
    // references pay off only if two more iterations follow
    rec = rec && mv < (double)reuse_rec_eps && (fixed_iterations > 0 || tr_cm[chosen] > (double)reuse_rec_conv);
  }
  if (lane == 0) st->rec = rec;
  LM_PROF(5);
#ifdef DDLO_LM_PROF
  if (tid == 0)
    printf("lm_prof %d %llu %llu %llu %llu %llu %llu %llu %llu %llu\n", it_pre, lm_t[1] - lm_t[0], lm_t[2] - lm_t[1],
           lm_t[3] - lm_t[2], lm_t[4] - lm_t[3], lm_t[5] - lm_t[4], lm_tt[0] - lm_t[2], lm_tt[1] - lm_tt[0],
           lm_tt[2] - lm_tt[1], lm_tt[3] - lm_tt[2]);
#endif
}

// publish (optional): a host-mapped AlignState the block copies the final
// state of this step to (also after an early exit), so the host reads a
// chunk's result from pinned memory without a device-to-host copy.
__global__ __launch_bounds__(kLmThreads) void k_lm_step(const AlignJob* __restrict__ job, AlignState* __restrict__ st,
                                                        const double* __restrict__ slab, int nblocks,
                                                        const double* __restrict__ premom,
                                                        AlignState* __restrict__ publish) {
  if (!__builtin_amdgcn_readfirstlane(st->done)) {
    if (premom) lm_step_body<true>(job, st, slab, nblocks, premom);
    else lm_step_body<false>(job, st, slab, nblocks, nullptr);
  }
  if (publish) publish_state(job, st, publish);
}

// ---------------------------------------------------------------------------
// K6: residuals (getResiduals) — unbounded 1-NN for points without a
// correspondence, at the pose of the last linearization.
__global__ __launch_bounds__(256) void k_residuals(const AlignJob* __restrict__ job, double* __restrict__ out) {
  const CloudDev src = job->src;
  const CloudDev tgt = job->tgt;
  const AlignState* st = job->state;
  float Rf[9], tf[3];
  for (int e = 0; e < 9; ++e) Rf[e] = (float)st->last_lin_R[e];
  for (int e = 0; e < 3; ++e) tf[e] = (float)st->last_lin_t[e];
  __shared__ WaveLds lds[4];
  WaveLds* L = &lds[threadIdx.x >> 6];
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves_total = (gridDim.x * blockDim.x) >> 6;
  const int ngroups = (src.n + 63) >> 6;
  for (int g = wave; g < ngroups; g += nwaves_total) {
    const int i = g * 64 + lane_id();
    const bool active = i < src.n;
    float d2 = active ? job->sqd[i] : 0.f;
    const bool need = active && !(d2 < INFINITY);
    if (__any(need)) {
      const float4 a = ldg4(src.pts, active ? i : src.n - 1);
      NN1Visitor vis;
      vis.qx = (Rf[0] * a.x + Rf[1] * a.y) + (Rf[2] * a.z + tf[0]);
      vis.qy = (Rf[3] * a.x + Rf[4] * a.y) + (Rf[5] * a.z + tf[1]);
      vis.qz = (Rf[6] * a.x + Rf[7] * a.y) + (Rf[8] * a.z + tf[2]);
      vis.active = need;
      vis.best = need ? INFINITY : -1.f;
      vis.bestj = -1;
      // seed: the nearest of a Morton window per lane (finite bound)
      if (need) {
        const int pos = min(wave_lower_bound_lane(tgt.keys, tgt.n,
                                                  morton_key(vis.qx, vis.qy, vis.qz, tgt.quant)), tgt.n - 1);
        for (int o = -4; o <= 4; ++o) {
          const int j = pos + o;
          if (j < 0 || j >= tgt.n) continue;
          const float4 p = ldg4(tgt.pts, j);
          const float d = dist2(vis.qx, vis.qy, vis.qz, p.x, p.y, p.z);
          if (d < vis.best || (d == vis.best && (unsigned)j < (unsigned)vis.bestj)) {
            vis.best = d;
            vis.bestj = j;
          }
        }
      }
      vis.skip_lo = 1;
      vis.skip_hi = 0;
      vis.box = make_wave_box(need, vis.qx, vis.qy, vis.qz, vis.best);
      traverse(tgt, vis, L);
      if (need) {
        d2 = vis.best;
        job->sqd[i] = d2;
      }
    }
    if (active && out) out[src.perm[i]] = sqrt((double)d2);
  }
}

// Residual image (odom.cc:804-827 -> detection.cpp
// projectResiduals :203-252).  Pixel of source point i (sensor frame, the
// scan the residuals belong to): theta = atan2(x, z), phi = atan2(y,
// sqrt(x^2 + z^2)) in double, u = int((theta - tmin) / (tmax - tmin) * W),
// v likewise with phi; points outside [0, W) x [0, H) are skipped.
// (Which atan2/sqrt overload the reference's unqualified calls on float
// members resolve to depends on the headers reaching odom.cc; this takes
// the C double functions.  Only pixel-boundary cases can differ.)  The
// reference fills the image in point order, so the HIGHEST original index
// that lands on a pixel wins: atomicMax of the index, then a gather pass.
__global__ __launch_bounds__(256) void k_resimg_claim(const float4* __restrict__ pts, const int* __restrict__ perm,
                                                      int n, double tmin, double tmax, int W, int H,
                                                      int* __restrict__ winner) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = pts[i];
  // x*x + z*z is float arithmetic in the reference (PointXYZI members);
  // atan2 / sqrt then run on the promoted values
  const float xz2 = p.x * p.x + p.z * p.z;
  const double theta = atan2((double)p.x, (double)p.z);
  const double phi = atan2((double)p.y, sqrt((double)xz2));
  const int u = (int)((theta - tmin) / (tmax - tmin) * W);
  const int v = (int)((phi - tmin) / (tmax - tmin) * H);
  if (u < 0 || u >= W || v < 0 || v >= H) return;
  atomicMax(&winner[(size_t)v * W + u], perm[i]);
}

__global__ __launch_bounds__(256) void k_resimg_fill(const int* __restrict__ winner, int npix,
                                                     const double* __restrict__ residual,
                                                     const float4* __restrict__ pts, const int* __restrict__ inv_perm,
                                                     float* __restrict__ img, float* __restrict__ xyz) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const int o = winner[p];
  float r = 0.f, x = 0.f, y = 0.f, z = 0.f;   // empty pixel: PCL's default point, intensity 0
  if (o >= 0) {
    r = (float)residual[o];
    const float4 q = pts[inv_perm[o]];
    x = q.x; y = q.y; z = q.z;
  }
  img[p] = r;
  if (xyz) {
    xyz[3 * (size_t)p + 0] = x;
    xyz[3 * (size_t)p + 1] = y;
    xyz[3 * (size_t)p + 2] = z;
  }
}

// pcl::transformPointCloud with final_transformation_ (float 4x4)
__global__ __launch_bounds__(256) void k_transform(const float4* __restrict__ pts, int n, const int* __restrict__ perm,
                                                   const float* __restrict__ T16, float* __restrict__ out,
                                                   size_t stride_floats) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 a = pts[i];
  float* o = out + (size_t)perm[i] * stride_floats;
  o[0] = (T16[0] * a.x + T16[1] * a.y) + (T16[2] * a.z + T16[3]);
  o[1] = (T16[4] * a.x + T16[5] * a.y) + (T16[6] * a.z + T16[7]);
  o[2] = (T16[8] * a.x + T16[9] * a.y) + (T16[10] * a.z + T16[11]);
}

// correspondences in original source order (original target indices)
__global__ __launch_bounds__(256) void k_export_corr(const AlignJob* __restrict__ job, int* __restrict__ corr_out,
                                                     float* __restrict__ sqd_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // sorted source index
  if (i >= job->src.n) return;
  const int o = job->src.perm[i];
  const int j = job->corr[i];
  if (corr_out) corr_out[o] = j >= 0 ? job->tgt.perm[j] : -1;
  if (sqd_out) sqd_out[o] = job->sqd[i];
}

}  // namespace ddlo

// ============================================================================
// host launchers
// ============================================================================
namespace ddlo {

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
static inline int group_blocks(int n) {  // 4 waves (256 threads) per block, one 64-query group per wave
  const int groups = cdiv(n, 64);
  return std::max(1, std::min(cdiv(groups, 4), 4096));
}

void launch_pack_bbox(hipStream_t s, const unsigned char* raw, size_t stride, int n, float4* out, float* partial,
                      int* nonfinite, int nblocks) {
  k_pack_bbox<<<nblocks, 256, 0, s>>>(raw, stride, n, out, partial, nonfinite);
}
void launch_bbox_final(hipStream_t s, const float* partial, int nparts, float* quant) {
  k_bbox_final<<<1, 256, 0, s>>>(partial, nparts, quant);
}
void launch_morton(hipStream_t s, const float4* pts, int n, const float* quant, unsigned long long* keys, int* vals) {
  k_morton<<<cdiv(n, 256), 256, 0, s>>>(pts, n, quant, keys, vals);
}
void launch_gather(hipStream_t s, const float4* raw, const int* perm, int n, int npad, float4* sorted, int* inv_perm) {
  k_gather<<<cdiv(npad, 256), 256, 0, s>>>(raw, perm, n, npad, sorted, inv_perm);
}
void launch_key_dir(hipStream_t s, const unsigned long long* keys, int n, int* dir) {
  k_key_dir<<<cdiv((1 << kDirBits) + 1, 256), 256, 0, s>>>(keys, n, dir);
  (void)hipMemsetAsync(dir + (1 << kDirBits) + 1, 0, sizeof(int), s);   // fine-slot counter
  k_key_big<<<(1 << kDirBits) / 256, 256, 0, s>>>(dir);
  const long max_slots = (long)n / (kFineMin + 1) + 1;   // (fine_dir_ints)
  k_key_fine<<<cdiv(max_slots, 4), 256, 0, s>>>(keys, dir);
}
void launch_leaf_soa_boxes(hipStream_t s, const float4* pts, int n, int nleaves, float* soa, float4* lo, float4* hi) {
  k_leaf_soa_boxes<<<cdiv(nleaves, 8), 256, 0, s>>>(pts, n, nleaves, soa, lo, hi);
}
void launch_level_boxes(hipStream_t s, const float4* clo, const float4* chi, int nchild, int nparent, float4* plo,
                        float4* phi) {
  k_level_boxes<<<cdiv(nparent, 4), 256, 0, s>>>(clo, chi, nchild, nparent, plo, phi);
}
static int env_knob(const char* name, int dflt) {   // development knobs (A/B of launch shapes)
  const char* v = dev_getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}
bool launch_covariances(hipStream_t s, const CloudDev& c, int k, int method, double* cov6, const unsigned char* redo,
                        TieList ties) {
  const int nb = group_blocks(c.n);
  static const int two_lanes = env_knob("DDLO_COV_2LANE", 1);   // two lanes per query (A/B)
  if (two_lanes && !redo && (k == 10 || k == 20)) {
    const int nb2 = std::max(1, std::min(cdiv(cdiv(c.n, 32), 4), 8192));
    static const int occ = env_knob("DDLO_COV_OCC", 3);
    // k = 20 at 2 waves / SIMD: 191 VGPRs, no spills (3 waves: 168 VGPRs + 16 spilled; DDLO_COV_OCC20=3)
    static const int occ20 = env_knob("DDLO_COV_OCC20", 2);
    if (k == 10 && occ == 4) k_covariances2<10, true, 4><<<nb2, 256, 0, s>>>(c, k, method, cov6, ties);
    else if (k == 10) k_covariances2<10, true, 3><<<nb2, 256, 0, s>>>(c, k, method, cov6, ties);
    else if (occ20 == 3) k_covariances2<20, true, 3><<<nb2, 256, 0, s>>>(c, k, method, cov6, ties);
    else k_covariances2<20, true, 2><<<nb2, 256, 0, s>>>(c, k, method, cov6, ties);
    return true;
  }
  if (k == 10) k_covariances<10, true><<<nb, 256, 0, s>>>(c, k, method, cov6, redo, ties);
  else if (k == 20) k_covariances<20, true><<<nb, 256, 0, s>>>(c, k, method, cov6, redo, ties);
  else if (k <= 16) k_covariances<16, false><<<nb, 256, 0, s>>>(c, k, method, cov6, redo, ties);
  else if (k <= 32) k_covariances<32, false><<<nb, 256, 0, s>>>(c, k, method, cov6, redo, ties);
  else if (k <= 64) k_covariances<64, false><<<nb, 256, 0, s>>>(c, k, method, cov6, redo, ties);
  else return false;
  return true;
}
bool launch_knn_query(hipStream_t s, const CloudDev& c, const float4* q, int nq, int k, int* out_idx, float* out_d,
                      TieList ties) {
  const int nb = group_blocks(nq);
  if (k == 1) k_knn_query<1, true><<<nb, 256, 0, s>>>(c, q, nq, k, out_idx, out_d, ties);
  else if (k == 10) k_knn_query<10, true><<<nb, 256, 0, s>>>(c, q, nq, k, out_idx, out_d, ties);
  else if (k == 20) k_knn_query<20, true><<<nb, 256, 0, s>>>(c, q, nq, k, out_idx, out_d, ties);
  else if (k <= 16) k_knn_query<16, false><<<nb, 256, 0, s>>>(c, q, nq, k, out_idx, out_d, ties);
  else if (k <= 32) k_knn_query<32, false><<<nb, 256, 0, s>>>(c, q, nq, k, out_idx, out_d, ties);
  else if (k <= 64) k_knn_query<64, false><<<nb, 256, 0, s>>>(c, q, nq, k, out_idx, out_d, ties);
  else return false;
  return true;
}
void launch_cov_import(hipStream_t s, const double* in, int layout, int n, const int* inv_perm, double* cov6) {
  k_cov_import<<<cdiv(n, 256), 256, 0, s>>>(in, layout, n, inv_perm, cov6);
}
void launch_cov_export(hipStream_t s, const double* cov6, int layout, int n, const int* perm, double* out) {
  k_cov_export<<<cdiv(n, 256), 256, 0, s>>>(cov6, layout, n, perm, out);
}
void launch_cov_remap(hipStream_t s, const double* old_cov6, const int* old_inv_perm, const int* new_perm, int n,
                      double* cov6) {
  k_cov_remap<<<cdiv(n, 256), 256, 0, s>>>(old_cov6, old_inv_perm, new_perm, n, cov6);
}
void launch_align_init(hipStream_t s, AlignJob* job, const AlignJob* job_src) {
  k_align_init<<<1, 128, 0, s>>>(job, job_src);
}
size_t collect_lds_bytes(int upper_count) {
  return (size_t)kLinWaves * kTaskLdsBytes + 2 * sizeof(f4v) * (size_t)upper_count;
}
// kTaskRegions-multiple grid of the scan kernel (4 waves per block)
static int scan_blocks(int nsrc) {
  const int groups = (nsrc + kTaskQ - 1) / kTaskQ;
  static const int cap = [] {   // development knob
    const char* v = dev_getenv("DDLO_SCAN_WAVES");
    return v && *v ? std::max(kTaskRegions, std::atoi(v)) : 8192;
  }();
  int waves = std::min(std::max(groups, kTaskRegions), cap);
  waves = (waves + 8 * kTaskRegions - 1) / (8 * kTaskRegions) * (8 * kTaskRegions);
  return waves / kScanWaves;
}
// Bucketed launch geometry: scans of similar size (cfg 5: +-1k points per
// frame) share one captured chunk graph, and a graph never runs with a grid
// or LDS size smaller than the clouds need (all of it is in the graph key).
LinGeom linearize_geometry(int nsrc, int tgt_upper) {
  LinGeom g;
  const int groups = cdiv(std::max(nsrc, 1), kSearchQ);
  const int gcap = cdiv(groups, 1024) * 1024;                    // 16k-point steps
  g.seed_blocks = gcap / kLinWaves;                               // grid-stride kernel: any grid is exact
  g.collect_blocks = (gcap + kHardMax) / kLinWaves;               // one wave per sub-group: >= the groups
  g.scan_blocks = scan_blocks(gcap * kSearchQ);                   // any grid is exact
  g.mom_blocks = moment_blocks(cdiv(std::max(nsrc, 1), 32768) * 32768);   // grid-stride; = the slab rows
  g.lds_boxes = std::min(2048, cdiv(std::max(tgt_upper, 1), 128) * 128);   // >= the target's upper boxes
  g.lookup_blocks = gcap / kLinWaves;                                      // one 16-query sub-group per wave
  return g;
}

void launch_linearize(hipStream_t s, const AlignJob* job, const LinGeom& g, AlignState* publish) {
  static const int fused_lookup = env_knob("DDLO_GRID_FUSED", 1);   // 0: separate lookup kernel (A/B)
  if (g.grid && !g.grid_walk && fused_lookup) {
    // every query is answered by its cell: the lookup runs inside the moment kernel
    if (g.fuse_lm) k_moments<true, true><<<g.mom_blocks, 64 * kMomWaves, 0, s>>>(job, g.state, publish);
    else k_moments<false, true><<<g.mom_blocks, 64 * kMomWaves, 0, s>>>(job, g.state, nullptr);
    return;
  }
  if (g.grid) k_cell_lookup<<<g.lookup_blocks, 256, 0, s>>>(job);
  if (g.grid && !g.grid_walk) {
    // every query is answered by its cell (or provably unmatched): no walk
  } else {
    static const int occ_seed = env_knob("DDLO_OCC_SEED", 4), occ_col = env_knob("DDLO_OCC_COLLECT", 3),
                     occ_scan = env_knob("DDLO_OCC_SCAN", 5);
    static const int fused = env_knob("DDLO_FUSED_SEED", 1);   // 0: separate seed and collect kernels (A/B)
    const size_t lds = collect_lds_bytes(g.lds_boxes);
    // with candidate cells the walk gets the few sub-groups without a list:
    // small grids (the kernels are grid-stride loops), so that the usual
    // empty launches cost little
    const int seed_blocks = g.grid ? std::min(g.seed_blocks, 256) : g.seed_blocks;
    const int scan_blocks = g.grid ? std::min(g.scan_blocks, 8 * kTaskRegions / kScanWaves) : g.scan_blocks;
    if (fused) {
      static const int occ_fused = env_knob("DDLO_OCC_FUSED", 4);
      if (occ_fused == 2) k_nn_seed<2, true><<<seed_blocks, 64 * kLinWaves, lds, s>>>(job);
      else if (occ_fused == 4) k_nn_seed<4, true><<<seed_blocks, 64 * kLinWaves, lds, s>>>(job);
      else k_nn_seed<3, true><<<seed_blocks, 64 * kLinWaves, lds, s>>>(job);
    } else {
      if (occ_seed == 6) k_nn_seed<6, false><<<g.seed_blocks, 64 * kLinWaves, 0, s>>>(job);
      else k_nn_seed<4, false><<<g.seed_blocks, 64 * kLinWaves, 0, s>>>(job);
      if (occ_col == 4) k_nn_collect<4><<<g.collect_blocks, 64 * kLinWaves, lds, s>>>(job);
      else k_nn_collect<3><<<g.collect_blocks, 64 * kLinWaves, lds, s>>>(job);
    }
    if (g.grid && fused) {
      // the walk scanned its (few) sub-groups' tasks inline (AlignJob::task_cap_r = 0)
    } else if (occ_scan == 6) k_nn_scan<6><<<scan_blocks, 64 * kScanWaves, 0, s>>>(job);
    else if (occ_scan == 5) k_nn_scan<5, 6><<<scan_blocks, 64 * kScanWaves, 0, s>>>(job);   // 6-task batches: 7.5 KB LDS per wave
    else k_nn_scan<4><<<scan_blocks, 64 * kScanWaves, 0, s>>>(job);
  }
  if (g.fuse_lm) k_moments<true><<<g.mom_blocks, 64 * kMomWaves, 0, s>>>(job, g.state, publish);
  else k_moments<false><<<g.mom_blocks, 64 * kMomWaves, 0, s>>>(job, g.state, nullptr);
}
int search_queries_per_wave() { return kSearchQ; }
int task_cap_per_region(int nsrc) {
  const long groups = (nsrc + kTaskQ - 1) / kTaskQ;
  return (int)std::max<long>(1024, (groups * kTasksPerGroup + kTaskRegions - 1) / kTaskRegions);
}
int moment_blocks(int nsrc) {
  const int groups = (nsrc + 63) / 64;
  return std::max(1, std::min((groups + kMomWaves - 1) / kMomWaves, kMomBlocksMax));
}
void launch_lm_step(hipStream_t s, const AlignJob* job, AlignState* st, const double* slab, int nblocks,
                    const double* premom, AlignState* publish) {
  k_lm_step<<<1, kLmThreads, 0, s>>>(job, st, slab, nblocks, premom, publish);
}
void launch_mom_reduce(hipStream_t s, const AlignJob* job) { k_mom_reduce<<<1, kLmThreads, 0, s>>>(job); }
void launch_residual_image(hipStream_t s, const float4* pts, const int* perm, const int* inv_perm, int n,
                           const double* residual, double tmin, double tmax, int W, int H, int* winner, float* img,
                           float* xyz) {
  k_resimg_claim<<<cdiv(n, 256), 256, 0, s>>>(pts, perm, n, tmin, tmax, W, H, winner);
  k_resimg_fill<<<cdiv((long)W * H, 256), 256, 0, s>>>(winner, W * H, residual, pts, inv_perm, img, xyz);
}
void launch_residuals(hipStream_t s, const AlignJob* job, int nsrc, double* out) {
  k_residuals<<<group_blocks(nsrc), 256, 0, s>>>(job, out);
}
void launch_transform(hipStream_t s, const float4* pts, int n, const int* perm, const float* T16, float* out,
                      size_t stride_floats) {
  k_transform<<<cdiv(n, 256), 256, 0, s>>>(pts, n, perm, T16, out, stride_floats);
}
void launch_export_corr(hipStream_t s, const AlignJob* job, int nsrc, int* corr, float* sqd) {
  k_export_corr<<<cdiv(nsrc, 256), 256, 0, s>>>(job, corr, sqd);
}

}  // namespace ddlo

#ifdef DDLO_COV_PROF
// developer build: k_covariances2's per-group records of the last launch, [group][4]
extern "C" int ddlo_dev_cov_prof2(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(ddlo::g_cov_prof2), sizeof(ddlo::g_cov_prof2));
}
extern "C" int ddlo_dev_cov_prof(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(ddlo::g_cov_prof), sizeof(ddlo::g_cov_prof));
}
#endif
#ifdef DDLO_MOM_PROF
// developer build: the fused moment kernel's wave stamps of the last align, [iteration][wave][6]
extern "C" int ddlo_dev_mom_prof(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(ddlo::g_mom_prof), sizeof(ddlo::g_mom_prof));
}
#endif
