// preprocess.hip — device-side scan preprocessing and keyframe plumbing of
// the odometry driver (odom.hip), SURVEY.md §8(f) ranks 1 and 3:
//
//   k_crop_keep / compaction   pcl::CropBox with setNegative(true)
//                              (odom.cc:114-119,460-465)
//   voxel_grid()               pcl::VoxelGrid<PointXYZI>::applyFilter
//                              (odom.cc:121-122,469-475,1133-1137)
//   k_ranges + median          OdomNode::computeSpaciousness (odom.cc:981-1001)
//   k_transform4               pcl::transformPointCloud of a device cloud to
//                              the world frame, original order (odom.cc:492,
//                              transformScans :941-947)
//   k_gather_cov6              keyframe covariances back to original order
//
// Compiled with -ffp-contract=off: the voxel index, the range and the
// transform follow the reference's float / double operation order.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>

#include "gicp_types.hpp"
#include "launch.hpp"

namespace ddlo {

namespace {
inline int cdiv_l(long a, long b) { return (int)((a + b - 1) / b); }
}

// ---- upload: strided host layout (e.g. 32-B PointXYZI) -> packed float4 ----
__global__ __launch_bounds__(256) void k_pack4(const unsigned char* __restrict__ raw, size_t stride, int n,
                                               float4* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* p = reinterpret_cast<const float*>(raw + (size_t)i * stride);
  out[i] = make_float4(p[0], p[1], p[2], 0.f);
}

// ---- crop box (negative: keep the points strictly outside [-s, s]^3) ----
__global__ __launch_bounds__(256) void k_crop_flags(const float4* __restrict__ in, int n, float s, int* __restrict__ keep) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = in[i];
  // CropBox::applyFilter: non-finite points are dropped; a point with any
  // coordinate below min or above max is outside the box (kept when negative)
  const bool finite = isfinite(p.x) && isfinite(p.y) && isfinite(p.z);
  const bool outside = p.x < -s || p.y < -s || p.z < -s || p.x > s || p.y > s || p.z > s;
  keep[i] = finite && outside ? 1 : 0;
}

__global__ __launch_bounds__(256) void k_compact(const float4* __restrict__ in, int n, const int* __restrict__ keep,
                                                 const int* __restrict__ pos, float4* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !keep[i]) return;
  out[pos[i]] = in[i];
}

// ---- voxel grid --------------------------------------------------------------
// The points a voxel pass sees: finite, and — when the crop box is folded
// into the pass (crop > 0) — outside [-crop, crop]^3 (k_crop_flags' rule).
__device__ __forceinline__ bool voxel_input(float4 p, float crop) {
  if (!(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) return false;
  return !(crop > 0.f) || (p.x < -crop || p.y < -crop || p.z < -crop || p.x > crop || p.y > crop || p.z > crop);
}

// bbox of those points: per-block partial min/max, then one block
__global__ __launch_bounds__(256) void k_minmax_partial(const float4* __restrict__ in, int n, float crop,
                                                        float* __restrict__ part) {
  float v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float4 p = in[i];
    if (!voxel_input(p, crop)) continue;
    v[0] = fminf(v[0], p.x); v[1] = fminf(v[1], p.y); v[2] = fminf(v[2], p.z);
    v[3] = fmaxf(v[3], p.x); v[4] = fmaxf(v[4], p.y); v[5] = fmaxf(v[5], p.z);
  }
  __shared__ float red[6][256];
  for (int a = 0; a < 6; ++a) red[a][threadIdx.x] = v[a];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int a = 0; a < 6; ++a)
        red[a][threadIdx.x] = a < 3 ? fminf(red[a][threadIdx.x], red[a][threadIdx.x + w])
                                    : fmaxf(red[a][threadIdx.x], red[a][threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = red[threadIdx.x][0];
}

// Grid geometry of VoxelGrid::applyFilter: min_b = floor(min_p * inv),
// max_b = floor(max_p * inv), div_b = max_b - min_b + 1, divb_mul =
// (1, div_b.x, div_b.x * div_b.y); geo[0..2] = min_b, geo[3..4] = divb_mul
// y/z, geo[5] = 1 if the grid overflows an int index (the reference then
// returns the input unchanged), geo[6] = 1 if there is no finite point.
// From the 64 partial boxes (min / max are exact in any order); every block
// of the key kernel derives it itself (no single-thread geometry launch).
constexpr int kVoxParts = 64;
__device__ void voxel_geometry(const float* __restrict__ part, float inv_x, float inv_y, float inv_z, int* geo) {
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int b = 0; b < kVoxParts; ++b)
    for (int a = 0; a < 3; ++a) {
      mn[a] = fminf(mn[a], part[b * 6 + a]);
      mx[a] = fmaxf(mx[a], part[b * 6 + 3 + a]);
    }
  geo[6] = !(mn[0] <= mx[0]);
  if (geo[6]) return;
  const float inv[3] = {inv_x, inv_y, inv_z};
  long long d[3];
  for (int a = 0; a < 3; ++a) d[a] = (long long)((mx[a] - mn[a]) * inv[a]) + 1;
  geo[5] = (d[0] * d[1] * d[2]) > (long long)INT_MAX;
  int minb[3], divb[3];
  for (int a = 0; a < 3; ++a) {
    minb[a] = (int)floorf(mn[a] * inv[a]);
    const int maxb = (int)floorf(mx[a] * inv[a]);
    divb[a] = maxb - minb[a] + 1;
  }
  geo[0] = minb[0]; geo[1] = minb[1]; geo[2] = minb[2];
  geo[3] = divb[0];
  geo[4] = divb[0] * divb[1];
}

// Voxel index of every point (non-finite or cropped points get UINT_MAX and
// sort last, they are dropped by the caller's count).
__global__ __launch_bounds__(256) void k_voxel_keys(const float4* __restrict__ in, int n, float inv_x, float inv_y,
                                                    float inv_z, float crop, const float* __restrict__ part,
                                                    int* __restrict__ small, unsigned* __restrict__ key,
                                                    int* __restrict__ idx) {
  __shared__ float sp[kVoxParts * 6];
  __shared__ int geo[7];
  for (int e = threadIdx.x; e < kVoxParts * 6; e += blockDim.x) sp[e] = part[e];
  __syncthreads();
  if (threadIdx.x == 0) {
    geo[5] = 0;
    voxel_geometry(sp, inv_x, inv_y, inv_z, geo);
    if (blockIdx.x == 0) {   // the flags the host reads
      small[6] = geo[6];
      small[5] = geo[6] ? 0 : geo[5];
    }
  }
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = in[i];
  unsigned k = 0xffffffffu;
  if (voxel_input(p, crop)) {   // (no such point when geo[6]: the geometry is not read)
    const int i0 = (int)(floorf(p.x * inv_x) - (float)geo[0]);
    const int i1 = (int)(floorf(p.y * inv_y) - (float)geo[1]);
    const int i2 = (int)(floorf(p.z * inv_z) - (float)geo[2]);
    k = (unsigned)(i0 + i1 * geo[3] + i2 * geo[4]);
  }
  key[i] = k;
  idx[i] = i;
}

// Whether any point left the voxel pass (non-finite or cropped): their keys
// (UINT_MAX) sort last and form the last run.  small[9] = n - 1 if so, else
// n.  (Counting the valid points with atomics on one word serialised the key
// kernel: ~25 us per scan per point, still ~23 us with one add per wavefront.)
__global__ void k_voxel_tail(const unsigned* __restrict__ uniq, int n, int* __restrict__ small) {
  if (threadIdx.x == 0) {
    const int nr = small[8];
    small[9] = (nr > 0 && uniq[nr - 1] == 0xffffffffu) ? n - 1 : n;
  }
}

// Centroid of each run of equal voxel index: float sums in input order
// (the radix sort is stable), divided by the count (CentroidPoint /
// AccumulatorXYZ).
__global__ __launch_bounds__(256) void k_voxel_centroids(const float4* __restrict__ in, const int* __restrict__ order,
                                                         const int* __restrict__ offsets, const int* __restrict__ counts,
                                                         int nruns, float4* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nruns) return;
  const int o = offsets[r], c = counts[r];
  float sx = 0.f, sy = 0.f, sz = 0.f;
  for (int k = 0; k < c; ++k) {
    const float4 p = in[order[o + k]];
    sx += p.x;
    sy += p.y;
    sz += p.z;
  }
  const float fc = (float)c;
  out[r] = make_float4(sx / fc, sy / fc, sz / fc, 0.f);
}

// ---- spaciousness: ranges ---------------------------------------------------
// d = sqrt(pow(x, 2) + pow(y, 2) + pow(z, 2)) with the float coordinates
// promoted to double (std::pow(float, int) returns double), stored as float
__global__ __launch_bounds__(256) void k_ranges(const float4* __restrict__ in, int n, float* __restrict__ d) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = in[i];
  const double x = p.x, y = p.y, z = p.z;
  d[i] = (float)sqrt((x * x + y * y) + z * z);
}

// ---- keyframes ----------------------------------------------------------------
// world-frame copy of a device cloud in ORIGINAL order: out[perm[i]] = T * p
// in the order of PCL's transformPointCloud, (c0 x + c1 y) + (c2 z + c3)
struct T34 {
  float m[12];
};
__global__ __launch_bounds__(256) void k_transform4(const float4* __restrict__ pts, const int* __restrict__ perm, int n,
                                                    T34 T, float4* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = pts[i];
  const float* m = T.m;
  out[perm[i]] = make_float4((m[0] * p.x + m[1] * p.y) + (m[2] * p.z + m[3]),
                             (m[4] * p.x + m[5] * p.y) + (m[6] * p.z + m[7]),
                             (m[8] * p.x + m[9] * p.y) + (m[10] * p.z + m[11]), 0.f);
}

// covariances of a cloud (sym6 per SORTED point) back to original order
__global__ __launch_bounds__(256) void k_gather_cov6(const double* __restrict__ cov_sorted, const int* __restrict__ perm,
                                                     int n, double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int o = perm[i];
  for (int e = 0; e < 6; ++e) out[6 * (size_t)o + e] = cov_sorted[6 * (size_t)i + e];
}

// ============================================================================
// host launchers
// ============================================================================
int crop_box(hipStream_t s, const float4* in, int n, float size, float4* out, int* keep, int* pos, void* tmp,
             size_t tmp_bytes, int* count_host, int* pin) {
  if (n <= 0) {
    *count_host = 0;
    return 0;
  }
  k_crop_flags<<<cdiv_l(n, 256), 256, 0, s>>>(in, n, size, keep);
  size_t need = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, need, keep, pos, n, s);
  if (need > tmp_bytes) return -1;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, need, keep, pos, n, s);
  k_compact<<<cdiv_l(n, 256), 256, 0, s>>>(in, n, keep, pos, out);
  (void)hipMemcpyAsync(pin, pos + n - 1, sizeof(int), hipMemcpyDeviceToHost, s);
  (void)hipMemcpyAsync(pin + 1, keep + n - 1, sizeof(int), hipMemcpyDeviceToHost, s);
  (void)hipStreamSynchronize(s);
  *count_host = pin[0] + pin[1];
  return 0;
}
size_t crop_box_tmp_bytes(int n) {
  size_t need = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, need, (int*)nullptr, (int*)nullptr, n, (hipStream_t)0);
  return need;
}

size_t voxel_tmp_bytes(int n) {
  size_t a = 0, b = 0, c = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (unsigned*)nullptr, (unsigned*)nullptr, (int*)nullptr,
                                           (int*)nullptr, n, 0, 32, (hipStream_t)0);
  (void)hipcub::DeviceRunLengthEncode::Encode(nullptr, b, (unsigned*)nullptr, (unsigned*)nullptr, (int*)nullptr,
                                              (int*)nullptr, n, (hipStream_t)0);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (int*)nullptr, (int*)nullptr, n, (hipStream_t)0);
  return std::max(a, std::max(b, c));
}

// VoxelGrid of n device points.  Scratch layout (ints unless noted): keys[n],
// keys_sorted[n], idx[n], order[n], uniq[n], counts[n], offsets[n], small[16],
// part[6 * 64] floats.  Returns the output count in *count_host (-1 if the
// grid overflows: the caller copies the input, as the reference does).
// pin: 16 ints of pinned host memory (the read-back of small).  small needs
// no clearing: every slot the host reads ([5], [6], [8], [9]) is written.
int voxel_grid(hipStream_t s, const float4* in, int n, float leaf, float4* out, int* scratch, void* tmp, size_t tmp_bytes,
               int* count_host, float crop, int* pin) {
  *count_host = 0;
  if (n <= 0) return 0;
  unsigned* keys = reinterpret_cast<unsigned*>(scratch);
  unsigned* keys_sorted = keys + n;
  int* idx = reinterpret_cast<int*>(keys_sorted + n);
  int* order = idx + n;
  unsigned* uniq = reinterpret_cast<unsigned*>(order + n);
  int* counts = reinterpret_cast<int*>(uniq + n);
  int* offsets = counts + n;
  int* small = offsets + n;   // [0..6] geometry, [8] nruns, [9] < n: some point left the pass
  float* part = reinterpret_cast<float*>(small + 16);
  // inverse_leaf_size_ = 1 / leaf_size_ (float)
  const float inv = 1.0f / leaf;
  k_minmax_partial<<<kVoxParts, 256, 0, s>>>(in, n, crop, part);
  k_voxel_keys<<<cdiv_l(n, 256), 256, 0, s>>>(in, n, inv, inv, inv, crop, part, small, keys, idx);
  size_t need = voxel_tmp_bytes(n);
  if (need > tmp_bytes) return -2;
  size_t t = tmp_bytes;
  (void)hipcub::DeviceRadixSort::SortPairs(tmp, t, keys, keys_sorted, idx, order, n, 0, 32, s);
  t = tmp_bytes;
  (void)hipcub::DeviceRunLengthEncode::Encode(tmp, t, keys_sorted, uniq, counts, small + 8, n, s);
  k_voxel_tail<<<1, 64, 0, s>>>(uniq, n, small);
  t = tmp_bytes;
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, t, counts, offsets, n, s);
  int* const h = pin;
  (void)hipMemcpyAsync(h, small, 16 * sizeof(int), hipMemcpyDeviceToHost, s);
  (void)hipStreamSynchronize(s);
  if (h[6]) return 0;            // no (finite, uncropped) point
  if (h[5]) {                    // grid overflow: the reference leaves the cloud as it is
    *count_host = -1;
    return 0;
  }
  // runs of the voxel-pass points only (the others' keys = UINT_MAX sort last
  // and form the last run; a real voxel index never reaches UINT_MAX here)
  int nruns = h[8];
  if (h[9] < n) nruns -= 1;
  k_voxel_centroids<<<cdiv_l(std::max(nruns, 1), 256), 256, 0, s>>>(in, order, offsets, counts, nruns, out);
  *count_host = nruns;
  return 0;
}

// median range: the element n/2 of the sorted ranges (computeSpaciousness
// sorts them, odom.cc:981-1001), found by a three-digit radix select on the
// float bit patterns (non-negative floats order like their bits): 11 + 11 +
// 10 bits, one histogram pass per digit over the ranges; each pass's blocks
// first locate the digits chosen so far in the earlier histograms.  Copied
// to `out` (pinned host memory) in stream order; the caller reads it after
// waiting on the stream.  (A full radix sort of the ranges took ~30 us.)
namespace {
constexpr int kMedBins = 2048;
constexpr int kMedThreads = 256;

// block-wide: the bin of `hist` (nb bins) holding rank `rank` (0-based) and
// the rank inside it; every thread returns both.  Each thread sums `per`
// consecutive bins, a block scan of those sums (wavefront shuffles + the four
// wavefront totals) finds the one thread whose range holds the rank, and that
// thread walks its own bins (a serial walk of the 256 sums by one thread cost
// ~7 us per call in the odometry chain's trace).
__device__ void med_find(const unsigned* __restrict__ hist, int nb, unsigned rank, unsigned* sh, unsigned& bin,
                         unsigned& rin) {
  const int t = threadIdx.x;
  const int per = nb / kMedThreads;   // 8 or 4
  unsigned h[8];
  unsigned local = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    h[k] = k < per ? hist[t * per + k] : 0u;
    local += h[k];
  }
  const int lane = t & 63, w = t >> 6;
  unsigned incl = local;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned v = __shfl_up(incl, d);
    if (lane >= d) incl += v;
  }
  if (lane == 63) sh[w] = incl;
  __syncthreads();
  for (int k = 0; k < w; ++k) incl += sh[k];
  const unsigned excl = incl - local;
  if (excl <= rank && rank < incl) {   // exactly one thread (rank < the total)
    unsigned a = excl;
    int b = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (b == k && k < per - 1 && a + h[k] <= rank) {
        a += h[k];
        b = k + 1;
      }
    }
    sh[kMedThreads] = (unsigned)(t * per + b);
    sh[kMedThreads + 1] = rank - a;
  }
  __syncthreads();
  bin = sh[kMedThreads];
  rin = sh[kMedThreads + 1];
  __syncthreads();
}

template <int PASS>
__global__ __launch_bounds__(kMedThreads) void k_med_hist(const float4* __restrict__ in, int n, unsigned* __restrict__ d,
                                                          unsigned* __restrict__ hist) {
  __shared__ unsigned lh[kMedBins];
  __shared__ unsigned sh[kMedThreads + 2];
  for (int b = threadIdx.x; b < kMedBins; b += kMedThreads) lh[b] = 0;
  unsigned prefix = 0;
  if constexpr (PASS >= 1) {
    unsigned b0, r0;
    med_find(hist, kMedBins, (unsigned)(n / 2), sh, b0, r0);
    prefix = b0;
    if constexpr (PASS == 2) {
      unsigned b1, r1;
      med_find(hist + kMedBins, kMedBins, r0, sh, b1, r1);
      prefix = (b0 << 11) | b1;
    }
  }
  __syncthreads();
  constexpr int shift = PASS == 0 ? 21 : (PASS == 1 ? 10 : 0);
  constexpr unsigned dmask = PASS == 2 ? 1023u : 2047u;
  for (int i = blockIdx.x * kMedThreads + threadIdx.x; i < n; i += gridDim.x * kMedThreads) {
    unsigned v;
    if constexpr (PASS == 0) {
      const float4 p = in[i];
      const double x = p.x, y = p.y, z = p.z;
      v = __float_as_uint((float)sqrt((x * x + y * y) + z * z));   // k_ranges' operation order
      d[i] = v;
    } else {
      v = d[i];
    }
    const bool take = PASS == 0 ? true : (PASS == 1 ? (v >> 21) == prefix : (v >> 10) == prefix);
    if (take) atomicAdd(&lh[(v >> shift) & dmask], 1u);
  }
  __syncthreads();
  unsigned* const out = hist + PASS * kMedBins;
  for (int b = threadIdx.x; b < kMedBins; b += kMedThreads)
    if (lh[b]) atomicAdd(out + b, lh[b]);
}

__global__ __launch_bounds__(kMedThreads) void k_med_final(const unsigned* __restrict__ hist, int n,
                                                           float* __restrict__ result) {
  __shared__ unsigned sh[kMedThreads + 2];
  unsigned b0, r0, b1, r1, b2, r2;
  med_find(hist, kMedBins, (unsigned)(n / 2), sh, b0, r0);
  med_find(hist + kMedBins, kMedBins, r0, sh, b1, r1);
  med_find(hist + 2 * kMedBins, 1024, r1, sh, b2, r2);
  if (threadIdx.x == 0) result[0] = __uint_as_float((b0 << 21) | (b1 << 10) | b2);
}
}  // namespace

void median_range_async(hipStream_t s, const float4* in, int n, float* d, float* result, void* tmp, size_t tmp_bytes,
                        float* out) {
  (void)tmp_bytes;   // >= median_tmp_bytes(n)
  unsigned* const hist = static_cast<unsigned*>(tmp);
  (void)hipMemsetAsync(hist, 0, sizeof(unsigned) * 3 * kMedBins, s);
  const int blocks = std::max(1, std::min(cdiv_l(n, kMedThreads * 8), 256));
  unsigned* const du = reinterpret_cast<unsigned*>(d);
  k_med_hist<0><<<blocks, kMedThreads, 0, s>>>(in, n, du, hist);
  k_med_hist<1><<<blocks, kMedThreads, 0, s>>>(in, n, du, hist);
  k_med_hist<2><<<blocks, kMedThreads, 0, s>>>(in, n, du, hist);
  k_med_final<<<1, kMedThreads, 0, s>>>(hist, n, result);
  (void)hipMemcpyAsync(out, result, sizeof(float), hipMemcpyDeviceToHost, s);
}
size_t median_tmp_bytes(int n) {
  (void)n;
  return sizeof(unsigned) * 3 * kMedBins;
}

void launch_pack4(hipStream_t s, const unsigned char* raw, size_t stride, int n, float4* out) {
  k_pack4<<<cdiv_l(n, 256), 256, 0, s>>>(raw, stride, n, out);
}
void launch_transform4(hipStream_t s, const float4* pts, const int* perm, int n, const float* T12, float4* out) {
  T34 T;
  for (int e = 0; e < 12; ++e) T.m[e] = T12[e];
  k_transform4<<<cdiv_l(n, 256), 256, 0, s>>>(pts, perm, n, T, out);
}
void launch_gather_cov6(hipStream_t s, const double* cov_sorted, const int* perm, int n, double* out) {
  k_gather_cov6<<<cdiv_l(n, 256), 256, 0, s>>>(cov_sorted, perm, n, out);
}

}  // namespace ddlo
