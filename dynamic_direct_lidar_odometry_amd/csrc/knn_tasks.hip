// knn_tasks.hip — task-based exact kNN-k of a cloud's own points, the
// neighbour search of calculate_covariances (reference
// include/nano_gicp/impl/nano_gicp_impl.hpp:373-441; nanoflann
// KNNResultSet semantics, nanoflann_impl.hpp:161-242, with the sorted
// position breaking exact distance ties).
//
// The lane-per-query traversal (kernels.hip k_covariances) lasts as long as
// its slowest wavefront: a sparse far-range point whose k-th neighbour is
// metres away walks and scans hundreds of leaves alone.  Here that work is
// spread over the chip as tasks, like the correspondence search
// (nn_tasks.hpp):
//
//   k_knn_seed     lane per point: the k-th smallest distance among the 32
//                  Morton-adjacent points — k real points, so an exact upper
//                  bound on the k-th neighbour's distance: the ball.
//   k_knn_collect  wave per 16-point sub-group: walk + exact (leaf, point)
//                  box tests against the balls -> tasks (leaf, sub-group,
//                  mask) — the TaskCollector of the correspondence search.
//   k_knn_scan     tasks from the list: every point of the leaf inside a
//                  masked query's ball is appended to that query's candidate
//                  list (staged per run in LDS, one atomicAdd per query and
//                  run).
//   k_knn_select   lane per point: the k smallest (distance, position) keys
//                  of its candidates, then mean / covariance / regularisation
//                  in neighbour order (cov_math.hpp).
//
// Every point within the ball is a candidate and the ball contains the k
// nearest, so the selection is exact.  The collect also shrinks each ball to
// the farthest corner of the nearest full leaf (32 >= k real points inside).
// A point with more candidates than slots goes through collect / scan /
// select a second time with the k-th of its stored candidates as the ball;
// a sub-group whose tasks do not fit the list, or a point that overflows
// again, is recomputed by the lane-per-query kernel (k_covariances with its
// `redo` filter).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gicp_types.hpp"
#include "search.hpp"
#include "nn_tasks.hpp"
#include "cov_math.hpp"
#include "launch.hpp"

namespace ddlo {

constexpr int kKnnWaves = 4;        // waves per block (collect / scan)
constexpr int kKnnRunCap = 64;      // LDS candidate slots per query and run (scan)

template <int KCAP>
__global__ __launch_bounds__(256) void k_knn_seed(KnnJob j) {
  const CloudDev& c = j.c;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < kTaskRegions) j.task_ctr[threadIdx.x * kCtrStride] = 0u;
  if (blockIdx.x == 0 && threadIdx.x == 0) *j.n2 = 0u;
  if (i >= c.n) return;
  if ((i & 63) == 0) j.redo[i >> 6] = 0;
  j.cnt[i] = 0u;
  j.again[i] = 0;
  const float4 q = ldg4(c.pts, i);
  // 32 Morton-adjacent real points (the point itself included)
  const int w = min(32, c.n);
  const int w0 = min(max(i - 16, 0), c.n - w);
  float kd[KCAP];
#pragma unroll
  for (int s = 0; s < KCAP; ++s) kd[s] = INFINITY;
  for (int h = 0; h < w; ++h) {
    const float4 p = ldg4(c.pts, w0 + h);
    float d = dist2(q.x, q.y, q.z, p.x, p.y, p.z);
#pragma unroll
    for (int s = 0; s < KCAP; ++s) {   // ascending insertion
      const float lo = fminf(d, kd[s]);
      d = fmaxf(d, kd[s]);
      kd[s] = lo;
    }
  }
  float b = kd[0];
#pragma unroll
  for (int s = 0; s < KCAP; ++s)
    if (s == j.k - 1) b = kd[s];
  j.qstate[i] = make_float4(q.x, q.y, q.z, b);
}

__global__ __launch_bounds__(64 * kKnnWaves) void k_knn_collect(KnnJob j) {
  constexpr int Q = kTaskQ;
  const CloudDev& c = j.c;
  const int lane = lane_id();
  const int qi = lane % Q;
  const int wib = threadIdx.x >> 6;
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  TaskLds* TL = reinterpret_cast<TaskLds*>(dsm) + wib;
  f4v* upper = reinterpret_cast<f4v*>(dsm + kKnnWaves * kTaskLdsBytes);
  TaskList tl;
  tl.tasks = j.tasks;
  tl.ctr = j.task_ctr;
  tl.cap_r = j.task_cap_r;
  const int ngroups = (c.n + Q - 1) / Q;
  const int g = (int)blockIdx.x * kKnnWaves + wib;
  if (j.round == 2) {
    // only the points flagged by the first round's selection: every wave
    // reads the block's 64 flags itself (block-uniform exit, no barrier)
    const int p = (int)blockIdx.x * kKnnWaves * Q + lane;
    if (!__any(p < c.n && j.again[p])) return;
  }
  fill_upper(c, upper);
  __syncthreads();
  if (g >= ngroups) return;
  const int i = g * Q + qi;
  const bool inrange = i < c.n && (j.round == 1 || j.again[min(i, c.n - 1)]);
  const int ic = inrange ? i : c.n - 1;
  const float4 q = ldg4(j.qstate, ic);
  TaskCollector col;
  col.L = TL;
  col.U = upper;
  col.nup = upper_count(c);
  col.qx = q.x;
  col.qy = q.y;
  col.qz = q.z;
  col.active = inrange;
  col.bk = dkey(q.w, -1);
  col.wr = q.w;
  col.sg = g;
  col.knn = true;
  col.nfull = c.n / kLeafSize;
  col.run(c, tl, gp(c.keys)[ic], j.split_extent);
  if (col.ovf && lane == 0) j.redo[(g * Q) >> 6] = 1;
  // the tightened ball (per query: lanes qi, qi + 16, qi + 32, qi + 48)
  float t = fminf(col.tight, __shfl_xor(col.tight, 16));
  t = fminf(t, __shfl_xor(t, 32));
  if (inrange && lane < Q && t < q.w) j.qstate[i].w = t;
}

constexpr int kKnnScanBatch = 8;
constexpr int kKnnTaskBytes = 3 * kLeafSize * 4 + kTaskQ * 16;   // 384 B points + 256 B query balls

__global__ __launch_bounds__(64 * kKnnWaves) void k_knn_scan(KnnJob j) {
  const CloudDev& c = j.c;
  const int lane = lane_id();
  const int qi = lane & 15, s = lane >> 4;
  constexpr int kBatchBytes = kKnnScanBatch * kKnnTaskBytes;
  __shared__ __attribute__((aligned(16))) unsigned char lds_all[kKnnWaves][2][kBatchBytes];
  __shared__ unsigned long long run_keys[kKnnWaves][kTaskQ][kKnnRunCap];
  unsigned char* const L0 = lds_all[threadIdx.x >> 6][0];
  unsigned char* const L1 = lds_all[threadIdx.x >> 6][1];
  unsigned long long (*RK)[kKnnRunCap] = run_keys[threadIdx.x >> 6];
  const int nwaves = (int)((gridDim.x * blockDim.x) >> 6);
  const int wpr = nwaves / kTaskRegions;
  // (region, chunk) of this wave, XCD-aware as in k_nn_scan (speed only)
  int r, ch;
  if (wpr % 8 == 0) {
    const int x = blockIdx.x % 8, u = (int)(blockIdx.x / 8) * kKnnWaves + (int)(threadIdx.x >> 6);
    r = u % kTaskRegions;
    ch = x * (wpr / 8) + u / kTaskRegions;
  } else {
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    r = wave % kTaskRegions;
    ch = wave / kTaskRegions;
  }
  const int n = min((int)__builtin_amdgcn_readfirstlane(j.task_ctr[r * kCtrStride]), j.task_cap_r);
  const int chunk = (n + wpr - 1) / wpr;
  const int lo = ch * chunk, hi = min(n, lo + chunk);
  const unsigned long long* rt = j.tasks + (size_t)r * j.task_cap_r;
  int run_sg = -1;
  int run_cnt = 0;   // candidates of query qi staged in RK[qi] (same value in its 4 lanes)
  // a run's staged candidates -> the queries' global lists (one atomicAdd per query)
  auto flush_run = [&]() {
    if (run_sg < 0) return;
    const int qg = run_sg * kTaskQ + qi;
    int base = 0;
    if (s == 0 && run_cnt > 0) base = (int)atomicAdd(j.cnt + qg, (unsigned)run_cnt);
    base = __shfl(base, qi);   // lane qi (slice 0) holds the query's base
    // first round: the point's own list; second round: its compact list
    // first round: slot-major lists (cand[slot * n + point]: the selection
    // reads them coalesced); second round: the point's compact list
    unsigned long long* list = j.cand + qg;
    size_t stride = (size_t)j.c.n;
    int cap = j.cap;
    if (j.round == 2 && run_cnt > 0) {
      list = j.cand2 + (size_t)j.slot2[qg] * j.cap2;
      stride = 1;
      cap = j.cap2;
    }
    for (int e = s; e < run_cnt; e += 4) {
      const int slot = base + e;
      if (slot < cap) list[(size_t)slot * stride] = RK[qi][e];
    }
    run_cnt = 0;
  };
  for (int wbase = lo; wbase < hi; wbase += 64) {
    const int wcnt = min(64, hi - wbase);
    const unsigned long long tl = lane < wcnt ? rt[wbase + lane] : 0ull;
    auto issue = [&](int b0, unsigned char* buf) {
#pragma unroll
      for (int u = 0; u < kBatchBytes / 1024; ++u) {
        const int o = u * 1024 + lane * 16;
        const int kk = min(b0 + o / kKnnTaskBytes, wcnt - 1), w = o % kKnnTaskBytes;
        const unsigned long long tk = __shfl(tl, kk);
        const char* src = w < 3 * kLeafSize * 4
                              ? (const char*)(c.soa + (size_t)(tk >> 40) * (3 * kLeafSize)) + w
                              : (const char*)(j.qstate + (size_t)((tk >> 16) & 0xffffffull) * kTaskQ) + (w - 3 * kLeafSize * 4);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(buf + u * 1024), 16, 0, 0);
      }
    };
    issue(0, L0);
    for (int b0 = 0; b0 < wcnt; b0 += kKnnScanBatch) {
      unsigned char* const cur = ((b0 / kKnnScanBatch) & 1) ? L1 : L0;
      if (b0 + kKnnScanBatch < wcnt) {
        issue(b0 + kKnnScanBatch, ((b0 / kKnnScanBatch) & 1) ? L0 : L1);
        __builtin_amdgcn_s_waitcnt(0x0F75);  // vmcnt(5): the current batch landed
      } else {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      }
      __builtin_amdgcn_wave_barrier();
      const int nb = min(kKnnScanBatch, wcnt - b0);
      for (int kt = 0; kt < nb; ++kt) {
        const unsigned lo32 = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)tl, b0 + kt);
        const unsigned hi32 = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(tl >> 32), b0 + kt);
        const unsigned long long t = ((unsigned long long)hi32 << 32) | lo32;
        const int sg = (int)((t >> 16) & 0xffffffull);
        // a new sub-group's run, or no room for another leaf (<= 32 per query)
        if (sg != run_sg || __any(run_cnt > kKnnRunCap - kLeafSize)) {
          __builtin_amdgcn_wave_barrier();
          flush_run();
          __builtin_amdgcn_wave_barrier();
          run_sg = sg;
        }
        const unsigned char* T = cur + kt * kKnnTaskBytes;
        const f4v x0 = *(const f4v*)(T + s * 32), x1 = *(const f4v*)(T + s * 32 + 16);
        const f4v y0 = *(const f4v*)(T + 128 + s * 32), y1 = *(const f4v*)(T + 128 + s * 32 + 16);
        const f4v z0 = *(const f4v*)(T + 256 + s * 32), z1 = *(const f4v*)(T + 256 + s * 32 + 16);
        const f4v q = *(const f4v*)(T + 384 + qi * 16);
        const float X[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const float Y[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
        const float Z[8] = {z0.x, z0.y, z0.z, z0.w, z1.x, z1.y, z1.z, z1.w};
        const bool on = ((t >> qi) & 1ull) != 0ull;
        const int pos0 = (int)(t >> 40) * kLeafSize + s * 8;
        unsigned m8 = 0u;
        float dd[8];
#pragma unroll
        for (int h = 0; h < 8; ++h) {
          dd[h] = dist2(q.x, q.y, q.z, X[h], Y[h], Z[h]);
          if (on && dd[h] <= q.w) m8 |= 1u << h;
        }
        // slot of this lane's first candidate: run_cnt + candidates of the
        // query's lower slices (lanes qi, qi + 16, qi + 32, qi + 48)
        const int c8 = __popc(m8);
        const int c_s1 = __shfl(c8, qi + 16), c_s0 = __shfl(c8, qi), c_s2 = __shfl(c8, qi + 32),
                  c_s3 = __shfl(c8, qi + 48);
        int off = run_cnt + (s > 0 ? c_s0 : 0) + (s > 1 ? c_s1 : 0) + (s > 2 ? c_s2 : 0);
#pragma unroll
        for (int h = 0; h < 8; ++h)
          if ((m8 >> h) & 1u) RK[qi][off++] = dkey(dd[h], pos0 + h);
        run_cnt += c_s0 + c_s1 + c_s2 + c_s3;
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  __builtin_amdgcn_wave_barrier();
  flush_run();
}

template <int KCAP, bool EXACT>
__global__ __launch_bounds__(256) void k_knn_select(KnnJob j) {
  const CloudDev& c = j.c;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c.n) return;
  const int k = j.k;
  if (blockIdx.x == 0 && threadIdx.x < kTaskRegions) j.task_ctr[threadIdx.x * kCtrStride] = 0u;   // for round 2
  if (j.redo[i >> 6]) return;
  if (j.round == 2 && !j.again[i]) return;
  const unsigned nc = j.cnt[i];
  const unsigned cap = j.round == 2 ? (unsigned)j.cap2 : (unsigned)j.cap;
  if (nc < (unsigned)k || (nc > cap && j.round == 2)) {   // still overflowing (or a bug guard):
    j.redo[i >> 6] = 1;                                     // the fallback recomputes the group
    return;
  }
  unsigned long long K[KCAP];
#pragma unroll
  for (int s = 0; s < KCAP; ++s) K[s] = ~0ull;
  const unsigned long long* cl = j.round == 2 ? j.cand2 + (size_t)j.slot2[i] * j.cap2 : j.cand + i;
  const size_t stride = j.round == 2 ? 1 : (size_t)c.n;
  const unsigned ne = min(nc, cap);
  unsigned long long out_min = ~0ull;   // the smallest key not kept (the exact-tie test below)
  for (unsigned e = 0; e < ne; ++e) {
    unsigned long long key = cl[(size_t)e * stride];
#pragma unroll
    for (int s = 0; s < KCAP; ++s) {
      if (key == K[s]) key = ~0ull;   // a leaf scanned twice (two walk entries): drop the duplicate
      const unsigned long long lo = key < K[s] ? key : K[s];
      key = key < K[s] ? K[s] : key;
      K[s] = lo;
    }
    out_min = key < out_min ? key : out_min;
  }
  if (nc > cap) {
    // first-round overflow: the k-th of the stored candidates (k real points)
    // is a far tighter ball than the first one; the point goes again with a
    // compact list of cap2 slots
    const int sl = (int)atomicAdd(j.n2, 1u);
    if (sl >= j.max2) {
      j.redo[i >> 6] = 1;
      return;
    }
    unsigned long long kk = K[0];
#pragma unroll
    for (int s = 0; s < KCAP; ++s)
      if (s == k - 1) kk = K[s];
    j.qstate[i].w = key_dist(kk);
    j.cnt[i] = 0u;
    j.slot2[i] = sl;
    j.again[i] = 1;
    return;
  }
  if (j.tie_list) {
    // a point at exactly the k-th distance left out: nanoflann's walk decides
    // which of the tied points is kept (nftree.hip re-runs this query)
    // (or two of the kept k equidistant: their order is nanoflann's walk order)
    unsigned long long kth = K[0];
    bool inner = false;
#pragma unroll
    for (int s = 0; s < KCAP; ++s) {
      if (s == k - 1) kth = K[s];
      if (!EXACT && s >= k && K[s] < out_min) out_min = K[s];
      if (s >= 1 && s < k) inner |= (K[s] >> 32) == (K[s - 1] >> 32);
    }
    if (inner || (out_min != ~0ull && (out_min >> 32) == (kth >> 32))) {
      const int slot = atomicAdd(j.tie_count, 1);
      if (slot < j.tie_cap) j.tie_list[slot] = i;
    }
  }
  // mean and biased covariance in neighbour order (nano_gicp_impl.hpp:392-399)
  double mx = 0, my = 0, mz = 0;
#pragma unroll
  for (int s = 0; s < KCAP; ++s) {
    if (EXACT || s < k) {
      const float4 p = ldg4(c.pts, (int)(unsigned)K[s]);
      mx += (double)p.x;
      my += (double)p.y;
      mz += (double)p.z;
    }
  }
  mx /= k;
  my /= k;
  mz /= k;
  double C[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < KCAP; ++s) {
    if (EXACT || s < k) {
      const float4 p = ldg4(c.pts, (int)(unsigned)K[s]);
      const double d0 = (double)p.x - mx, d1 = (double)p.y - my, d2 = (double)p.z - mz;
      C[0] += d0 * d0; C[1] += d0 * d1; C[2] += d0 * d2;
      C[3] += d1 * d0; C[4] += d1 * d1; C[5] += d1 * d2;
      C[6] += d2 * d0; C[7] += d2 * d1; C[8] += d2 * d2;
    }
  }
  for (int e = 0; e < 9; ++e) C[e] /= k;
  double out[6];
  regularize(C, j.method, out);
  double* o = j.cov6 + 6 * (size_t)i;
  for (int e = 0; e < 6; ++e) o[e] = out[e];
}

static inline int cdiv_k(long a, long b) { return (int)((a + b - 1) / b); }

int knn_task_cap_per_region(int n) {
  const long groups = (n + kTaskQ - 1) / kTaskQ;
  return (int)std::max<long>(1024, (groups * kTasksPerGroup + kTaskRegions - 1) / kTaskRegions);
}

static int knn_scan_blocks(int n) {
  const int groups = (n + kTaskQ - 1) / kTaskQ;
  int waves = std::min(std::max(groups, kTaskRegions), 8192);
  waves = (waves + 8 * kTaskRegions - 1) / (8 * kTaskRegions) * (8 * kTaskRegions);
  return waves / kKnnWaves;
}

bool launch_knn_covariances(hipStream_t s, const KnnJob& j, int upper) {
  const int n = j.c.n;
  if (j.k > 32) return false;
  const int nb = cdiv_k(n, 256);
  const int groups = cdiv_k(n, kTaskQ);
  if (j.k <= 10) k_knn_seed<10><<<nb, 256, 0, s>>>(j);
  else if (j.k <= 20) k_knn_seed<20><<<nb, 256, 0, s>>>(j);
  else k_knn_seed<32><<<nb, 256, 0, s>>>(j);
  const size_t lds = (size_t)kKnnWaves * kTaskLdsBytes + 2 * sizeof(f4v) * (size_t)upper;
  for (int round = 1; round <= 2; ++round) {
    KnnJob jr = j;
    jr.round = round;
    k_knn_collect<<<cdiv_k(groups, kKnnWaves), 64 * kKnnWaves, lds, s>>>(jr);
    k_knn_scan<<<knn_scan_blocks(n), 64 * kKnnWaves, 0, s>>>(jr);
    if (j.k == 10) k_knn_select<10, true><<<nb, 256, 0, s>>>(jr);
    else if (j.k == 20) k_knn_select<20, true><<<nb, 256, 0, s>>>(jr);
    else if (j.k <= 16) k_knn_select<16, false><<<nb, 256, 0, s>>>(jr);
    else k_knn_select<32, false><<<nb, 256, 0, s>>>(jr);
  }
  return true;
}

}  // namespace ddlo
