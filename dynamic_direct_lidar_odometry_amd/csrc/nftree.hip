// nftree.hip — device build of nanoflann's kd-tree (the tie-break order of
// the reference's searches, see nftree.hpp) and the kernels that re-run the
// flagged tied queries through it.
//
// Build = the recursion of divideTree (reference
// include/nano_gicp/impl/nanoflann_impl.hpp:987-1043) unrolled into levels:
//   big levels   every node of > kNfT points of one depth at once: its
//                middleSplit_ cut (:1045-1096) from the passed-down box and
//                the node's min / max, then planeSplit's two Hoare passes
//                (:1107-1143) as rank pairings (below), 6 kernels per level;
//   small nodes  a node of <= kNfT points: one wavefront splits its whole
//                subtree in LDS, depth first;
//   refit        leaf boxes up to the root: an inner node's box is the union
//                of its children's (:1035-1039), divlow / divhigh are the
//                children's box faces along divfeat (:1032-1033).
// Hoare pass as a rank pairing: with L = #{v < cut} (the final lim1), the
// loop "while (v[left] < cut) ++left; while (v[right] >= cut) --right; swap"
// swaps the r-th element >= cut inside [0, L) (ascending) with the r-th
// element < cut inside [L, n) (descending) for every r, and nothing else —
// so every element's destination follows from two prefix counts.  The
// second pass is the same over [lim1, n) with "<= cut".
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstdio>
#include <cstdlib>

#include "cov_math.hpp"
#include "gicp_types.hpp"
#include "launch.hpp"
#include "nftree.hpp"
#include "devknobs.hpp"

namespace ddlo {

namespace {

constexpr int kNfT = 8192;     // nodes up to this size are split by one workgroup in LDS (k_nf_sub)
constexpr int kNfCH = 2048;    // points per block in the big-level passes
constexpr int kNfBT = 256;     // threads per big-level block (8 points each)
constexpr int kNfPer = kNfCH / kNfBT;
constexpr int kNfLevelMargin = 9;   // big levels beyond log2(n / kNfT): ray-cast scans need 5-7 of them
constexpr int kNfSubWaves = 16;     // k_nf_sub: wavefronts per workgroup
constexpr int kNfSubQ = 168;        // k_nf_sub: nodes per depth (<= 2 x kNfT / (kNfLeafMax + 1))

__device__ __forceinline__ unsigned f2o(float f) {   // order-preserving float -> uint
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(unsigned o) {
  const unsigned u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return __uint_as_float(u);
}
// Coordinate f of a point in registers, as a bit-mask blend: LLVM folds a
// select chain on f (either form) into an element extract at a runtime
// index, i.e. a store of the float4 to scratch and an indexed load
// (k_nf_pass<2, false> had 144 B of scratch).
__device__ __forceinline__ float coord(const float4& p, int f) {
  const unsigned mx = 0u - (unsigned)(f == 0), my = 0u - (unsigned)(f == 1), mz = 0u - (unsigned)(f == 2);
  return __uint_as_float((__float_as_uint(p.x) & mx) | (__float_as_uint(p.y) & my) | (__float_as_uint(p.z) & mz));
}
// Coordinate f of a point in memory: one load at a computed address.  (The
// select form on a memory operand was lowered by ROCm 7.2's hipcc into a
// per-lane branch whose z address is computed under the f <= 0 branch's exec
// mask, so the f == 2 lanes loaded from the loop index taken as an address:
// wrong z splits in LDS, a fault in global memory.  ISA of the pre-fix code:
// profiles/r04_fc2aa78_isa.md, tools/isa_fc2aa78.sh.)
__device__ __forceinline__ float coord_at(const float4* p, int f) { return reinterpret_cast<const float*>(p)[f]; }

// middleSplit_ (:1045-1087): cut dimension and value from the passed-down
// box (lo, hi) and the node's point min / max (computeMinMax, :965-978).
// Constant indices only (registers, no private-memory arrays).
__device__ __forceinline__ void nf_cut3(const float lo[3], const float hi[3], const float mn[3], const float mx[3],
                                        int* feat, float* cut) {
  const float EPS = 0.00001f;
  float max_span = hi[0] - lo[0];
#pragma unroll
  for (int i = 1; i < 3; ++i) {
    const float span = hi[i] - lo[i];
    if (span > max_span) max_span = span;
  }
  float max_spread = -1;
  int cf = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float span = hi[i] - lo[i];
    if (span > (1 - EPS) * max_span) {
      const float spread = mx[i] - mn[i];
      if (spread > max_spread) {
        cf = i;
        max_spread = spread;
      }
    }
  }
  const float lc = cf == 0 ? lo[0] : (cf == 1 ? lo[1] : lo[2]);
  const float hc = cf == 0 ? hi[0] : (cf == 1 ? hi[1] : hi[2]);
  const float mnc = cf == 0 ? mn[0] : (cf == 1 ? mn[1] : mn[2]);
  const float mxc = cf == 0 ? mx[0] : (cf == 1 ? mx[1] : mx[2]);
  const float split_val = (lc + hc) / 2;
  float cv;
  if (split_val < mnc) cv = mnc;
  else if (split_val > mxc) cv = mxc;
  else cv = split_val;
  *feat = cf;
  *cut = cv;
}
__device__ __forceinline__ void nf_cut(const NfTask& t, int* feat, float* cut) {
  const float lo[3] = {t.lo[0], t.lo[1], t.lo[2]}, hi[3] = {t.hi[0], t.hi[1], t.hi[2]};
  const float mn[3] = {o2f(t.mm[0]), o2f(t.mm[1]), o2f(t.mm[2])};
  const float mx[3] = {o2f(t.mm[3]), o2f(t.mm[4]), o2f(t.mm[5])};
  nf_cut3(lo, hi, mn, mx, feat, cut);
}

// divlow / divhigh of node p (:1032-1033): the max of its left child's points
// along the cut dimension, the min of its right child's
__device__ __forceinline__ void nf_set_div(NfNode* nodes, int child, const float mn[3], const float mx[3]) {
  const int p = nodes[child].parent;
  if (p < 0) return;
  const int f = nodes[p].feat;
  if (nodes[p].c1 == child) nodes[p].divlow = f == 0 ? mx[0] : (f == 1 ? mx[1] : mx[2]);
  else nodes[p].divhigh = f == 0 ? mn[0] : (f == 1 ? mn[1] : mn[2]);
}

// :1090-1095
__device__ __forceinline__ int nf_index(int count, int lim1, int lim2) {
  if (lim1 > count / 2) return lim1;
  if (lim2 < count / 2) return lim2;
  return count / 2;
}

// ---- block-level helpers (blockDim.x a multiple of 64, <= 1024) -------------
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = __lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int o = __shfl_up(v, d);
    if (lane >= d) v += o;
  }
  return v;
}
// exclusive prefix of v over the block (thread order); *total = sum
__device__ __forceinline__ int block_excl_scan(int v, int* total, int* sh /* >= 17 ints */) {
  const int lane = __lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int inc = wave_incl_scan(v);
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int i = 0; i < nw; ++i) {
      const int t = sh[i];
      sh[i] = s;
      s += t;
    }
    sh[16] = s;
  }
  __syncthreads();
  const int r = sh[w] + inc - v;
  *total = sh[16];
  __syncthreads();
  return r;
}
__device__ __forceinline__ int block_sum(int v, int* sh) {
  int tot;
  (void)block_excl_scan(v, &tot, sh);
  return tot;
}

struct TaskView {   // a big-level block's task and chunk
  int t, c, blk;
  NfTask tk;
};
// The block's chunk and task: the map kernel's per-chunk task copy and the
// chunk count are independent loads (one round trip).  The copy's feat /
// cut are not the count kernel's: the pass kernels recompute the cut.
__device__ __forceinline__ bool task_of_block(const NfBuild& b, int L, TaskView* v) {
  const int par = L & 1;
  const int blk = blockIdx.x;
  v->tk = b.ctask[par * b.max_chunks + blk];   // grid = max_chunks: in bounds
  if (blk >= b.ctl->nchunks[par]) return false;
  v->blk = blk;
  v->t = v->tk.pad;
  v->c = blk - v->tk.chunk0;
  return true;
}

// sums of a per-chunk count over the task's chunks: all of them, and those before blk
__device__ __forceinline__ void task_chunk_sums(const int* cnt, const NfTask& tk, int blk, int* total, int* before, int* sh) {
  int a = 0, p = 0;
  for (int c = tk.chunk0 + (int)threadIdx.x; c < tk.chunk0 + tk.nch; c += blockDim.x) {
    const int v = cnt[c];
    a += v;
    if (c < blk) p += v;
  }
  *total = block_sum(a, sh);
  *before = block_sum(p, sh);
}

}  // namespace

// ---------------------------------------------------------------------------
// build kernels

// a gated build (NfBuild::gate, the tied-query count) does nothing when no
// query is tied: one scalar load per block
__device__ __forceinline__ bool nf_gated_off(const NfBuild* __restrict__ bp) {
  const int* g = bp->gate;
  return g && *g == 0;
}

__global__ void k_nf_init(const NfBuild* __restrict__ bp) {
  if (nf_gated_off(bp)) return;
  const NfBuild& b = *bp;
  if (threadIdx.x == 0) {
    NfCtl* ctl = b.ctl;
    ctl->nnodes = 1;
    ctl->nsmall = 0;
    ctl->err = 0;
    ctl->nchunks[0] = ctl->nchunks[1] = 0;
    for (int l = 0; l <= kNfMaxLevels; ++l) ctl->ntask[l] = 0;
    for (int l = 0; l < 16; ++l) ctl->dbg[l] = 0;
    NfTask r;
    r.node = 0;
    r.begin = 0;
    r.count = b.n;
    r.chunk0 = 0;
    r.nch = 0;
    r.feat = 0;
    r.cut = 0.f;
    // root_bbox = computeBoundingBox (:1459-1487): the min / max of all points
    for (int a = 0; a < 3; ++a) {
      const float mn = b.quant[a], mx = b.quant[4 + a];
      r.lo[a] = mn;
      r.hi[a] = mx;
      r.mm[a] = f2o(mn);
      r.mm[3 + a] = f2o(mx);
    }
    b.pend[0] = r;
    b.nodes[0].parent = -1;
    b.box[0] = make_float4(b.quant[0], b.quant[1], b.quant[2], 0.f);   // root_bbox
    b.box[1] = make_float4(b.quant[4], b.quant[5], b.quant[6], 0.f);
  }
}

// Level L's task list from the children its parent level produced (pend[L]):
// nodes > kNfT points become big tasks (their chunks listed), the others
// small tasks; the final call lists every remaining node as small.
__global__ __launch_bounds__(1024) void k_nf_map(const NfBuild* __restrict__ bp, int L) {
  if (nf_gated_off(bp)) return;
  const NfBuild& b = *bp;
  __shared__ int sh[17];
  __shared__ int s_big, s_small, s_ch, s_small0;
  NfCtl* ctl = b.ctl;
  const int np = L == 0 ? 1 : 2 * ctl->ntask[L - 1];
  const NfTask* P = b.pend + (size_t)L * b.max_pend;
  NfTask* T = b.tasks + (size_t)L * b.max_task;
  const bool final = L >= b.Lmax;
  if (threadIdx.x == 0) {
    s_big = s_small = s_ch = 0;
    s_small0 = ctl->nsmall;
  }
  __syncthreads();
  for (int base = 0; base < np; base += blockDim.x) {
    const int i = base + threadIdx.x;
    NfTask e;
    bool valid = false;
    if (i < np) {
      e = P[i];
      valid = e.count > 0 && e.node > 0 && e.node < b.cap;
      if (L == 0 && i == 0) valid = e.count > 0;
    }
    const bool big = valid && !final && e.count > kNfT;
    const bool sml = valid && !big;
    const int nch = big ? (e.count + kNfCH - 1) / kNfCH : 0;
    int tb, ts, tc;
    const int xb = block_excl_scan(big ? 1 : 0, &tb, sh);
    const int xs = block_excl_scan(sml ? 1 : 0, &ts, sh);
    const int xc = block_excl_scan(nch, &tc, sh);
    if (big && s_big + xb < b.max_task) {
      e.chunk0 = s_ch + xc;
      e.nch = nch;
      T[s_big + xb] = e;
    }
    if (sml && s_small0 + s_small + xs < b.max_small) b.small[s_small0 + s_small + xs] = e;
    __syncthreads();
    if (threadIdx.x == 0) {
      s_big += tb;
      s_small += ts;
      s_ch += tc;
    }
    __syncthreads();
  }
  const int nbig = min(s_big, b.max_task);
  if (threadIdx.x == 0) {
    if (s_big > b.max_task || s_small0 + s_small > b.max_small || s_ch > b.max_chunks) atomicOr(&ctl->err, 8);
    ctl->ntask[L] = final ? 0 : nbig;
    if (final) ctl->nnodes = b.cap;   // the small subtrees number their nodes in their own ranges
    ctl->nsmall = min(s_small0 + s_small, b.max_small);
    ctl->nchunks[L & 1] = final ? 0 : min(s_ch, b.max_chunks);
  }
  __threadfence_block();
  __syncthreads();
  if (final) return;
  // chunk -> task map (tasks are in chunk0 order)
  const int nchunks = min(s_ch, b.max_chunks);
  int* cmap = b.chunk_task + (L & 1) * b.max_chunks;
  NfTask* ct = b.ctask + (L & 1) * b.max_chunks;
  for (int c = threadIdx.x; c < nchunks; c += blockDim.x) {
    int lo = 0, hi = nbig - 1;
    while (lo < hi) {   // last task with chunk0 <= c
      const int mid = (lo + hi + 1) >> 1;
      if (T[mid].chunk0 <= c) lo = mid;
      else hi = mid - 1;
    }
    cmap[c] = lo;
    NfTask e = T[lo];
    e.pad = lo;
    ct[c] = e;
  }
  // the children this level will produce: their min / max start empty
  NfTask* C = b.pend + (size_t)(L + 1) * b.max_pend;
  for (int i = threadIdx.x; i < 2 * nbig; i += blockDim.x) {
    C[i].count = 0;
    for (int a = 0; a < 3; ++a) {
      C[i].mm[a] = 0xffffffffu;
      C[i].mm[3 + a] = 0u;
    }
  }
}

// Level L's map, fused into its count kernel (one launch less per level):
// every block scans the children its parent level produced (pend[L], a few
// dozen entries) for the big task holding its chunk and writes that chunk's
// task copy; block 0 also writes the task list, the small tasks and the
// counters, and the blocks clear the next level's children entries.  The
// same lists as k_nf_map (which still runs the final, all-small call).
__device__ __forceinline__ bool map_level_block(const NfBuild& b, int L, TaskView* v, int* sh) {
  __shared__ int s_big, s_small, s_ch, s_small0, s_t, s_found;
  __shared__ NfTask s_task;
  NfCtl* ctl = b.ctl;
  const int np = L == 0 ? 1 : 2 * ctl->ntask[L - 1];
  const NfTask* P = b.pend + (size_t)L * b.max_pend;
  NfTask* T = b.tasks + (size_t)L * b.max_task;
  const int blk = blockIdx.x;
  const bool lead = blk == 0;
  if (threadIdx.x == 0) {
    s_big = s_small = s_ch = 0;
    s_small0 = lead ? ctl->nsmall : 0;
    s_found = 0;
  }
  __syncthreads();
  for (int base = 0; base < np; base += blockDim.x) {
    const int i = base + threadIdx.x;
    NfTask e;
    bool valid = false;
    if (i < np) {
      e = P[i];
      valid = e.count > 0 && e.node > 0 && e.node < b.cap;
      if (L == 0 && i == 0) valid = e.count > 0;
    }
    const bool big = valid && e.count > kNfT;
    const bool sml = valid && !big;
    const int nch = big ? (e.count + kNfCH - 1) / kNfCH : 0;
    int tb, ts, tc;
    const int xb = block_excl_scan(big ? 1 : 0, &tb, sh);
    const int xs = block_excl_scan(sml ? 1 : 0, &ts, sh);
    const int xc = block_excl_scan(nch, &tc, sh);
    const int t = s_big + xb, c0 = s_ch + xc;
    if (big && t < b.max_task) {
      e.chunk0 = c0;
      e.nch = nch;
      if (lead) T[t] = e;
      if (blk >= c0 && blk < c0 + nch) {   // this block's chunk
        e.pad = t;
        s_task = e;
        s_t = t;
        s_found = 1;
      }
    }
    if (lead && sml && s_small0 + s_small + xs < b.max_small) b.small[s_small0 + s_small + xs] = e;
    __syncthreads();
    if (threadIdx.x == 0) {
      s_big += tb;
      s_small += ts;
      s_ch += tc;
    }
    __syncthreads();
  }
  const int nbig = min(s_big, b.max_task);
  const int nchunks = min(s_ch, b.max_chunks);
  if (lead && threadIdx.x == 0) {
    if (s_big > b.max_task || s_small0 + s_small > b.max_small || s_ch > b.max_chunks) atomicOr(&ctl->err, 8);
    ctl->ntask[L] = nbig;
    ctl->nsmall = min(s_small0 + s_small, b.max_small);
    ctl->nchunks[L & 1] = nchunks;
  }
  // the children this level will produce: their min / max start empty
  NfTask* C = b.pend + (size_t)(L + 1) * b.max_pend;
  for (int i = blk * (int)blockDim.x + (int)threadIdx.x; i < 2 * nbig; i += (int)(gridDim.x * blockDim.x)) {
    C[i].count = 0;
    for (int a = 0; a < 3; ++a) {
      C[i].mm[a] = 0xffffffffu;
      C[i].mm[3 + a] = 0u;
    }
  }
  if (!s_found || blk >= nchunks) return false;
  if (threadIdx.x == 0) b.ctask[(L & 1) * b.max_chunks + blk] = s_task;   // the pass kernels' one-load copy
  v->tk = s_task;
  v->blk = blk;
  v->t = s_t;
  v->c = blk - s_task.chunk0;
  return true;
}

// middleSplit_'s cut per task; #{v < cut} and #{v <= cut} per chunk
__global__ __launch_bounds__(kNfBT) void k_nf_count(const NfBuild* __restrict__ bp, int L) {
  if (nf_gated_off(bp)) return;
  const NfBuild& b = *bp;
  __shared__ int sh[17];
  TaskView v;
  if (!map_level_block(b, L, &v, sh)) return;
  int feat;
  float cut;
  nf_cut(v.tk, &feat, &cut);
  const int p0 = v.c * kNfCH, p1 = min(p0 + kNfCH, v.tk.count);
  int a = 0, ae = 0;
  float xs[kNfPer];   // the chunk's kNfPer loads per thread in flight together
#pragma unroll
  for (int j = 0; j < kNfPer; ++j) {
    const int p = p0 + (int)threadIdx.x + j * kNfBT;
    xs[j] = p < p1 ? coord_at(&b.vpts[v.tk.begin + p], feat) : NAN;   // NaN: both comparisons false
  }
#pragma unroll
  for (int j = 0; j < kNfPer; ++j) {
    a += xs[j] < cut;
    ae += xs[j] <= cut;
  }
  a = block_sum(a, sh);
  ae = block_sum(ae, sh);
  if (threadIdx.x == 0) {
    b.cA[v.blk] = a;
    b.cAE[v.blk] = ae;
    if (v.c == 0) {   // (the task list's feat / cut stay unset: every pass kernel recomputes the cut)
      const float mn[3] = {o2f(v.tk.mm[0]), o2f(v.tk.mm[1]), o2f(v.tk.mm[2])};
      const float mx[3] = {o2f(v.tk.mm[3]), o2f(v.tk.mm[4]), o2f(v.tk.mm[5])};
      nf_set_div(b.nodes, v.tk.node, mn, mx);   // the children's min / max are final now
    }
  }
}

// Hoare pass as rank pairing.  PASS 1: over [0, n), "good" = v < cut,
// boundary lo = lim1.  PASS 2: over [lim1, n), "good" = v == cut (<= cut
// there), boundary lim2.  TABLE: write each misplaced element into its rank
// slot; else (APPLY) overwrite each misplaced position with its partner.
template <int PASS, bool TABLE>
__global__ __launch_bounds__(kNfBT) void k_nf_pass(const NfBuild* __restrict__ bp, int L) {
  if (nf_gated_off(bp)) return;
  const NfBuild& b = *bp;
  __shared__ int sh[17];
  TaskView v;
  if (!task_of_block(b, L, &v)) return;
  const NfTask& tk = v.tk;
  int feat;
  float cut;
  nf_cut(tk, &feat, &cut);   // the count kernel's cut (a pure function of the task)
  // pass 1: the chunk's points first, their loads overlap the count sums'
  // (pass 2 loads them after its early exit: most nodes skip it)
  const int p0 = v.c * kNfCH + threadIdx.x * kNfPer;
  float4 e[kNfPer];
  if constexpr (PASS == 1) {
#pragma unroll
    for (int j = 0; j < kNfPer; ++j) {
      const int p = p0 + j;
      if (p < tk.count) e[j] = b.vpts[tk.begin + p];
    }
  }
  int lim1, before1, lim2 = 0, before2;
  task_chunk_sums(b.cA, tk, v.blk, &lim1, &before1, sh);
  int before = before1;
  int zlo = 0, zhi = lim1;   // the "good" zone [zlo, zhi) of this pass
  if (PASS == 2 || !TABLE) task_chunk_sums(b.cAE, tk, v.blk, &lim2, &before2, sh);
  // no element equals the cut (most nodes): pass 2 swaps nothing, and pass
  // 1's apply already finished the node (its children and record)
  const bool pass2_empty = lim2 == lim1;
  if (PASS == 2) {
    if (pass2_empty) return;
    task_chunk_sums(b.cE2, tk, v.blk, &before2, &before, sh);   // E after pass 1: none before lim1
    zlo = lim1;
    zhi = lim2;
  }
  const int ngood = zhi - zlo;
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < kNfPer; ++j) {
    const int p = p0 + j;
    if (p < tk.count) {
      if constexpr (PASS == 2) e[j] = b.vpts[tk.begin + p];
      const float x = coord(e[j], feat);
      cnt += PASS == 1 ? (x < cut) : (x == cut);
    }
  }
  int tot;
  int pref = before + block_excl_scan(cnt, &tot, sh);
  int ecount = 0;   // APPLY of pass 1: "== cut" after the pass (pass 2's counts)
#pragma unroll
  for (int j = 0; j < kNfPer; ++j) {
    const int p = p0 + j;
    if (p >= tk.count) continue;   // (p grows with j: the rest are past the task too; continue keeps e[] in registers)
    const float x = coord(e[j], feat);
    const bool good = PASS == 1 ? (x < cut) : (x == cut);
    float4 out = e[j];
    bool moved = false;
    int r = -1;
    if (p >= zlo && p < zhi && !good) r = (p - zlo) - pref;   // misplaced left: rank among the zone's bad ones
    else if (p >= zhi && good) r = ngood - pref - 1;          // misplaced right: rank from the end
    else r = -2;
    if (r == -1 || r < -2 || r >= tk.count) {   // never: a rank outside the task (guard against corrupt counts)
      atomicOr(&b.ctl->err, 16);
      r = -2;
    }
    if (r >= 0) {
      const bool left = p < zhi;
      if (TABLE) (left ? b.tblL : b.tblR)[tk.begin + r] = e[j];
      else out = (left ? b.tblR : b.tblL)[tk.begin + r];
      moved = true;
    }
    if (!TABLE) {
      // (w holds the index bits: a float compare would see small indices as
      // equal denormals, so the write follows the rank logic, not the values)
      if (moved) b.vpts[tk.begin + p] = out;
      if (PASS == 1) ecount += coord(out, feat) == cut;
      e[j] = out;
    }
    pref += good;
  }
  if (!TABLE && PASS == 1) {
    ecount = block_sum(ecount, sh);
    if (threadIdx.x == 0) b.cE2[v.blk] = ecount;
  }
  if (!TABLE && (PASS == 2 || pass2_empty)) {
    // the split index, the children's point min / max, and (one thread per
    // task) the node record and the children's pending entries
    const int index = nf_index(tk.count, lim1, lim2);
    // the two children's min / max, constant indices only (registers, no
    // private-memory array: a runtime child index put m[][] on the stack)
    float m[2][6];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        m[s][a] = INFINITY;
        m[s][3 + a] = -INFINITY;
      }
#pragma unroll
    for (int j = 0; j < kNfPer; ++j) {
      const int p = p0 + j;
      const bool in = p < tk.count;
      const bool left = p < index;
      const float cc[3] = {e[j].x, e[j].y, e[j].z};
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const float lo_c = in ? cc[a] : INFINITY, hi_c = in ? cc[a] : -INFINITY;
        m[0][a] = fminf(m[0][a], left ? lo_c : INFINITY);
        m[0][3 + a] = fmaxf(m[0][3 + a], left ? hi_c : -INFINITY);
        m[1][a] = fminf(m[1][a], left ? INFINITY : lo_c);
        m[1][3 + a] = fmaxf(m[1][3 + a], left ? -INFINITY : hi_c);
      }
    }
    NfTask* C = b.pend + (size_t)(L + 1) * b.max_pend;
    __shared__ unsigned smm[kNfBT / 64][12];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        float x = m[s][a];
        for (int d = 32; d >= 1; d >>= 1) {
          const float o = __shfl_xor(x, d);
          x = a < 3 ? fminf(x, o) : fmaxf(x, o);
        }
        if (__lane_id() == 0) smm[threadIdx.x >> 6][6 * s + a] = f2o(x);
      }
    __syncthreads();
    if (threadIdx.x < 12) {   // one atomic per block and value
      const int s = threadIdx.x / 6, a = threadIdx.x % 6;
      unsigned u = smm[0][threadIdx.x];
      for (int w = 1; w < kNfBT / 64; ++w) u = a < 3 ? min(u, smm[w][threadIdx.x]) : max(u, smm[w][threadIdx.x]);
      const float x = o2f(u);
      if (x == x && !isinf(x)) {
        unsigned* dst = &C[2 * v.t + s].mm[a];
        if (a < 3) atomicMin(dst, u);
        else atomicMax(dst, u);
      }
    }
    if (v.c == 0 && threadIdx.x == 0) {
      NfCtl* ctl = b.ctl;
      const int c1 = atomicAdd(&ctl->nnodes, 2);
      if (c1 + 2 > b.big_ids) {
        atomicOr(&ctl->err, 1);
        return;
      }
      NfNode* nd = b.nodes;
      nd[tk.node].c1 = c1;
      nd[tk.node].c2 = c1 + 1;
      nd[tk.node].feat = feat;
      nd[c1].parent = tk.node;
      nd[c1 + 1].parent = tk.node;
      // left_bbox / right_bbox (:1024-1030)
      for (int s = 0; s < 2; ++s) {
        NfTask& ch = C[2 * v.t + s];
        ch.node = c1 + s;
        ch.begin = tk.begin + (s == 0 ? 0 : index);
        ch.count = s == 0 ? index : tk.count - index;
        for (int a = 0; a < 3; ++a) {
          ch.lo[a] = tk.lo[a];
          ch.hi[a] = tk.hi[a];
        }
        if (s == 0) ch.hi[feat] = cut;
        else ch.lo[feat] = cut;
      }
    }
  }
}

// Small nodes (<= kNfT points): one workgroup per node, its whole subtree in
// LDS, breadth first — all nodes of one depth at once, one wavefront per
// node (k_nf_sub).  A node the big levels left larger than kNfT (a very
// unbalanced cloud) is split depth first by one wavefront in global memory
// (k_nf_small_global, rank lists in the pairing tables).  Node ids of a
// subtree come from the task's own range (NfBuild::big_ids), and every node
// writes its parent's divlow / divhigh from its own min / max, so no global
// atomics and no bottom-up pass.

__device__ __forceinline__ float wred(float x, bool mx) {
  for (int d = 32; d >= 1; d >>= 1) {
    const float o = __shfl_xor(x, d);
    x = mx ? fmaxf(x, o) : fminf(x, o);
  }
  return x;
}
// wave-scope ordering of LDS / memory between lanes (a node is one wavefront's)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// one Hoare pass over [zlo0, n) of the node at P (good = v < cut, or
// v == cut for pass 2), boundary zhi: pair the r-th bad element of
// [zlo0, zhi) with the r-th good element of [zhi, n) from the end.
// One wavefront; returns false on an (impossible) count mismatch.
template <class IT>
__device__ bool wave_pass(float4* P, IT* ML, IT* MR, int cap, int zlo0, int zhi, int n, int feat, float cut, bool pass2,
                          NfCtl* ctl) {
  const int lane = __lane_id();
  int m = 0;
  for (int i0 = zlo0; i0 < zhi; i0 += 64) {
    const int i = i0 + lane;
    bool f = false;
    if (i < zhi) {
      const float x = coord_at(&P[i], feat);
      f = !(pass2 ? x == cut : x < cut);
    }
    const unsigned long long mask = __ballot(f);
    const int slot = m + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
    if (f && slot < cap) ML[slot] = (IT)i;
    m += __popcll(mask);
  }
  int m2 = 0;
  for (int i0 = n; i0 > zhi; i0 -= 64) {
    const int i = i0 - 1 - lane;   // lane order = descending positions
    bool f = false;
    if (i >= zhi) {
      const float x = coord_at(&P[i], feat);
      f = pass2 ? x == cut : x < cut;
    }
    const unsigned long long mask = __ballot(f);
    const int slot = m2 + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
    if (f && slot < cap) MR[slot] = (IT)i;
    m2 += __popcll(mask);
  }
  wave_sync();
  if (m != m2 || m > cap) {   // never (equal by construction): report, swap nothing
    if (lane == 0) {
      atomicOr(&ctl->err, 32);
      int* dbg = ctl->dbg;
      if (atomicCAS(dbg, 0, 1) == 0) {
        dbg[1] = zlo0; dbg[2] = zhi; dbg[3] = n; dbg[4] = feat; dbg[5] = __float_as_int(cut);
        dbg[6] = pass2; dbg[7] = m; dbg[8] = m2; dbg[9] = cap; dbg[10] = (int)blockIdx.x;
      }
    }
    return false;
  }
  for (int r = lane; r < m; r += 64) {
    const int a = ML[r], c = MR[r];
    const float4 t = P[a];
    P[a] = P[c];
    P[c] = t;
  }
  wave_sync();
  return true;
}

// A node to split (or a leaf to record), as the subtree kernels queue it.
struct NfSubNode {
  int lb, n, node, par;   // first point (local), count, node id, parent id
  float lo[3], hi[3];     // the box divideTree passes down
};

// One wavefront splits one node whose points are Q[0, n) (local offset lb
// from the task's first point `base`): computeMinMax, the parent's div,
// leaf or middleSplit_ + planeSplit + the children's entries.  Returns the
// children through ch[2] (count 0 = a leaf was recorded).
template <class IT>
__device__ int wave_split(const NfBuild& b, float4* Q, IT* ML, IT* MR, int cap, const NfSubNode& nd, int base,
                          int c1, NfSubNode ch[2]) {
  NfCtl* ctl = b.ctl;
  const int lane = __lane_id();
  const int n = nd.n;
  // computeMinMax over the node (also the leaf's bbox, :998-1013)
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = lane; i < n; i += 64) {
    const float4 p = Q[i];
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
  for (int a = 0; a < 3; ++a) {
    mn[a] = wred(mn[a], false);
    mx[a] = wred(mx[a], true);
  }
  if (lane == 0 && nd.par >= 0) {   // the parent's divlow / divhigh (:1032-1033)
    const int f = b.nodes[nd.par].feat;
    if (b.nodes[nd.par].c1 == nd.node) b.nodes[nd.par].divlow = f == 0 ? mx[0] : (f == 1 ? mx[1] : mx[2]);
    else b.nodes[nd.par].divhigh = f == 0 ? mn[0] : (f == 1 ? mn[1] : mn[2]);
  }
  if (n <= kNfLeafMax) {   // leaf (:992-1014)
    if (lane == 0) {
      b.nodes[nd.node].c1 = base + nd.lb;
      b.nodes[nd.node].c2 = base + nd.lb + n;
      b.nodes[nd.node].feat = -1;
    }
    return 0;
  }
  int feat;
  float cut;
  nf_cut3(nd.lo, nd.hi, mn, mx, &feat, &cut);
  feat = __builtin_amdgcn_readfirstlane(feat);   // wave-uniform by construction: scalar from here on
  cut = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(cut)));
  int lim1 = 0, lim2 = 0;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    const float x = i < n ? coord_at(&Q[i], feat) : INFINITY;
    lim1 += __popcll(__ballot(i < n && x < cut));
    lim2 += __popcll(__ballot(i < n && x <= cut));
  }
  if (!wave_pass(Q, ML, MR, cap, 0, lim1, n, feat, cut, false, ctl)) return -1;
  // pass 2 swaps nothing when no element equals the cut (most nodes)
  if (lim2 > lim1 && !wave_pass(Q, ML, MR, cap, lim1, lim2, n, feat, cut, true, ctl)) return -1;
  const int index = nf_index(n, lim1, lim2);
  if (lane == 0) {
    b.nodes[nd.node].c1 = c1;
    b.nodes[nd.node].c2 = c1 + 1;
    b.nodes[nd.node].feat = feat;
    b.nodes[c1].parent = nd.node;
    b.nodes[c1 + 1].parent = nd.node;
  }
  // left_bbox / right_bbox (:1024-1030)
  for (int s = 0; s < 2; ++s) {
    ch[s].lb = nd.lb + (s == 0 ? 0 : index);
    ch[s].n = s == 0 ? index : n - index;
    ch[s].node = c1 + s;
    ch[s].par = nd.node;
    for (int a = 0; a < 3; ++a) {
      ch[s].lo[a] = nd.lo[a];
      ch[s].hi[a] = nd.hi[a];
    }
  }
  if (feat == 0) { ch[0].hi[0] = cut; ch[1].lo[0] = cut; }
  else if (feat == 1) { ch[0].hi[1] = cut; ch[1].lo[1] = cut; }
  else { ch[0].hi[2] = cut; ch[1].lo[2] = cut; }
  return 2;
}

struct SubLds {
  float4 P[kNfT];
  unsigned short ML[kNfT / 2], MR[kNfT / 2];   // per node: the slots [lb / 2, (lb + n) / 2)
  NfSubNode q[2][kNfSubQ];
  int qn[2], next_id, pad;
  // a depth of few nodes is split by groups of wavefronts (group_depth)
  float gred[kNfSubWaves][6];
  int gcnt[kNfSubWaves][2];
  int gfeat[kNfSubWaves], gleaf[kNfSubWaves];
  float gcut[kNfSubWaves];
};

// One Hoare pass of a node by a group of G wavefronts (gw = this one's
// index), every wavefront of the workgroup in lockstep (barriers inside; a
// wavefront without a node passes act = false).  The zone [zlo0, zhi) is
// cut into 64-position chunks from its start, the rest [zhi, n) from its
// end; chunk counts (kept in `cnt`, 256 slots of this group's, the ML
// space: they are read into registers before ML is written) give every
// chunk its first rank slot.
__device__ void group_pass(float4* Q, unsigned short* ML, unsigned short* MR, unsigned short* cnt, bool act, int gw,
                           int G, int zlo0, int zhi, int n, int feat, float cut, bool pass2, NfCtl* ctl) {
  const int lane = __lane_id();
  const int nz = act ? (zhi - zlo0 + 63) / 64 : 0;   // zone chunks, ascending
  const int nr = act ? (n - zhi + 63) / 64 : 0;       // right chunks, descending from n
  for (int z = gw; z < nz; z += G) {
    const int i = zlo0 + 64 * z + lane;
    bool f = false;
    if (i < zhi) {
      const float x = coord_at(&Q[i], feat);
      f = !(pass2 ? x == cut : x < cut);
    }
    const int c = __popcll(__ballot(f));
    if (lane == 0) cnt[z] = (unsigned short)c;
  }
  for (int r = gw; r < nr; r += G) {
    const int i = n - 1 - 64 * r - lane;
    bool f = false;
    if (i >= zhi) {
      const float x = coord_at(&Q[i], feat);
      f = pass2 ? x == cut : x < cut;
    }
    const int c = __popcll(__ballot(f));
    if (lane == 0) cnt[128 + r] = (unsigned short)c;
  }
  __syncthreads();
  // exclusive chunk prefixes (<= 128 chunks each: two per lane)
  const int a0 = lane < nz ? cnt[lane] : 0, a1 = lane + 64 < nz ? cnt[lane + 64] : 0;
  const int b0 = lane < nr ? cnt[128 + lane] : 0, b1 = lane + 64 < nr ? cnt[128 + lane + 64] : 0;
  const int sa0 = wave_incl_scan(a0), ta = __builtin_amdgcn_readlane(sa0, 63);
  const int sa1 = wave_incl_scan(a1) + ta;
  const int sb0 = wave_incl_scan(b0), tb = __builtin_amdgcn_readlane(sb0, 63);
  const int sb1 = wave_incl_scan(b1) + tb;
  const int ea0 = sa0 - a0, ea1 = sa1 - a1, eb0 = sb0 - b0, eb1 = sb1 - b1;
  const int m = __builtin_amdgcn_readlane(sa1, 63), m2 = __builtin_amdgcn_readlane(sb1, 63);
  __syncthreads();   // the counts are in registers: ML may be written
  const bool ok = m == m2;
  if (act && !ok && gw == 0 && lane == 0) atomicOr(&ctl->err, 32);
  if (act && ok) {
    for (int z = gw; z < nz; z += G) {
      const int i = zlo0 + 64 * z + lane;
      bool f = false;
      if (i < zhi) {
        const float x = coord_at(&Q[i], feat);
        f = !(pass2 ? x == cut : x < cut);
      }
      const unsigned long long mask = __ballot(f);
      const int off = __builtin_amdgcn_readlane(z < 64 ? ea0 : ea1, z & 63);
      const int slot = off + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
      if (f) ML[slot] = (unsigned short)i;
    }
    for (int r = gw; r < nr; r += G) {
      const int i = n - 1 - 64 * r - lane;
      bool f = false;
      if (i >= zhi) {
        const float x = coord_at(&Q[i], feat);
        f = pass2 ? x == cut : x < cut;
      }
      const unsigned long long mask = __ballot(f);
      const int off = __builtin_amdgcn_readlane(r < 64 ? eb0 : eb1, r & 63);
      const int slot = off + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
      if (f) MR[slot] = (unsigned short)i;
    }
  }
  __syncthreads();
  if (act && ok) {
    for (int rr = gw * 64 + lane; rr < m; rr += 64 * G) {
      const int a = ML[rr], c = MR[rr];
      const float4 t = Q[a];
      Q[a] = Q[c];
      Q[c] = t;
    }
  }
  __syncthreads();
}

// A depth of nq <= kNfSubWaves / 2 nodes: node j by the G = kNfSubWaves /
// pow2(nq) wavefronts [j G, (j + 1) G); the same steps as wave_split.
__device__ void group_depth(const NfBuild& b, SubLds& S, int cur, int nq, int base, int id_end) {
  const int lane = __lane_id(), wave = threadIdx.x >> 6;
  int p2 = 1;
  while (p2 < nq) p2 <<= 1;
  const int G = kNfSubWaves / p2;
  const int j = wave / G, gw = wave % G;
  const bool has = j < nq;
  NfSubNode nd;
  if (has) nd = S.q[cur][j];
  else {
    nd.lb = 0;
    nd.n = 0;
  }
  float4* Q = S.P + nd.lb;
  // computeMinMax (:965-978, leaf bbox :998-1013)
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = gw * 64 + lane; i < nd.n; i += 64 * G) {
    const float4 p = Q[i];
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
  for (int a = 0; a < 3; ++a) {
    mn[a] = wred(mn[a], false);
    mx[a] = wred(mx[a], true);
  }
  if (lane == 0)
    for (int a = 0; a < 3; ++a) {
      S.gred[wave][a] = mn[a];
      S.gred[wave][3 + a] = mx[a];
    }
  __syncthreads();
  if (has && gw == 0 && lane == 0) {
    for (int g = 1; g < G; ++g)
      for (int a = 0; a < 3; ++a) {
        mn[a] = fminf(mn[a], S.gred[wave + g][a]);
        mx[a] = fmaxf(mx[a], S.gred[wave + g][3 + a]);
      }
    if (nd.par >= 0) {   // the parent's divlow / divhigh (:1032-1033)
      const int f = b.nodes[nd.par].feat;
      if (b.nodes[nd.par].c1 == nd.node) b.nodes[nd.par].divlow = f == 0 ? mx[0] : (f == 1 ? mx[1] : mx[2]);
      else b.nodes[nd.par].divhigh = f == 0 ? mn[0] : (f == 1 ? mn[1] : mn[2]);
    }
    if (nd.n <= kNfLeafMax) {   // leaf (:992-1014)
      b.nodes[nd.node].c1 = base + nd.lb;
      b.nodes[nd.node].c2 = base + nd.lb + nd.n;
      b.nodes[nd.node].feat = -1;
      S.gleaf[j] = 1;
    } else {
      int feat;
      float cut;
      nf_cut3(nd.lo, nd.hi, mn, mx, &feat, &cut);
      S.gfeat[j] = feat;
      S.gcut[j] = cut;
      S.gleaf[j] = 0;
    }
  }
  __syncthreads();
  const bool act = has && !S.gleaf[j];
  const int feat = act ? S.gfeat[j] : 0;
  const float cut = act ? S.gcut[j] : 0.f;
  int c_lt = 0, c_le = 0;
  for (int i0 = gw * 64; act && i0 < nd.n; i0 += 64 * G) {
    const int i = i0 + lane;
    const float x = i < nd.n ? coord_at(&Q[i], feat) : INFINITY;
    c_lt += __popcll(__ballot(i < nd.n && x < cut));
    c_le += __popcll(__ballot(i < nd.n && x <= cut));
  }
  if (lane == 0) {
    S.gcnt[wave][0] = c_lt;
    S.gcnt[wave][1] = c_le;
  }
  __syncthreads();
  int lim1 = 0, lim2 = 0;
  if (has)
    for (int g = 0; g < G; ++g) {
      lim1 += S.gcnt[j * G + g][0];
      lim2 += S.gcnt[j * G + g][1];
    }
  unsigned short* cnt = S.ML + 256 * (has ? j : 0);
  group_pass(Q, S.ML + nd.lb / 2, S.MR + nd.lb / 2, cnt, act, gw, G, 0, lim1, nd.n, feat, cut, false, b.ctl);
  // pass 2 (barriers inside: a workgroup-uniform decision) only if a node of
  // this depth has elements equal to its cut
  bool need2 = false;
  for (int jj = 0; jj < nq; ++jj) {
    int l1 = 0, l2 = 0;
    for (int g = 0; g < G; ++g) {
      l1 += S.gcnt[jj * G + g][0];
      l2 += S.gcnt[jj * G + g][1];
    }
    need2 |= !S.gleaf[jj] && l2 > l1;
  }
  if (need2)
    group_pass(Q, S.ML + nd.lb / 2, S.MR + nd.lb / 2, cnt, act && lim2 > lim1, gw, G, lim1, lim2, nd.n, feat, cut, true,
               b.ctl);
  if (act && gw == 0 && lane == 0) {
    const int index = nf_index(nd.n, lim1, lim2);
    const int c1 = atomicAdd(&S.next_id, 2);
    if (c1 + 2 > id_end) {
      atomicOr(&b.ctl->err, 1);
    } else {
      b.nodes[nd.node].c1 = c1;
      b.nodes[nd.node].c2 = c1 + 1;
      b.nodes[nd.node].feat = feat;
      b.nodes[c1].parent = nd.node;
      b.nodes[c1 + 1].parent = nd.node;
      NfSubNode ch[2];
      for (int s2 = 0; s2 < 2; ++s2) {   // left_bbox / right_bbox (:1024-1030)
        ch[s2].lb = nd.lb + (s2 == 0 ? 0 : index);
        ch[s2].n = s2 == 0 ? index : nd.n - index;
        ch[s2].node = c1 + s2;
        ch[s2].par = nd.node;
        for (int a = 0; a < 3; ++a) {
          ch[s2].lo[a] = nd.lo[a];
          ch[s2].hi[a] = nd.hi[a];
        }
      }
      if (feat == 0) { ch[0].hi[0] = cut; ch[1].lo[0] = cut; }
      else if (feat == 1) { ch[0].hi[1] = cut; ch[1].lo[1] = cut; }
      else { ch[0].hi[2] = cut; ch[1].lo[2] = cut; }
      const int slot = atomicAdd(&S.qn[cur ^ 1], 2);
      if (slot + 2 <= kNfSubQ) {
        S.q[cur ^ 1][slot] = ch[0];
        S.q[cur ^ 1][slot + 1] = ch[1];
      } else {
        atomicOr(&b.ctl->err, 4);
      }
    }
  }
}

__global__ __launch_bounds__(64 * kNfSubWaves) void k_nf_sub(const NfBuild* __restrict__ bp) {
  if (nf_gated_off(bp)) return;
  const NfBuild& b = *bp;
  __shared__ SubLds S;   // ~157 KB: one workgroup per CU
  if ((int)blockIdx.x >= b.ctl->nsmall) return;
  const NfTask tk = b.small[blockIdx.x];
  if (tk.count > kNfT) return;   // k_nf_small_global's
  const int lane = __lane_id(), wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < tk.count; i += blockDim.x) S.P[i] = b.vpts[tk.begin + i];
  if (threadIdx.x == 0) {
    NfSubNode r;
    r.lb = 0;
    r.n = tk.count;
    r.node = tk.node;
    r.par = b.nodes[tk.node].parent;
    for (int a = 0; a < 3; ++a) {
      r.lo[a] = tk.lo[a];
      r.hi[a] = tk.hi[a];
    }
    S.q[0][0] = r;
    S.qn[0] = 1;
    S.qn[1] = 0;
    S.next_id = b.big_ids + 2 * tk.begin;   // this subtree's ids: [big_ids + 2 begin, big_ids + 2 (begin + count))
  }
  __syncthreads();
  const int id_end = b.big_ids + 2 * (tk.begin + tk.count);
  for (int depth = 0, cur = 0; depth < kNfStack; ++depth, cur ^= 1) {
    const int nq = S.qn[cur];
    if (nq == 0) break;
    if (nq <= kNfSubWaves / 2) {
      group_depth(b, S, cur, nq, tk.begin, id_end);
    } else for (int j = wave; j < nq; j += kNfSubWaves) {
      const NfSubNode nd = S.q[cur][j];
      int c1 = 0;
      if (nd.n > kNfLeafMax) {
        if (lane == 0) c1 = atomicAdd(&S.next_id, 2);
        c1 = __builtin_amdgcn_readfirstlane(c1);
        if (c1 + 2 > id_end) {
          if (lane == 0) atomicOr(&b.ctl->err, 1);
          continue;
        }
      }
      NfSubNode ch[2];
      const int nc = wave_split(b, S.P + nd.lb, S.ML + nd.lb / 2, S.MR + nd.lb / 2, nd.n / 2, nd, tk.begin, c1, ch);
      if (nc == 2 && lane == 0) {
        const int slot = atomicAdd(&S.qn[cur ^ 1], 2);
        if (slot + 2 <= kNfSubQ) {
          S.q[cur ^ 1][slot] = ch[0];
          S.q[cur ^ 1][slot + 1] = ch[1];
        } else {
          atomicOr(&b.ctl->err, 4);
        }
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      S.qn[cur] = 0;
      if (S.qn[cur ^ 1] > kNfSubQ) S.qn[cur ^ 1] = kNfSubQ;
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < tk.count; i += blockDim.x) b.vpts[tk.begin + i] = S.P[i];
}

// a task larger than kNfT: depth first by one wavefront, in global memory
struct NfGStack {
  NfSubNode e[kNfStack];
};
__global__ __launch_bounds__(64) void k_nf_small_global(const NfBuild* __restrict__ bp) {
  if (nf_gated_off(bp)) return;
  const NfBuild& b = *bp;
  __shared__ NfGStack S;
  if ((int)blockIdx.x >= b.ctl->nsmall) return;
  const NfTask tk = b.small[blockIdx.x];
  if (tk.count <= kNfT) return;   // k_nf_sub's
  const int lane = __lane_id();
  float4* P = b.vpts + tk.begin;
  unsigned* ML = reinterpret_cast<unsigned*>(b.tblL + tk.begin);   // the pairing tables' space: slots [lb / 2, ...)
  unsigned* MR = reinterpret_cast<unsigned*>(b.tblR + tk.begin);
  int next_id = b.big_ids + 2 * tk.begin;
  const int id_end = b.big_ids + 2 * (tk.begin + tk.count);
  if (lane == 0) {
    NfSubNode r;
    r.lb = 0;
    r.n = tk.count;
    r.node = tk.node;
    r.par = b.nodes[tk.node].parent;
    for (int a = 0; a < 3; ++a) {
      r.lo[a] = tk.lo[a];
      r.hi[a] = tk.hi[a];
    }
    S.e[0] = r;
  }
  wave_sync();
  int sp = 1;
  while (sp > 0) {
    --sp;
    const NfSubNode nd = S.e[sp];
    wave_sync();
    int c1 = 0;
    if (nd.n > kNfLeafMax) {
      c1 = next_id;
      next_id += 2;
      if (c1 + 2 > id_end || sp + 2 > kNfStack) {
        if (lane == 0) atomicOr(&b.ctl->err, c1 + 2 > id_end ? 1 : 4);
        return;
      }
    }
    NfSubNode ch[2];
    const int nc = wave_split(b, P + nd.lb, ML + nd.lb / 2, MR + nd.lb / 2, nd.n / 2, nd, tk.begin, c1, ch);
    if (nc < 0) return;
    if (nc == 2) {
      if (lane == 0) {   // the left child is popped first
        S.e[sp] = ch[1];
        S.e[sp + 1] = ch[0];
      }
      sp += 2;
      wave_sync();
    }
  }
}

// ---------------------------------------------------------------------------
// tie resolution: re-run the flagged queries with nanoflann's search, one
// wavefront per query (nf_search_wave)
constexpr int kNfResolveWaves = 4;

// Lane j < k holds the j-th neighbour (original index rix): the mean and
// biased covariance in neighbour order (nano_gicp_impl.hpp:392-399),
// regularised, written by lane 0.  Whole wavefront.
__device__ __forceinline__ void nf_cov_wave(const CloudDev& c, int rix, int k, int method, double* o) {
  const int lane = __lane_id();
  float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
  if (lane < k) p = c.pts[c.inv_perm[rix]];
  double mx = 0, my = 0, mz = 0;
  for (int j = 0; j < k; ++j) {
    mx += (double)__shfl(p.x, j);
    my += (double)__shfl(p.y, j);
    mz += (double)__shfl(p.z, j);
  }
  mx /= k;
  my /= k;
  mz /= k;
  double C[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < k; ++j) {
    const double d0 = (double)__shfl(p.x, j) - mx, d1 = (double)__shfl(p.y, j) - my, d2 = (double)__shfl(p.z, j) - mz;
    C[0] += d0 * d0; C[1] += d0 * d1; C[2] += d0 * d2;
    C[3] += d1 * d0; C[4] += d1 * d1; C[5] += d1 * d2;
    C[6] += d2 * d0; C[7] += d2 * d1; C[8] += d2 * d2;
  }
  for (int e = 0; e < 9; ++e) C[e] /= k;
  double out[6];
  regularize(C, method, out);
  if (lane == 0)
    for (int e = 0; e < 6; ++e) o[e] = out[e];
}

__global__ __launch_bounds__(64 * kNfResolveWaves) void k_nf_resolve_cov(NfTreeDev t, CloudDev c, TieList ties, int k,
                                                                        int method, double* __restrict__ cov6,
                                                                        const int* __restrict__ status,
                                                                        int* __restrict__ err) {
  __shared__ NfWaveStack stk[kNfResolveWaves];
  NfWaveStack* S = &stk[threadIdx.x >> 6];
  const int lane = __lane_id();
  const int nc = *ties.count;
  const int nl = min(nc, ties.cap);
  if (nc > ties.cap && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, 8);   // list overflow (never: cap = 2n)
  const int* list = ties.list;
  if (*status) {   // the tree build failed: report, keep the Morton-order answers
    if (blockIdx.x == 0 && threadIdx.x == 0 && nl > 0) atomicOr(err, 2 | (*status << 8));
    return;
  }
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  for (int li = wave; li < nl; li += nwaves) {
    const int s = list[li];   // sorted position of the query point
    const float4 q = c.pts[s];
    float rd;
    int rix;
    if (!nf_search_wave(t, q.x, q.y, q.z, k, S, &rd, &rix)) {   // 1: deeper than kNfStack, 4: fewer than k
      if (lane == 0) atomicOr(err, rix == -2 ? 1 : 4);
      continue;
    }
    nf_cov_wave(c, rix, k, method, cov6 + 6 * (size_t)s);
  }
}

__global__ __launch_bounds__(64 * kNfResolveWaves) void k_nf_resolve_knn(NfTreeDev t, const float4* __restrict__ q,
                                                                        TieList ties, int k,
                                                                        int* __restrict__ out_idx,
                                                                        float* __restrict__ out_d,
                                                                        const int* __restrict__ status,
                                                                        int* __restrict__ err) {
  __shared__ NfWaveStack stk[kNfResolveWaves];
  NfWaveStack* S = &stk[threadIdx.x >> 6];
  const int lane = __lane_id();
  const int nc = *ties.count;
  const int nl = min(nc, ties.cap);
  if (nc > ties.cap && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, 8);   // list overflow (never: cap = 2n)
  const int* list = ties.list;
  if (*status) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && nl > 0) atomicOr(err, 2 | (*status << 8));
    return;
  }
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  for (int li = wave; li < nl; li += nwaves) {
    const int i = list[li];   // query row
    const float4 p = q[i];
    float rd;
    int rix;
    if (!nf_search_wave(t, p.x, p.y, p.z, k, S, &rd, &rix)) {
      if (lane == 0) atomicOr(err, rix == -2 ? 1 : 4);
      continue;
    }
    if (lane < k) {
      out_idx[(size_t)i * k + lane] = rix;
      out_d[(size_t)i * k + lane] = rd;
    }
  }
}

// ---------------------------------------------------------------------------
// Lazy tie resolution: nanoflann's search of one tied query with the tree
// built only where that search walks.  divideTree (:987-1043) works in place
// on vind, depth first, and a node's split reads and permutes only its own
// range, so a node's split depends only on its ancestors' splits: a search
// that splits each node the first time it enters it, on a private copy of
// vind, meets exactly the nodes, cuts, divlow / divhigh and leaf orders of
// the full tree.  One workgroup per tied query; every split is middleSplit_
// + planeSplit as rank pairings (as the full build), whole-workgroup passes
// over the node's range in global memory (L2).  A scan has ~1 tied query,
// so this replaces the whole-cloud build (~0.5-0.8 ms) by one path.
constexpr int kLzT = 512;            // threads per workgroup (256 VGPRs: the epilogue's fp64 regularisation spilled at 128)
constexpr int kLzW = kLzT / 64;
constexpr int kLzStack = 96;         // search frames (depth of the tree + 1)

struct LzFrame {
  int begin, count, state, feat;
  float lx, ly, lz, hx, hy, hz;      // the box divideTree passes down (named fields: a runtime-indexed
                                     // array member would put the frame copies in private memory)
  float fm, fd, divlow, divhigh;     // mindistsq, the saved dists[feat], the split's divs
  int index;                         // split position (relative to begin)
  float cut;
  int node;                          // >= 0: a node of the built top levels (its record); -1: a lazily split range
  int pad;
};
// left_bbox (.hi[feat] = cut) / right_bbox (.lo[feat] = cut) of divideTree (:1024-1030)
// (value selects: a store through a feat-dependent field pointer keeps the frame in private memory)
__device__ __forceinline__ void lz_set_hi(LzFrame& f, int feat, float v) {
  f.hx = feat == 0 ? v : f.hx;
  f.hy = feat == 1 ? v : f.hy;
  f.hz = feat == 2 ? v : f.hz;
}
__device__ __forceinline__ void lz_set_lo(LzFrame& f, int feat, float v) {
  f.lx = feat == 0 ? v : f.lx;
  f.ly = feat == 1 ? v : f.ly;
  f.lz = feat == 2 ? v : f.lz;
}

struct LzMem {                       // one workgroup's scratch: vind order as SoA + pairing tables
  float *x, *y, *z;
  int* id;
  int *ml, *mr, *cz, *cr;
};

static __host__ __device__ inline size_t lz_al(size_t b) { return (b + 255) / 256 * 256; }
static __host__ __device__ inline size_t lz_wg_bytes(int n) {
  return 4 * lz_al(4 * (size_t)n) + 2 * lz_al(4 * ((size_t)n / 2 + 64)) + 2 * lz_al(4 * ((size_t)n / 64 + 4));
}

__device__ __forceinline__ LzMem lz_mem(char* p, int n) {
  LzMem m;
  const size_t a = lz_al(4 * (size_t)n), t = lz_al(4 * ((size_t)n / 2 + 64)), q = lz_al(4 * ((size_t)n / 64 + 4));
  m.x = reinterpret_cast<float*>(p);
  m.y = reinterpret_cast<float*>(p + a);
  m.z = reinterpret_cast<float*>(p + 2 * a);
  m.id = reinterpret_cast<int*>(p + 3 * a);
  m.ml = reinterpret_cast<int*>(p + 4 * a);
  m.mr = reinterpret_cast<int*>(p + 4 * a + t);
  m.cz = reinterpret_cast<int*>(p + 4 * a + 2 * t);
  m.cr = reinterpret_cast<int*>(p + 4 * a + 2 * t + q);
  return m;
}

struct LzShared {
  LzFrame F[kLzStack];
  float rf[kLzW][8];
  int ri[kLzW][4];
  int sh[17];
  int tot[2];
  float ld[64];   // lz_leaf's staging (wave 0)
  int lx[64];
  int sp, fail;
  float worst;
  int wb, wc;   // the node range held in LDS (LzWin), wc = 0: none
  int prof;     // DDLO_LAZY_PROF (development): per-phase cycles of block 0's first query
  unsigned long long pt, pa[16];
};
// development profile: thread 0 adds the cycles since the last mark to phase i
__device__ __forceinline__ void lz_mark(LzShared& S, int i) {
  if (S.prof && threadIdx.x == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    S.pa[i] += t - S.pt;
    S.pt = t;
  }
}

// A node of <= kLzL points is split in LDS: when the search enters one, its
// range is copied there and its whole subtree is split in place in LDS (the
// search leaves a subtree only when done with it, so nothing is written back).
constexpr int kLzL = 6144;
struct LzWin {
  float x[kLzL], y[kLzL], z[kLzL];
  int id[kLzL];
  int ml[kLzL / 2 + 64], mr[kLzL / 2 + 64];
  int cz[kLzL / 64 + 4], cr[kLzL / 64 + 4];
};

__device__ __forceinline__ float* lz_axis(const LzMem& m, int f) { return f == 0 ? m.x : (f == 1 ? m.y : m.z); }

// Wave folds with DPP moves (no LDS round trip per step): quad xor 1 / 2,
// half-row and row mirrors, then row_bcast15 / 31 fold the rows into lane
// 63, which is read back.  OP: 0 min, 1 max, 2 integer sum.
template <int OP>
__device__ __forceinline__ int lz_dpp_step(int x, int c) {
  int r;
  switch (c) {
    case 0: r = __builtin_amdgcn_update_dpp(x, x, 0xb1, 0xf, 0xf, false); break;    // quad_perm [1,0,3,2]
    case 1: r = __builtin_amdgcn_update_dpp(x, x, 0x4e, 0xf, 0xf, false); break;    // quad_perm [2,3,0,1]
    case 2: r = __builtin_amdgcn_update_dpp(x, x, 0x141, 0xf, 0xf, false); break;   // row_half_mirror
    case 3: r = __builtin_amdgcn_update_dpp(x, x, 0x140, 0xf, 0xf, false); break;   // row_mirror
    case 4: r = __builtin_amdgcn_update_dpp(OP == 2 ? 0 : x, x, 0x142, 0xa, 0xf, false); break;   // row_bcast15
    default: r = __builtin_amdgcn_update_dpp(OP == 2 ? 0 : x, x, 0x143, 0xc, 0xf, false); break; // row_bcast31
  }
  if (OP == 2) return x + r;
  const float a = __int_as_float(x), b = __int_as_float(r);
  return __float_as_int(OP == 1 ? fmaxf(a, b) : fminf(a, b));
}
template <int OP>
__device__ __forceinline__ int lz_wave_fold(int x) {
#pragma unroll
  for (int c = 0; c < 6; ++c) x = lz_dpp_step<OP>(x, c);
  return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ float lz_wmin(float v) { return __int_as_float(lz_wave_fold<0>(__float_as_int(v))); }
__device__ __forceinline__ float lz_wmax(float v) { return __int_as_float(lz_wave_fold<1>(__float_as_int(v))); }
__device__ __forceinline__ int lz_wsum(int v) { return lz_wave_fold<2>(v); }

// min (v[0..2]) and max (v[3..5]) over the workgroup; every thread gets the result
__device__ __forceinline__ void lz_reduce6(float v[6], LzShared& S) {
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int a = 0; a < 6; ++a) v[a] = a >= 3 ? lz_wmax(v[a]) : lz_wmin(v[a]);
  if (__lane_id() == 0)
#pragma unroll
    for (int a = 0; a < 6; ++a) S.rf[w][a] = v[a];
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    float r = S.rf[0][a];
    for (int i = 1; i < kLzW; ++i) r = a >= 3 ? fmaxf(r, S.rf[i][a]) : fminf(r, S.rf[i][a]);
    v[a] = r;
  }
  __syncthreads();
}

// exclusive prefix of a[0, cnt) in place, returns the total (slot: this
// call site's total word; up to 64 entries one wavefront scans them)
__device__ __forceinline__ int lz_scan(int* a, int cnt, LzShared& S, int slot) {
  if (cnt <= 64) {
    if (threadIdx.x < 64) {
      const int lane = __lane_id();
      const int v = lane < cnt ? a[lane] : 0;
      const int inc = wave_incl_scan(v);
      if (lane < cnt) a[lane] = inc - v;
      if (lane == 63) S.tot[slot] = inc;
    }
    __syncthreads();
    return S.tot[slot];
  }
  const int per = (cnt + kLzT - 1) / kLzT;
  const int b0 = min((int)threadIdx.x * per, cnt), b1 = min(b0 + per, cnt);
  int s = 0;
  for (int i = b0; i < b1; ++i) s += a[i];
  int tot;
  int off = block_excl_scan(s, &tot, S.sh);
  for (int i = b0; i < b1; ++i) {
    const int t = a[i];
    a[i] = off;
    off += t;
  }
  return tot;
}

// The passes below keep kLzU independent loads in flight per thread: one
// workgroup reads its node from L2 at ~60 GB/s only with ~32 KB in flight
// (a load-use loop waits a full L2 round trip per element).
constexpr int kLzU = 8;    // global memory (the LDS window's passes use 2: a short
                           // instruction stream matters more there, each runs once per query, cold in the cache)

// One Hoare pass of the node at base b (count n) as a rank pairing: the r-th
// bad element of the zone [zlo, zhi) (ascending) swaps with the r-th good
// element of [zhi, n) (descending); good = v < cut (pass 1) or v == cut
// (pass 2).  False on an (impossible) count mismatch.
// Every element of A[b, b + n) through f (order-free reductions, global
// memory): 16-byte loads for the body from the first 16-byte boundary (the
// scratch arrays are 256-byte aligned), U of them in flight per thread, the
// head and tail element by element.  Absent elements are NaN (every
// comparison false; fminf / fmaxf ignore them).
template <int U, class F>
__device__ __forceinline__ void lz_vec_each(const float* A, int b, int n, F f) {
  const int h = min(n, (4 - (b & 3)) & 3);
  const int nv = (n - h) >> 2;
  const int t0 = h + 4 * nv;
  if ((int)threadIdx.x < h) f(A[b + threadIdx.x]);
  if ((int)threadIdx.x < n - t0) f(A[b + t0 + threadIdx.x]);
  const float4* V = reinterpret_cast<const float4*>(A + b + h);
  for (int i0 = threadIdx.x; i0 < nv; i0 += kLzT * U) {
    float4 q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * kLzT;
      q[u] = i < nv ? V[i] : make_float4(NAN, NAN, NAN, NAN);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f(q[u].x);
      f(q[u].y);
      f(q[u].z);
      f(q[u].w);
    }
  }
}

template <int kLzU>
__device__ __forceinline__ bool lz_hoare(const LzMem& m, int b, int zlo, int zhi, int n, int feat, float cut, bool pass2, LzShared& S) {
  const int lane = __lane_id(), w = threadIdx.x >> 6;
  const float* V = lz_axis(m, feat) + b;
  const int nz = (zhi - zlo + 63) / 64, nr = (n - zhi + 63) / 64;
  // chunk j < nz: zone chunk j (ascending from zlo); j >= nz: right chunk j - nz (descending from n)
  const int nch = nz + nr;
  auto chunk_flag = [&](int j, float x, bool in) -> bool {
    if (!in) return false;
    const bool good = pass2 ? x == cut : x < cut;
    return j < nz ? !good : good;
  };
  auto chunk_pos = [&](int j) -> int { return j < nz ? zlo + 64 * j + lane : n - 1 - 64 * (j - nz) - lane; };
  auto chunk_in = [&](int j, int i) -> bool { return j < nch && (j < nz ? i < zhi : i >= zhi); };
  for (int j0 = w; j0 < nch; j0 += kLzW * kLzU) {
    float xs[kLzU];
#pragma unroll
    for (int u = 0; u < kLzU; ++u) {
      const int j = j0 + u * kLzW, i = chunk_pos(j);
      xs[u] = chunk_in(j, i) ? V[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kLzU; ++u) {
      const int j = j0 + u * kLzW, i = chunk_pos(j);
      const int c = __popcll(__ballot(chunk_flag(j, xs[u], chunk_in(j, i))));
      if (lane == 0 && j < nch) (j < nz ? m.cz[j] : m.cr[j - nz]) = c;
    }
  }
  __syncthreads();
  lz_mark(S, 3);
  const int mz = lz_scan(m.cz, nz, S, 0);
  const int mr = lz_scan(m.cr, nr, S, 1);
  __syncthreads();
  lz_mark(S, 4);
  if (mz != mr) return false;
  if (mz == 0) return true;
  for (int j0 = w; j0 < nch; j0 += kLzW * kLzU) {
    float xs[kLzU];
    int base[kLzU];
#pragma unroll
    for (int u = 0; u < kLzU; ++u) {
      const int j = j0 + u * kLzW, i = chunk_pos(j);
      xs[u] = chunk_in(j, i) ? V[i] : 0.f;
      base[u] = j < nch ? (j < nz ? m.cz[j] : m.cr[j - nz]) : 0;
    }
#pragma unroll
    for (int u = 0; u < kLzU; ++u) {
      const int j = j0 + u * kLzW, i = chunk_pos(j);
      const bool f = chunk_flag(j, xs[u], chunk_in(j, i));
      const unsigned long long mask = __ballot(f);
      const int slot = base[u] + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
      if (f) (j < nz ? m.ml : m.mr)[slot] = i;   // right chunks: lane order = descending positions
    }
  }
  __syncthreads();
  lz_mark(S, 5);
  constexpr int U = kLzU > 1 ? kLzU / 2 : 1;
  for (int r0 = threadIdx.x; r0 < mz; r0 += kLzT * U) {
    int a[U], c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + u * kLzT;
      a[u] = r < mz ? b + m.ml[r] : -1;
      c[u] = r < mz ? b + m.mr[r] : -1;
    }
    float ax[U], ay[U], az[U], cx[U], cy[U], cz[U];
    int ai[U], ci[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (a[u] >= 0) {
        ax[u] = m.x[a[u]]; ay[u] = m.y[a[u]]; az[u] = m.z[a[u]]; ai[u] = m.id[a[u]];
        cx[u] = m.x[c[u]]; cy[u] = m.y[c[u]]; cz[u] = m.z[c[u]]; ci[u] = m.id[c[u]];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (a[u] >= 0) {
        m.x[a[u]] = cx[u]; m.y[a[u]] = cy[u]; m.z[a[u]] = cz[u]; m.id[a[u]] = ci[u];
        m.x[c[u]] = ax[u]; m.y[c[u]] = ay[u]; m.z[c[u]] = az[u]; m.id[c[u]] = ai[u];
      }
    }
  }
  __syncthreads();
  lz_mark(S, 6);
  return true;
}

// middleSplit_ + planeSplit of the node f (whole workgroup), in place; the
// split position and the children's faces along the cut dimension (divlow =
// the left child's max, divhigh = the right child's min, :1032-1033)
template <int kLzU>
__device__ __forceinline__ bool lz_split(const LzMem& m, int b, const LzFrame& f, int* feat_out, float* cut_out,
                                         int* index_out, float* dlo, float* dhi, LzShared& S) {
  const int n = f.count;
  const float lo[3] = {f.lx, f.ly, f.lz}, hi[3] = {f.hx, f.hy, f.hz};
  // computeMinMax (:965-978) only along the dimensions middleSplit_ measures
  // (span > (1 - EPS) max_span of the passed-down box, the test of nf_cut3)
  const float EPS = 0.00001f;
  float max_span = hi[0] - lo[0];
#pragma unroll
  for (int i = 1; i < 3; ++i) max_span = fmaxf(max_span, hi[i] - lo[i]);
  const bool c0 = hi[0] - lo[0] > (1 - EPS) * max_span, c1 = hi[1] - lo[1] > (1 - EPS) * max_span,
             c2 = hi[2] - lo[2] > (1 - EPS) * max_span;
  float v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  if constexpr (kLzU >= 4) {   // global memory: 16-byte loads, one pass per measured dimension
    if (c0) lz_vec_each<4>(m.x, b, n, [&](float x) { v[0] = fminf(v[0], x); v[3] = fmaxf(v[3], x); });
    if (c1) lz_vec_each<4>(m.y, b, n, [&](float x) { v[1] = fminf(v[1], x); v[4] = fmaxf(v[4], x); });
    if (c2) lz_vec_each<4>(m.z, b, n, [&](float x) { v[2] = fminf(v[2], x); v[5] = fmaxf(v[5], x); });
  } else {
    for (int i0 = threadIdx.x; i0 < n; i0 += kLzT * kLzU) {
      float xs[kLzU], ys[kLzU], zs[kLzU];
#pragma unroll
      for (int u = 0; u < kLzU; ++u) {   // NaN for absent elements: fminf / fmaxf ignore it
        const int i = i0 + u * kLzT;
        const bool in = i < n;
        xs[u] = c0 && in ? m.x[b + i] : NAN;
        ys[u] = c1 && in ? m.y[b + i] : NAN;
        zs[u] = c2 && in ? m.z[b + i] : NAN;
      }
#pragma unroll
      for (int u = 0; u < kLzU; ++u) {
        v[0] = fminf(v[0], xs[u]); v[1] = fminf(v[1], ys[u]); v[2] = fminf(v[2], zs[u]);
        v[3] = fmaxf(v[3], xs[u]); v[4] = fmaxf(v[4], ys[u]); v[5] = fmaxf(v[5], zs[u]);
      }
    }
  }
  lz_reduce6(v, S);
  lz_mark(S, 1);
  const float mn[3] = {v[0], v[1], v[2]}, mx[3] = {v[3], v[4], v[5]};
  int feat;
  float cut;
  nf_cut3(lo, hi, mn, mx, &feat, &cut);
  // lim1 = #(v < cut), lim2 = #(v <= cut), and the max below / min above the cut
  const float* V = lz_axis(m, feat) + b;
  int lt = 0, le = 0;
  float mlt = -INFINITY, mgt = INFINITY;
  auto stat = [&](float x) {   // NaN: every comparison false
    lt += x < cut;
    le += x <= cut;
    if (x < cut) mlt = fmaxf(mlt, x);
    if (x > cut) mgt = fminf(mgt, x);
  };
  if constexpr (kLzU >= 4) {
    lz_vec_each<4>(lz_axis(m, feat), b, n, stat);
  } else {
    for (int i0 = threadIdx.x; i0 < n; i0 += kLzT * kLzU) {
      float xs[kLzU];
#pragma unroll
      for (int u = 0; u < kLzU; ++u) {
        const int i = i0 + u * kLzT;
        xs[u] = i < n ? V[i] : NAN;
      }
#pragma unroll
      for (int u = 0; u < kLzU; ++u) stat(xs[u]);
    }
  }
  lt = lz_wsum(lt);
  le = lz_wsum(le);
  mlt = lz_wmax(mlt);
  mgt = lz_wmin(mgt);
  const int w = threadIdx.x >> 6;
  if (__lane_id() == 0) {
    S.ri[w][0] = lt;
    S.ri[w][1] = le;
    S.rf[w][0] = mlt;
    S.rf[w][1] = mgt;
  }
  __syncthreads();
  int lim1 = 0, lim2 = 0;
  float max_lt = -INFINITY, min_gt = INFINITY;
  for (int i = 0; i < kLzW; ++i) {
    lim1 += S.ri[i][0];
    lim2 += S.ri[i][1];
    max_lt = fmaxf(max_lt, S.rf[i][0]);
    min_gt = fminf(min_gt, S.rf[i][1]);
  }
  __syncthreads();
  lz_mark(S, 2);
  bool ok = lz_hoare<kLzU>(m, b, 0, lim1, n, feat, cut, false, S);
  if (ok && lim2 > lim1) ok = lz_hoare<kLzU>(m, b, lim1, lim2, n, feat, cut, true, S);   // pass 2 (:1128-1142)
  const int index = nf_index(n, lim1, lim2);
  *feat_out = feat;
  *cut_out = cut;
  *index_out = index;
  *dlo = index > lim1 ? cut : max_lt;
  *dhi = index < lim2 ? cut : min_gt;
  return ok;
}

// KNNResultSet::addPoint over one leaf (wave 0): candidates are the points
// below the worst distance read at the leaf (:1503-1516), inserted in leaf
// order; lane j < k holds the j-th result (kd, kx), count = results so far.
// The serial insertions keep the first k of the stable order (distance, then
// insertion time) of the kept list followed by the candidates in leaf order,
// so every item's final slot is a count: a kept entry moves down by the
// candidates strictly closer, a candidate lands after the entries and earlier
// candidates no farther and the later candidates strictly closer.
// (ld, lx: 64-entry LDS staging of wave 0.)
template <class LOAD>
__device__ __forceinline__ void lz_leaf(LOAD load, int b0, int b1, float qx, float qy, float qz, float worst, int k,
                                        float& kd, int& kx, int& count, float* ld, int* lx) {
  const int lane = __lane_id();
  const int m = b1 - b0;   // <= kNfLeafMax (100): two rounds of 64
  float r[2] = {FLT_MAX, FLT_MAX};
  int ip[2] = {-1, -1};
  bool cd[2] = {false, false};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = 64 * h + lane;
    if (i < m) {
      float px, py, pz;
      load(b0 + i, px, py, pz, ip[h]);
      float rr = 0.f;
      float diff = qx - px;
      rr += diff * diff;
      diff = qy - py;
      rr += diff * diff;
      diff = qz - pz;
      rr += diff * diff;
      r[h] = rr;
      cd[h] = rr < worst;
    }
  }
  const unsigned long long cm[2] = {__ballot(cd[0]), __ballot(cd[1])};
  const int nc = __popcll(cm[0]) + __popcll(cm[1]);
  if (nc == 0) return;
  // candidate ranks (own position p = 64 h + lane) and the entries' shifts
  int rk[2] = {0, 0};
  int sh_e = 0;   // candidates strictly closer than this lane's entry
  for (int j = 0; j < count; ++j) {   // (uniform lanes: v_readlane, not an LDS permute per step)
    const float e = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(kd), j));
    rk[0] += e <= r[0];
    rk[1] += e <= r[1];
  }
#pragma unroll
  for (int h2 = 0; h2 < 2; ++h2) {
    unsigned long long mk = cm[h2];
    while (mk) {
      const int bl = __ffsll((long long)mk) - 1;
      mk &= mk - 1;
      const float rc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r[h2]), bl));
      const int pc = 64 * h2 + bl;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int p = 64 * h + lane;
        rk[h] += pc < p ? (rc <= r[h]) : (pc > p ? (rc < r[h]) : 0);
      }
      sh_e += rc < kd;
    }
  }
  if (lane < count && lane + sh_e < k) {
    ld[lane + sh_e] = kd;
    lx[lane + sh_e] = kx;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h)
    if (cd[h] && rk[h] < k) {
      ld[rk[h]] = r[h];
      lx[rk[h]] = ip[h];
    }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  count = min(k, count + nc);
  if (lane < count) {
    kd = ld[lane];
    kx = lx[lane];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();   // the staging is read before the next leaf rewrites it
}

// COV: queries are the cloud's own points (sorted positions in the list),
// the result is their covariance; else rows of q, the result (index, distance).
// t: the cloud's partial tree (the top levels, stubs below, nftree_build
// partial_levels): the search walks the built nodes as nf_search does and,
// entering a stub, copies its range (vind order) into its private scratch and
// splits the stub's subtree lazily from there.
template <bool COV>
__global__ __launch_bounds__(kLzT) void k_nf_lazy(NfTreeDev t, CloudDev c, const float4* __restrict__ q, TieList ties,
                                                  int k, int method, double* __restrict__ cov6, int* __restrict__ out_idx,
                                                  float* __restrict__ out_d, char* __restrict__ scr, size_t wg_bytes,
                                                  const int* __restrict__ status, int* __restrict__ err, int prof) {
  __shared__ LzShared S;
  __shared__ LzWin Wn;
  const int n = c.n;
  const int lane = __lane_id();
  const int nc = *ties.count;
  const int nl = min(nc, ties.cap);
  if (nc > ties.cap && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, 8);
  if (*status) {   // the partial build failed: report, keep the Morton-order answers
    if (blockIdx.x == 0 && threadIdx.x == 0 && nl > 0) atomicOr(err, 2 | (*status << 8));
    return;
  }
  const LzMem gm = lz_mem(scr + (size_t)blockIdx.x * wg_bytes, n);
  LzMem wm;
  wm.x = Wn.x; wm.y = Wn.y; wm.z = Wn.z; wm.id = Wn.id;
  wm.ml = Wn.ml; wm.mr = Wn.mr; wm.cz = Wn.cz; wm.cr = Wn.cr;
  for (int li = blockIdx.x; li < nl; li += gridDim.x) {
    const int qi = ties.list[li];
    const float4 qp = COV ? c.pts[qi] : q[qi];
    // computeInitialDistances (:1145-1164) against root_bbox
    const float4 rl = t.box[0], rh = t.box[1];
    float d0 = 0.f, d1 = 0.f, d2 = 0.f, distsq = 0.f;
    if (qp.x < rl.x) { d0 = (qp.x - rl.x) * (qp.x - rl.x); distsq += d0; }
    if (qp.x > rh.x) { d0 = (qp.x - rh.x) * (qp.x - rh.x); distsq += d0; }
    if (qp.y < rl.y) { d1 = (qp.y - rl.y) * (qp.y - rl.y); distsq += d1; }
    if (qp.y > rh.y) { d1 = (qp.y - rh.y) * (qp.y - rh.y); distsq += d1; }
    if (qp.z < rl.z) { d2 = (qp.z - rl.z) * (qp.z - rl.z); distsq += d2; }
    if (qp.z > rh.z) { d2 = (qp.z - rh.z) * (qp.z - rh.z); distsq += d2; }
    if (threadIdx.x == 0) {
      S.prof = prof && li == 0;
      S.pt = __builtin_amdgcn_s_memtime();
      for (int e = 0; e < 16; ++e) S.pa[e] = 0;
      LzFrame r;
      r.node = 0;
      r.begin = 0;
      r.count = n;
      r.state = 0;
      r.feat = 0;
      r.fm = distsq;
      r.fd = 0.f;
      S.F[0] = r;
      S.sp = 1;
      S.fail = 0;
      S.worst = FLT_MAX;
      S.wb = 0;
      S.wc = 0;
    }
    float kd = FLT_MAX;   // wave 0: lane j's result slot (KNNResultSet)
    int kx = -1, count = 0;
    __syncthreads();
    for (;;) {
      const int sp = S.sp;
      if (sp == 0 || S.fail) break;
      LzFrame f = S.F[sp - 1];
      const float worst = S.worst;
      int wb = S.wb, wc = S.wc;
      __syncthreads();   // every thread has the frame before thread 0 rewrites it
      // a built node: its record.  A stub (feat -2) turns into a lazily split
      // range: its points (vind order) go to the private scratch first.
      int bfeat = -3;
      NfNode nd;
      if (f.node >= 0) {
        nd = t.nodes[f.node];
        bfeat = nd.feat;
        if (bfeat == -2) {
          f.begin = nd.c1;
          f.count = nd.c2 - nd.c1;
          const float4 lo = t.sbox[2 * f.node], hi = t.sbox[2 * f.node + 1];
          f.lx = lo.x; f.ly = lo.y; f.lz = lo.z;
          f.hx = hi.x; f.hy = hi.y; f.hz = hi.z;
          f.node = -1;
          // a stub that fits LDS goes straight into the window, a larger one
          // into the private scratch (at its own positions)
          const bool to_win = f.count <= kLzL;
          for (int j0 = threadIdx.x; j0 < f.count; j0 += kLzT * 4) {
            float4 ps[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) ps[u] = t.vpts[f.begin + min(j0 + u * kLzT, f.count - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int jl = j0 + u * kLzT, j = f.begin + jl;
              if (jl < f.count) {
                if (to_win) {
                  Wn.x[jl] = ps[u].x; Wn.y[jl] = ps[u].y; Wn.z[jl] = ps[u].z; Wn.id[jl] = __float_as_int(ps[u].w);
                } else {
                  gm.x[j] = ps[u].x; gm.y[j] = ps[u].y; gm.z[j] = ps[u].z; gm.id[j] = __float_as_int(ps[u].w);
                }
              }
            }
          }
          if (threadIdx.x == 0) {
            S.F[sp - 1] = f;
            if (to_win) {
              S.wb = f.begin;
              S.wc = f.count;
            }
            if (S.prof) S.pa[14] += 1;
          }
          __syncthreads();
          lz_mark(S, 0);
          continue;
        }
      }
      if (f.node >= 0 && bfeat == -1) {   // a built leaf: its vind range in the tree's points (:1503-1516)
        if (threadIdx.x < 64) {
          lz_leaf([&](int i, float& px, float& py, float& pz, int& ip) {
                    const float4 p = t.vpts[i];
                    px = p.x; py = p.y; pz = p.z; ip = __float_as_int(p.w);
                  }, nd.c1, nd.c2, qp.x, qp.y, qp.z, worst, k, kd, kx, count, S.ld, S.lx);
          const float wk = __shfl(kd, k - 1);
          if (lane == 0) {
            S.worst = count < k ? FLT_MAX : wk;
            S.sp = sp - 1;
          }
        }
        __syncthreads();
        lz_mark(S, 8);
        continue;
      }
      if (f.node >= 0) {   // a built inner node: searchLevel with its record (:1518-1566)
        const int feat = bfeat;
        const float val = feat == 0 ? qp.x : (feat == 1 ? qp.y : qp.z);
        const float diff1 = val - nd.divlow, diff2 = val - nd.divhigh;
        const bool first1 = (diff1 + diff2) < 0;
        if (f.state == 0) {
          if (threadIdx.x == 0) {
            if (sp >= kLzStack) {
              S.fail = 1;
            } else {
              S.F[sp - 1].state = 1;
              LzFrame ch = f;
              ch.node = first1 ? nd.c1 : nd.c2;
              ch.state = 0;
              S.F[sp] = ch;
              S.sp = sp + 1;
            }
          }
          __syncthreads();
          continue;
        }
        if (f.state == 1) {
          const float cut_dist = first1 ? (val - nd.divhigh) * (val - nd.divhigh) : (val - nd.divlow) * (val - nd.divlow);
          const float dst = feat == 0 ? d0 : (feat == 1 ? d1 : d2);
          const float mind = f.fm + cut_dist - dst;
          if (feat == 0) d0 = cut_dist;
          else if (feat == 1) d1 = cut_dist;
          else d2 = cut_dist;
          if (threadIdx.x == 0) {
            S.F[sp - 1].fd = dst;
            S.F[sp - 1].state = 2;
            if (mind * 1.0f <= worst) {
              if (sp >= kLzStack) {
                S.fail = 1;
              } else {
                LzFrame ch = f;
                ch.node = first1 ? nd.c2 : nd.c1;
                ch.state = 0;
                ch.fm = mind;
                S.F[sp] = ch;
                S.sp = sp + 1;
              }
            }
          }
          __syncthreads();
          continue;
        }
        if (feat == 0) d0 = f.fd;   // state 2
        else if (feat == 1) d1 = f.fd;
        else d2 = f.fd;
        if (threadIdx.x == 0) S.sp = sp - 1;
        __syncthreads();
        continue;
      }
      // a lazily split range
      bool inw = wc > 0 && f.begin >= wb && f.begin + f.count <= wb + wc;
      if (!inw && f.state == 0 && f.count > kNfLeafMax && f.count <= kLzL) {   // enter a subtree that fits LDS
        for (int j0 = threadIdx.x; j0 < f.count; j0 += kLzT * 4) {
          float xs[4], ys[4], zs[4];
          int is[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int j = min(j0 + u * kLzT, f.count - 1) + f.begin;
            xs[u] = gm.x[j]; ys[u] = gm.y[j]; zs[u] = gm.z[j]; is[u] = gm.id[j];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int j = j0 + u * kLzT;
            if (j < f.count) {
              Wn.x[j] = xs[u]; Wn.y[j] = ys[u]; Wn.z[j] = zs[u]; Wn.id[j] = is[u];
            }
          }
        }
        wb = f.begin;
        wc = f.count;
        inw = true;
        if (threadIdx.x == 0) {
          S.wb = wb;
          S.wc = wc;
          if (S.prof) S.pa[13] += 1;
        }
        __syncthreads();
        lz_mark(S, 7);
      }
      // the node's storage: the LDS window (offset wb) or the private scratch;
      // two inlined copies of each access path, so that the window's get LDS
      // instructions (a pointer select between the two would make both flat)
      if (f.count <= kNfLeafMax) {   // leaf: candidates below the worst distance read at the leaf (:1503-1516)
        if (threadIdx.x < 64) {
          if (inw)
            lz_leaf([&](int i, float& px, float& py, float& pz, int& ip) {
                      px = Wn.x[i - wb]; py = Wn.y[i - wb]; pz = Wn.z[i - wb]; ip = Wn.id[i - wb];
                    }, f.begin, f.begin + f.count, qp.x, qp.y, qp.z, worst, k, kd, kx, count, S.ld, S.lx);
          else
            lz_leaf([&](int i, float& px, float& py, float& pz, int& ip) {
                      px = gm.x[i]; py = gm.y[i]; pz = gm.z[i]; ip = gm.id[i];
                    }, f.begin, f.begin + f.count, qp.x, qp.y, qp.z, worst, k, kd, kx, count, S.ld, S.lx);
          const float wk = __shfl(kd, k - 1);
          if (lane == 0) {
            S.worst = count < k ? FLT_MAX : wk;
            S.sp = sp - 1;
            if (S.prof) S.pa[12] += 1;
          }
        }
        __syncthreads();
        lz_mark(S, 8);
        continue;
      }
      if (f.state == 0) {   // first visit: split the node (divideTree's recursion step)
        int feat, index;
        float cut, dlo, dhi;
        const bool ok = inw ? lz_split<2>(wm, f.begin - wb, f, &feat, &cut, &index, &dlo, &dhi, S)
                            : lz_split<kLzU>(gm, f.begin, f, &feat, &cut, &index, &dlo, &dhi, S);
        if (S.prof && threadIdx.x == 0) {
          S.pa[10] += 1;
          S.pa[11] += f.count;
        }
        const float val = feat == 0 ? qp.x : (feat == 1 ? qp.y : qp.z);
        const bool first1 = ((val - dlo) + (val - dhi)) < 0;   // searchLevel (:1525-1540)
        if (threadIdx.x == 0) {
          if (!ok || sp >= kLzStack) {
            S.fail = ok ? 1 : 16;
          } else {
            LzFrame& F = S.F[sp - 1];
            F.state = 1;
            F.feat = feat;
            F.cut = cut;
            F.index = index;
            F.divlow = dlo;
            F.divhigh = dhi;
            LzFrame ch = f;   // left_bbox / right_bbox (:1024-1030)
            ch.state = 0;
            if (first1) {
              ch.count = index;
              lz_set_hi(ch, feat, cut);
            } else {
              ch.begin = f.begin + index;
              ch.count = f.count - index;
              lz_set_lo(ch, feat, cut);
            }
            S.F[sp] = ch;
            S.sp = sp + 1;
          }
        }
        __syncthreads();
        continue;
      }
      const int feat = f.feat;
      const float val = feat == 0 ? qp.x : (feat == 1 ? qp.y : qp.z);
      const float diff1 = val - f.divlow, diff2 = val - f.divhigh;
      const bool first1 = (diff1 + diff2) < 0;
      if (f.state == 1) {   // the other child, if its box is within the worst distance (:1548-1560)
        const float cut_dist = first1 ? (val - f.divhigh) * (val - f.divhigh) : (val - f.divlow) * (val - f.divlow);
        const float dst = feat == 0 ? d0 : (feat == 1 ? d1 : d2);
        const float mind = f.fm + cut_dist - dst;
        if (feat == 0) d0 = cut_dist;
        else if (feat == 1) d1 = cut_dist;
        else d2 = cut_dist;
        if (threadIdx.x == 0) {
          S.F[sp - 1].fd = dst;
          S.F[sp - 1].state = 2;
          if (mind * 1.0f <= worst) {
            if (sp >= kLzStack) {
              S.fail = 1;
            } else {
              LzFrame ch = f;
              ch.state = 0;
              ch.fm = mind;
              if (first1) {   // the right child
                ch.begin = f.begin + f.index;
                ch.count = f.count - f.index;
                lz_set_lo(ch, feat, f.cut);
              } else {
                ch.count = f.index;
                lz_set_hi(ch, feat, f.cut);
              }
              S.F[sp] = ch;
              S.sp = sp + 1;
            }
          }
        }
        __syncthreads();
        continue;
      }
      if (feat == 0) d0 = f.fd;   // state 2: dists[idx] = dst, return
      else if (feat == 1) d1 = f.fd;
      else d2 = f.fd;
      if (threadIdx.x == 0) S.sp = sp - 1;
      __syncthreads();
    }
    lz_mark(S, 9);
    if (S.prof && threadIdx.x == 0)
      printf("[lazy] n %d cycles: stubcopy %llu minmax %llu stats %llu hcount %llu scan %llu scatter %llu swap %llu "
             "window %llu leaf %llu rest %llu | splits %llu split_pts %llu leaves %llu windows %llu stubs %llu\n", n,
             S.pa[0], S.pa[1], S.pa[2], S.pa[3], S.pa[4], S.pa[5], S.pa[6], S.pa[7], S.pa[8], S.pa[9], S.pa[10],
             S.pa[11], S.pa[12], S.pa[13], S.pa[14]);
    const int fail = S.fail;
    if (threadIdx.x < 64) {
      if (fail || count < k) {
        if (lane == 0) atomicOr(err, fail ? fail : 4);
      } else if (COV) {
        nf_cov_wave(c, kx, k, method, cov6 + 6 * (size_t)qi);
      } else if (lane < k) {
        out_idx[(size_t)qi * k + lane] = kx;
        out_d[(size_t)qi * k + lane] = kd;
      }
    }
    __syncthreads();
  }
}

// vind starts as the identity (init_vind): the cloud's points in original order
__global__ __launch_bounds__(256) void k_nf_unsort(const NfBuild* __restrict__ bp) {
  if (nf_gated_off(bp)) return;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= bp->n) return;
  const float4 p = bp->sorted[s];
  bp->vpts[__float_as_int(p.w)] = p;
}

// Partial build: after the top Lmax levels, every node the final map listed
// (all of level Lmax's children, and the small nodes of the levels above)
// becomes a stub: feat = -2, its vind range, the box divideTree passes it,
// and its parent's divlow / divhigh from its points' min / max.
__global__ __launch_bounds__(256) void k_nf_stub(const NfBuild* __restrict__ bp) {
  if (nf_gated_off(bp)) return;
  const NfBuild& b = *bp;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b.ctl->nsmall) return;
  const NfTask e = b.small[i];
  if (e.node < 0 || e.node >= b.big_ids) {
    atomicOr(&b.ctl->err, 1);
    return;
  }
  NfNode* nd = b.nodes;
  nd[e.node].c1 = e.begin;
  nd[e.node].c2 = e.begin + e.count;
  nd[e.node].feat = e.count <= kNfLeafMax ? -1 : -2;   // a node of <= leaf_max_size points is a leaf (:992)
  b.sbox[2 * e.node] = make_float4(e.lo[0], e.lo[1], e.lo[2], 0.f);
  b.sbox[2 * e.node + 1] = make_float4(e.hi[0], e.hi[1], e.hi[2], 0.f);
  const float mn[3] = {o2f(e.mm[0]), o2f(e.mm[1]), o2f(e.mm[2])};
  const float mx[3] = {o2f(e.mm[3]), o2f(e.mm[4]), o2f(e.mm[5])};
  nf_set_div(nd, e.node, mn, mx);
}

// diagnostics / tests: the tree as nanoflann would hold it (status[1] = nodes)
__global__ void k_nf_export(NfTreeDev t, const int* __restrict__ status, int cap, int* __restrict__ vind,
                            int* __restrict__ nodes_out, float* __restrict__ f_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < t.n) vind[i] = __float_as_int(t.vpts[i].w);
  const int nn = min(status[1], cap);
  if (i < nn) {
    const NfNode nd = t.nodes[i];
    nodes_out[4 * i + 0] = nd.c1;
    nodes_out[4 * i + 1] = nd.c2;
    nodes_out[4 * i + 2] = nd.feat;
    nodes_out[4 * i + 3] = nd.parent;
    f_out[2 * i + 0] = nd.divlow;
    f_out[2 * i + 1] = nd.divhigh;
  }
}

// ---------------------------------------------------------------------------
// host side
static inline int cdivl(long a, long b) { return (int)((a + b - 1) / b); }

NfSizes nf_sizes(int n) {
  NfSizes z;
  z.Lmax = 0;
  if (n > kNfT) {   // levels until halving nodes are <= kNfT, plus margin: middleSplit_ cuts the box, not
    int l = 0;      // the points, so clustered clouds split unevenly (a node still larger after the last
    while ((long)kNfT << l < n) ++l;   // level is split by the small kernel in global memory, slowly)
    z.Lmax = std::min(l + kNfLevelMargin, kNfMaxLevels);
  }
  z.max_task = n / kNfT + 2;
  z.max_pend = 2 * z.max_task;
  z.max_small = 2 * (z.Lmax + 1) * z.max_task + 2;
  z.max_chunks = cdivl(n, kNfCH) + z.max_task;
  z.big_ids = 2 * (z.Lmax + 1) * z.max_task + 2;   // the root and two children per big task
  return z;
}


__global__ void k_nf_set_desc(NfBuild b, NfBuild* __restrict__ db) {
  if (threadIdx.x == 0) *db = b;
}
void launch_nf_set_desc(hipStream_t s, const NfBuild& b, NfBuild* db) { k_nf_set_desc<<<1, 64, 0, s>>>(b, db); }

// hb: the descriptor on the host (grid sizes); db: the same in device memory
// (the kernels' argument, so that a captured graph serves any cloud of the
// size bucket: only the descriptor is rewritten).  stop >= 0: that many big
// levels, nothing after (diagnostics).
void launch_nf_build(hipStream_t s, const NfBuild& hb, const NfBuild* db, int stop) {
  k_nf_unsort<<<cdivl(hb.nbucket, 256), 256, 0, s>>>(db);
  k_nf_init<<<1, 64, 0, s>>>(db);
  const int G = std::max(1, hb.max_chunks);
  for (int L = 0; L < hb.Lmax; ++L) {
    if (stop >= 0 && L >= stop) return;
    k_nf_count<<<G, kNfBT, 0, s>>>(db, L);   // the level's map + its counts
    k_nf_pass<1, true><<<G, kNfBT, 0, s>>>(db, L);
    k_nf_pass<1, false><<<G, kNfBT, 0, s>>>(db, L);
    k_nf_pass<2, true><<<G, kNfBT, 0, s>>>(db, L);
    k_nf_pass<2, false><<<G, kNfBT, 0, s>>>(db, L);
  }
  k_nf_map<<<1, 1024, 0, s>>>(db, hb.Lmax);
  if (hb.sbox) {   // partial: the rest is split lazily by the searches that need it
    k_nf_stub<<<cdivl(hb.max_small, 256), 256, 0, s>>>(db);
    return;
  }
  k_nf_sub<<<hb.max_small, 64 * kNfSubWaves, 0, s>>>(db);
  k_nf_small_global<<<hb.max_small, 64, 0, s>>>(db);
}

void launch_nf_export(hipStream_t s, const NfTreeDev& t, const int* status, int cap, int* vind, int* nodes, float* f) {
  k_nf_export<<<cdivl(std::max(t.n, cap), 256), 256, 0, s>>>(t, status, cap, vind, nodes, f);
}

bool launch_nf_resolve_cov(hipStream_t s, const NfTreeDev& t, const CloudDev& c, TieList ties, int k, int method,
                           double* cov6, const int* status, int* err) {
  if (k > 64) return false;
  k_nf_resolve_cov<<<256, 64 * kNfResolveWaves, 0, s>>>(t, c, ties, k, method, cov6, status, err);
  return true;
}

size_t nf_lazy_bytes(int n, int wgs) { return (size_t)wgs * lz_wg_bytes(n); }

bool launch_nf_lazy(hipStream_t s, const NfTreeDev& t, const CloudDev& c, const float4* q, TieList ties, int k,
                    int method, double* cov6, int* out_idx, float* out_d, void* scratch, int wgs, const int* status,
                    int* err) {
  if (k > 64 || wgs < 1 || !t.partial) return false;
  static const int prof = dev_getenv("DDLO_LAZY_PROF") != nullptr;   // development: per-phase cycles (printf)
  char* wg = static_cast<char*>(scratch);
  if (cov6)
    k_nf_lazy<true><<<wgs, kLzT, 0, s>>>(t, c, q, ties, k, method, cov6, out_idx, out_d, wg, lz_wg_bytes(c.n), status,
                                         err, prof);
  else
    k_nf_lazy<false><<<wgs, kLzT, 0, s>>>(t, c, q, ties, k, method, cov6, out_idx, out_d, wg, lz_wg_bytes(c.n), status,
                                          err, prof);
  return true;
}

bool launch_nf_resolve_knn(hipStream_t s, const NfTreeDev& t, const float4* q, TieList ties, int k, int* out_idx,
                           float* out_d, const int* status, int* err) {
  if (k > 64) return false;
  k_nf_resolve_knn<<<256, 64 * kNfResolveWaves, 0, s>>>(t, q, ties, k, out_idx, out_d, status, err);
  return true;
}

}  // namespace ddlo
