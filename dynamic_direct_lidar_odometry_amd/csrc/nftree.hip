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

#include "cov_math.hpp"
#include "gicp_types.hpp"
#include "launch.hpp"
#include "nftree.hpp"

namespace ddlo {

namespace {

constexpr int kNfT = 4096;     // nodes up to this size are split by one wavefront in LDS
constexpr int kNfCH = 2048;    // points per block in the big-level passes
constexpr int kNfBT = 256;     // threads per big-level block (8 points each)
constexpr int kNfPer = kNfCH / kNfBT;

__device__ __forceinline__ unsigned f2o(float f) {   // order-preserving float -> uint
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(unsigned o) {
  const unsigned u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return __uint_as_float(u);
}
__device__ __forceinline__ float coord(const float4& p, int f) { return f == 0 ? p.x : (f == 1 ? p.y : p.z); }
// Coordinate f of a point in memory: one load at a computed address.  (The
// select form on a memory operand was lowered by ROCm 7.2's hipcc into a
// per-lane branch that left the f == 2 lanes loading from an unset address:
// wrong z splits in LDS, a fault in global memory.)
__device__ __forceinline__ float coord_at(const float4* p, int f) { return reinterpret_cast<const float*>(p)[f]; }

// middleSplit_ (:1045-1087): cut dimension and value from the passed-down
// box and the node's point min / max (computeMinMax, :965-978)
__device__ __forceinline__ void nf_cut(const NfTask& t, int* feat, float* cut) {
  const float EPS = 0.00001f;
  float max_span = t.hi[0] - t.lo[0];
  for (int i = 1; i < 3; ++i) {
    const float span = t.hi[i] - t.lo[i];
    if (span > max_span) max_span = span;
  }
  float max_spread = -1;
  int cf = 0;
  for (int i = 0; i < 3; ++i) {
    const float span = t.hi[i] - t.lo[i];
    if (span > (1 - EPS) * max_span) {
      const float spread = o2f(t.mm[3 + i]) - o2f(t.mm[i]);
      if (spread > max_spread) {
        cf = i;
        max_spread = spread;
      }
    }
  }
  const float split_val = (t.lo[cf] + t.hi[cf]) / 2;
  const float mn = o2f(t.mm[cf]), mx = o2f(t.mm[3 + cf]);
  float cv;
  if (split_val < mn) cv = mn;
  else if (split_val > mx) cv = mx;
  else cv = split_val;
  *feat = cf;
  *cut = cv;
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
__device__ int block_excl_scan(int v, int* total, int* sh /* >= 17 ints */) {
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
__device__ int block_sum(int v, int* sh) {
  int tot;
  (void)block_excl_scan(v, &tot, sh);
  return tot;
}

struct TaskView {   // a big-level block's task and chunk
  int t, c, blk;
  NfTask tk;
};
__device__ __forceinline__ bool task_of_block(const NfBuild& b, int L, TaskView* v) {
  const int par = L & 1;
  const int blk = blockIdx.x;
  if (blk >= b.ctl->nchunks[par]) return false;
  v->blk = blk;
  v->t = b.chunk_task[par * b.max_chunks + blk];
  v->tk = b.tasks[(size_t)L * b.max_task + v->t];
  v->c = blk - v->tk.chunk0;
  return true;
}

// sums of a per-chunk count over the task's chunks: all of them, and those before blk
__device__ void task_chunk_sums(const int* cnt, const NfTask& tk, int blk, int* total, int* before, int* sh) {
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
__global__ void k_nf_init(NfBuild b) {
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
  }
}

// Level L's task list from the children its parent level produced (pend[L]):
// nodes > kNfT points become big tasks (their chunks listed), the others
// small tasks; the final call lists every remaining node as small.
__global__ __launch_bounds__(1024) void k_nf_map(NfBuild b, int L) {
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
    ctl->nsmall = min(s_small0 + s_small, b.max_small);
    ctl->nchunks[L & 1] = final ? 0 : min(s_ch, b.max_chunks);
  }
  __threadfence_block();
  __syncthreads();
  if (final) return;
  // chunk -> task map (tasks are in chunk0 order)
  const int nchunks = min(s_ch, b.max_chunks);
  int* cmap = b.chunk_task + (L & 1) * b.max_chunks;
  for (int c = threadIdx.x; c < nchunks; c += blockDim.x) {
    int lo = 0, hi = nbig - 1;
    while (lo < hi) {   // last task with chunk0 <= c
      const int mid = (lo + hi + 1) >> 1;
      if (T[mid].chunk0 <= c) lo = mid;
      else hi = mid - 1;
    }
    cmap[c] = lo;
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

// middleSplit_'s cut per task; #{v < cut} and #{v <= cut} per chunk
__global__ __launch_bounds__(kNfBT) void k_nf_count(NfBuild b, int L) {
  __shared__ int sh[17];
  TaskView v;
  if (!task_of_block(b, L, &v)) return;
  int feat;
  float cut;
  nf_cut(v.tk, &feat, &cut);
  const int p0 = v.c * kNfCH, p1 = min(p0 + kNfCH, v.tk.count);
  int a = 0, ae = 0;
  for (int p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    const float x = coord_at(&b.vpts[v.tk.begin + p], feat);
    a += x < cut;
    ae += x <= cut;
  }
  a = block_sum(a, sh);
  ae = block_sum(ae, sh);
  if (threadIdx.x == 0) {
    b.cA[v.blk] = a;
    b.cAE[v.blk] = ae;
    if (v.c == 0) {
      NfTask* T = b.tasks + (size_t)L * b.max_task;
      T[v.t].feat = feat;
      T[v.t].cut = cut;
    }
  }
}

// Hoare pass as rank pairing.  PASS 1: over [0, n), "good" = v < cut,
// boundary lo = lim1.  PASS 2: over [lim1, n), "good" = v == cut (<= cut
// there), boundary lim2.  TABLE: write each misplaced element into its rank
// slot; else (APPLY) overwrite each misplaced position with its partner.
template <int PASS, bool TABLE>
__global__ __launch_bounds__(kNfBT) void k_nf_pass(NfBuild b, int L) {
  __shared__ int sh[17];
  TaskView v;
  if (!task_of_block(b, L, &v)) return;
  const NfTask& tk = v.tk;
  const int feat = tk.feat;
  const float cut = tk.cut;
  int lim1, before1, lim2, before2;
  task_chunk_sums(b.cA, tk, v.blk, &lim1, &before1, sh);
  int before = before1;
  int zlo = 0, zhi = lim1;   // the "good" zone [zlo, zhi) of this pass
  if (PASS == 2) {
    task_chunk_sums(b.cAE, tk, v.blk, &lim2, &before2, sh);
    task_chunk_sums(b.cE2, tk, v.blk, &before2, &before, sh);   // E after pass 1: none before lim1
    zlo = lim1;
    zhi = lim2;
  }
  const int ngood = zhi - zlo;
  const int p0 = v.c * kNfCH + threadIdx.x * kNfPer;
  float4 e[kNfPer];
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < kNfPer; ++j) {
    const int p = p0 + j;
    if (p < tk.count) {
      e[j] = b.vpts[tk.begin + p];
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
    if (p >= tk.count) break;
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
  if (!TABLE && PASS == 2) {
    // the split index, the children's point min / max, and (one thread per
    // task) the node record and the children's pending entries
    const int index = nf_index(tk.count, lim1, lim2);
    float m[2][6];
    for (int s = 0; s < 2; ++s)
      for (int a = 0; a < 3; ++a) {
        m[s][a] = INFINITY;
        m[s][3 + a] = -INFINITY;
      }
#pragma unroll
    for (int j = 0; j < kNfPer; ++j) {
      const int p = p0 + j;
      if (p >= tk.count) break;
      const int s = p < index ? 0 : 1;
      const float cc[3] = {e[j].x, e[j].y, e[j].z};
      for (int a = 0; a < 3; ++a) {
        if (s == 0) {
          m[0][a] = fminf(m[0][a], cc[a]);
          m[0][3 + a] = fmaxf(m[0][3 + a], cc[a]);
        } else {
          m[1][a] = fminf(m[1][a], cc[a]);
          m[1][3 + a] = fmaxf(m[1][3 + a], cc[a]);
        }
      }
    }
    NfTask* C = b.pend + (size_t)(L + 1) * b.max_pend;
    for (int s = 0; s < 2; ++s)
      for (int a = 0; a < 6; ++a) {
        float x = m[s][a];
        for (int d = 32; d >= 1; d >>= 1) {
          const float o = __shfl_xor(x, d);
          x = a < 3 ? fminf(x, o) : fmaxf(x, o);
        }
        if (__lane_id() == 0 && x == x && !isinf(x)) {
          unsigned* dst = &C[2 * v.t + s].mm[a];
          if (a < 3) atomicMin(dst, f2o(x));
          else atomicMax(dst, f2o(x));
        }
      }
    if (v.c == 0 && threadIdx.x == 0) {
      NfCtl* ctl = b.ctl;
      const int c1 = atomicAdd(&ctl->nnodes, 2);
      if (c1 + 2 > b.cap) {
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

// One wavefront per small node: its whole subtree, depth first, in LDS.  A
// node the big levels left larger than kNfT (a very unbalanced cloud) is
// split the same way in global memory (rank lists in the pairing tables).
struct SmallLds {
  float4 P[kNfT];
  unsigned short ML[kNfT / 2], MR[kNfT / 2];
  int sb[kNfStack], sc[kNfStack], sn[kNfStack];
  float slo[3][kNfStack], shi[3][kNfStack];
};

__device__ __forceinline__ float wred(float x, bool mx) {
  for (int d = 32; d >= 1; d >>= 1) {
    const float o = __shfl_xor(x, d);
    x = mx ? fmaxf(x, o) : fminf(x, o);
  }
  return x;
}

// one Hoare pass over [zlo0, n) of the node at P (good = v < cut, or
// v == cut for pass 2), boundary zhi: pair the r-th bad element of
// [zlo0, zhi) with the r-th good element of [zhi, n) from the end
template <class IT>
__device__ void small_pass(float4* P, IT* ML, IT* MR, int cap, int zlo0, int zhi, int n, int feat, float cut, bool pass2,
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
  __syncthreads();
  if (m != m2 || m > cap) {   // never (equal by construction): report, swap nothing
    if (lane == 0) {
      atomicOr(&ctl->err, 32);
      int* dbg = ctl->dbg;
      if (atomicCAS(dbg, 0, 1) == 0) {
        dbg[1] = zlo0; dbg[2] = zhi; dbg[3] = n; dbg[4] = feat; dbg[5] = __float_as_int(cut);
        dbg[6] = pass2; dbg[7] = m; dbg[8] = m2; dbg[9] = cap; dbg[10] = (int)blockIdx.x;
      }
    }
    return;
  }
  const int mm = m;
  for (int r = lane; r < mm; r += 64) {
    const int a = ML[r], c = MR[r];
    const float4 t = P[a];
    P[a] = P[c];
    P[c] = t;
  }
  __syncthreads();
}

// divideTree below one node, depth first: P = the node's points (LDS, or
// global for an oversized node), base = their vind offset
template <class IT>
__device__ void small_tree(const NfBuild& b, SmallLds* S, float4* P, IT* ML, IT* MR, int mlcap, const NfTask& tk) {
  NfCtl* ctl = b.ctl;
  const int lane = __lane_id();
  const int base = tk.begin;
  if (lane == 0) {
    S->sb[0] = 0;
    S->sc[0] = tk.count;
    S->sn[0] = tk.node;
    for (int a = 0; a < 3; ++a) {
      S->slo[a][0] = tk.lo[a];
      S->shi[a][0] = tk.hi[a];
    }
  }
  __syncthreads();
  int sp = 1;
  while (sp > 0) {
    --sp;
    const int lb = S->sb[sp], n = S->sc[sp], node = S->sn[sp];
    NfTask t;
    for (int a = 0; a < 3; ++a) {
      t.lo[a] = S->slo[a][sp];
      t.hi[a] = S->shi[a][sp];
    }
    __syncthreads();
    float4* Q = P + lb;
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
    if (n <= kNfLeafMax) {   // leaf (:992-1014)
      if (lane == 0) {
        b.nodes[node].c1 = base + lb;
        b.nodes[node].c2 = base + lb + n;
        b.nodes[node].feat = -1;
        b.box[2 * node] = make_float4(mn[0], mn[1], mn[2], 0.f);
        b.box[2 * node + 1] = make_float4(mx[0], mx[1], mx[2], 0.f);
      }
      continue;
    }
    for (int a = 0; a < 3; ++a) {
      t.mm[a] = f2o(mn[a]);
      t.mm[3 + a] = f2o(mx[a]);
    }
    int feat;
    float cut;
    nf_cut(t, &feat, &cut);
    feat = __builtin_amdgcn_readfirstlane(feat);   // wave-uniform by construction: scalar from here on
    cut = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(cut)));
    int lim1 = 0, lim2 = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + lane;
      const float x = i < n ? coord_at(&Q[i], feat) : INFINITY;
      lim1 += __popcll(__ballot(i < n && x < cut));
      lim2 += __popcll(__ballot(i < n && x <= cut));
    }
    small_pass(Q, ML, MR, mlcap, 0, lim1, n, feat, cut, false, ctl);
    small_pass(Q, ML, MR, mlcap, lim1, lim2, n, feat, cut, true, ctl);
    const int index = nf_index(n, lim1, lim2);
    int c1 = 0;
    if (lane == 0) c1 = atomicAdd(&ctl->nnodes, 2);
    c1 = __builtin_amdgcn_readfirstlane(c1);
    if (c1 + 2 > b.cap || sp + 2 > kNfStack) {
      if (lane == 0) atomicOr(&ctl->err, c1 + 2 > b.cap ? 1 : 4);
      return;
    }
    if (lane == 0) {
      b.nodes[node].c1 = c1;
      b.nodes[node].c2 = c1 + 1;
      b.nodes[node].feat = feat;
      b.nodes[c1].parent = node;
      b.nodes[c1 + 1].parent = node;
      // left_bbox / right_bbox (:1024-1030); the left child is popped first
      for (int s = 1; s >= 0; --s) {
        const int k = sp + (1 - s);
        S->sb[k] = lb + (s == 0 ? 0 : index);
        S->sc[k] = s == 0 ? index : n - index;
        S->sn[k] = c1 + s;
        for (int a = 0; a < 3; ++a) {
          S->slo[a][k] = t.lo[a];
          S->shi[a][k] = t.hi[a];
        }
        if (s == 0) S->shi[feat][k] = cut;
        else S->slo[feat][k] = cut;
      }
    }
    sp += 2;
    __syncthreads();
  }
}

__global__ __launch_bounds__(64) void k_nf_small(NfBuild b) {
  __shared__ SmallLds S_lds;   // static (~79 KB: gfx950 gives one workgroup up to 160 KB)
  SmallLds* S = &S_lds;
  if ((int)blockIdx.x >= b.ctl->nsmall) return;
  const NfTask tk = b.small[blockIdx.x];
  const int lane = __lane_id();
  if (tk.count <= kNfT) {
    for (int i = lane; i < tk.count; i += 64) S->P[i] = b.vpts[tk.begin + i];
    __syncthreads();
    small_tree<unsigned short>(b, S, S->P, S->ML, S->MR, kNfT / 2, tk);
    __syncthreads();
    for (int i = lane; i < tk.count; i += 64) b.vpts[tk.begin + i] = S->P[i];
  } else {   // in place in global memory; the rank lists use the pairing tables' space
    small_tree<unsigned>(b, S, b.vpts + tk.begin, reinterpret_cast<unsigned*>(b.tblL + tk.begin),
                         reinterpret_cast<unsigned*>(b.tblR + tk.begin), tk.count, tk);
  }
}

// Bottom-up boxes: one thread per leaf walks to the root; the second child
// to arrive at a node computes the node (device-scope ordering, no waiting).
__device__ __forceinline__ float4 ld_box(const float4* p) {
  const unsigned* u = reinterpret_cast<const unsigned*>(p);
  float4 r;
  r.x = __uint_as_float(__hip_atomic_load(u + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  r.y = __uint_as_float(__hip_atomic_load(u + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  r.z = __uint_as_float(__hip_atomic_load(u + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  r.w = 0.f;
  return r;
}
__device__ __forceinline__ void st_box(float4* p, float4 v) {
  unsigned* u = reinterpret_cast<unsigned*>(p);
  __hip_atomic_store(u + 0, __float_as_uint(v.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(u + 1, __float_as_uint(v.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(u + 2, __float_as_uint(v.z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void k_nf_refit(NfBuild b) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int nn = min(b.ctl->nnodes, b.cap);
  if (i >= nn || b.ctl->err) return;
  if (b.nodes[i].feat != -1) return;
  int cur = i;
  for (int step = 0; step < kNfMaxLevels + kNfStack + 8; ++step) {   // bounded: a tree is never deeper
    const int p = b.nodes[cur].parent;
    if (p < 0) break;
    __threadfence();
    if (atomicAdd(&b.arrive[p], 1) == 0) break;   // the sibling's thread finishes the node
    __threadfence();
    const NfNode nd = b.nodes[p];
    const float4 l1 = ld_box(&b.box[2 * nd.c1]), h1 = ld_box(&b.box[2 * nd.c1 + 1]);
    const float4 l2 = ld_box(&b.box[2 * nd.c2]), h2 = ld_box(&b.box[2 * nd.c2 + 1]);
    // bbox = (std::min / std::max of the children's boxes) (:1035-1039)
    const float4 lo = make_float4(l2.x < l1.x ? l2.x : l1.x, l2.y < l1.y ? l2.y : l1.y, l2.z < l1.z ? l2.z : l1.z, 0.f);
    const float4 hi = make_float4(h1.x < h2.x ? h2.x : h1.x, h1.y < h2.y ? h2.y : h1.y, h1.z < h2.z ? h2.z : h1.z, 0.f);
    st_box(&b.box[2 * p], lo);
    st_box(&b.box[2 * p + 1], hi);
    b.nodes[p].divlow = coord(h1, nd.feat);    // left_bbox[cutfeat].high
    b.nodes[p].divhigh = coord(l2, nd.feat);   // right_bbox[cutfeat].low
    cur = p;
  }
}

// ---------------------------------------------------------------------------
// tie resolution: re-run the flagged queries with nanoflann's search
template <int KMAX>
__global__ __launch_bounds__(64) void k_nf_resolve_cov(NfTreeDev t, CloudDev c, const int* __restrict__ list,
                                                       const int* __restrict__ count, int k, int method,
                                                       double* __restrict__ cov6, const int* __restrict__ status,
                                                       int* __restrict__ err) {
  const int nl = *count;
  if (*status) {   // the tree build failed: report, keep the Morton-order answers
    if (blockIdx.x == 0 && threadIdx.x == 0 && nl > 0) atomicOr(err, 2);
    return;
  }
  for (int li = blockIdx.x * blockDim.x + threadIdx.x; li < nl; li += gridDim.x * blockDim.x) {
    const int s = list[li];              // sorted position of the query point
    const float4 q = c.pts[s];
    NfResult<KMAX> rs;
    rs.init(k);
    if (!nf_search<KMAX>(t, q.x, q.y, q.z, rs) || rs.count < k) {
      atomicOr(err, 1);
      continue;
    }
    // mean and biased covariance in neighbour order (nano_gicp_impl.hpp:392-399)
    double mx = 0, my = 0, mz = 0;
    for (int j = 0; j < k; ++j) {
      const float4 p = c.pts[c.inv_perm[rs.ix[j]]];
      mx += (double)p.x;
      my += (double)p.y;
      mz += (double)p.z;
    }
    mx /= k;
    my /= k;
    mz /= k;
    double C[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const float4 p = c.pts[c.inv_perm[rs.ix[j]]];
      const double d0 = (double)p.x - mx, d1 = (double)p.y - my, d2 = (double)p.z - mz;
      C[0] += d0 * d0; C[1] += d0 * d1; C[2] += d0 * d2;
      C[3] += d1 * d0; C[4] += d1 * d1; C[5] += d1 * d2;
      C[6] += d2 * d0; C[7] += d2 * d1; C[8] += d2 * d2;
    }
    for (int e = 0; e < 9; ++e) C[e] /= k;
    double out[6];
    regularize(C, method, out);
    double* o = cov6 + 6 * (size_t)s;
    for (int e = 0; e < 6; ++e) o[e] = out[e];
  }
}

template <int KMAX>
__global__ __launch_bounds__(64) void k_nf_resolve_knn(NfTreeDev t, const float4* __restrict__ q,
                                                       const int* __restrict__ list, const int* __restrict__ count,
                                                       int k, int* __restrict__ out_idx, float* __restrict__ out_d,
                                                       const int* __restrict__ status, int* __restrict__ err) {
  const int nl = *count;
  if (*status) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && nl > 0) atomicOr(err, 2);
    return;
  }
  for (int li = blockIdx.x * blockDim.x + threadIdx.x; li < nl; li += gridDim.x * blockDim.x) {
    const int i = list[li];   // query row
    const float4 p = q[i];
    NfResult<KMAX> rs;
    rs.init(k);
    if (!nf_search<KMAX>(t, p.x, p.y, p.z, rs) || rs.count < k) {
      atomicOr(err, 1);
      continue;
    }
    for (int j = 0; j < k; ++j) {
      out_idx[(size_t)i * k + j] = rs.ix[j];
      out_d[(size_t)i * k + j] = rs.d[j];
    }
  }
}

// vind starts as the identity (init_vind): the cloud's points in original order
__global__ __launch_bounds__(256) void k_nf_unsort(const float4* __restrict__ sorted, int n, float4* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const float4 p = sorted[s];
  out[__float_as_int(p.w)] = p;
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
  if (n > kNfT) {
    int l = 0;
    while ((long)kNfT << l < n) ++l;
    z.Lmax = std::min(l + 2, kNfMaxLevels);
  }
  z.max_task = n / kNfT + 2;
  z.max_pend = 2 * z.max_task;
  z.max_small = 2 * (z.Lmax + 1) * z.max_task + 2;
  z.max_chunks = cdivl(n, kNfCH) + z.max_task;
  return z;
}

size_t nf_small_lds_bytes() { return sizeof(SmallLds); }

void launch_nf_build(hipStream_t s, const NfBuild& b, const float4* sorted_pts, int stop) {
  k_nf_unsort<<<cdivl(b.n, 256), 256, 0, s>>>(sorted_pts, b.n, b.vpts);
  k_nf_init<<<1, 64, 0, s>>>(b);
  const int G = std::max(1, b.max_chunks);
  for (int L = 0; L < b.Lmax; ++L) {
    if (stop >= 0 && L >= stop) return;
    k_nf_map<<<1, 1024, 0, s>>>(b, L);
    k_nf_count<<<G, kNfBT, 0, s>>>(b, L);
    k_nf_pass<1, true><<<G, kNfBT, 0, s>>>(b, L);
    k_nf_pass<1, false><<<G, kNfBT, 0, s>>>(b, L);
    k_nf_pass<2, true><<<G, kNfBT, 0, s>>>(b, L);
    k_nf_pass<2, false><<<G, kNfBT, 0, s>>>(b, L);
  }
  k_nf_map<<<1, 1024, 0, s>>>(b, b.Lmax);
  k_nf_small<<<b.max_small, 64, 0, s>>>(b);
  k_nf_refit<<<cdivl(b.cap, 256), 256, 0, s>>>(b);
}

void launch_nf_export(hipStream_t s, const NfTreeDev& t, const int* status, int cap, int* vind, int* nodes, float* f) {
  k_nf_export<<<cdivl(std::max(t.n, cap), 256), 256, 0, s>>>(t, status, cap, vind, nodes, f);
}

bool launch_nf_resolve_cov(hipStream_t s, const NfTreeDev& t, const CloudDev& c, const int* list, const int* count,
                           int k, int method, double* cov6, const int* status, int* err) {
  const int nb = 64;
  if (k <= 16) k_nf_resolve_cov<16><<<nb, 64, 0, s>>>(t, c, list, count, k, method, cov6, status, err);
  else if (k <= 32) k_nf_resolve_cov<32><<<nb, 64, 0, s>>>(t, c, list, count, k, method, cov6, status, err);
  else if (k <= 64) k_nf_resolve_cov<64><<<nb, 64, 0, s>>>(t, c, list, count, k, method, cov6, status, err);
  else return false;
  return true;
}

bool launch_nf_resolve_knn(hipStream_t s, const NfTreeDev& t, const float4* q, const int* list, const int* count, int k,
                           int* out_idx, float* out_d, const int* status, int* err) {
  const int nb = 64;
  if (k <= 16) k_nf_resolve_knn<16><<<nb, 64, 0, s>>>(t, q, list, count, k, out_idx, out_d, status, err);
  else if (k <= 32) k_nf_resolve_knn<32><<<nb, 64, 0, s>>>(t, q, list, count, k, out_idx, out_d, status, err);
  else if (k <= 64) k_nf_resolve_knn<64><<<nb, 64, 0, s>>>(t, q, list, count, k, out_idx, out_d, status, err);
  else return false;
  return true;
}

}  // namespace ddlo
