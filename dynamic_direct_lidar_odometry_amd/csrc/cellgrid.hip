// cellgrid.hip — candidate cells of an S2M target (DESIGN.md §4 "Candidate
// cells"): built once per (target, correspondence bound), they turn the
// bounded 1-NN of update_correspondences (reference
// include/nano_gicp/impl/nano_gicp_impl.hpp:249-258, nanoflann_impl.hpp:1495-1566)
// into a cell lookup plus a scan of a short list, for every outer iteration
// of every scan aligned against the target.
//
// Build (once per target):
//   K7a k_cg_occ / k_cg_dilate x3 / k_cg_band: coarse cells within reach of
//       the target (Chebyshev dilation of the occupied cells by the bound);
//   K7b the exact nearest target point of each band cell's centre
//       (k_knn_query, kernels.hip);
//   K7c k_cg_coarse: one wavefront per band cell walks the Morton hierarchy
//       for the points within the cell's reach, keeps those the centre's
//       nearest point does not dominate, finds the corners' nearest points
//       among them and prunes with all nine dominators (cellgrid.hpp);
//   K7d k_cg_decide / k_cg_refine (levels 1..3): a coarse cell whose lists
//       are longer than lmax is split 2x2x2 from its parent lists (the parent
//       list holds the nearest point of every point of the parent box, so
//       the children's dominators are found in it);
//   K7e k_cg_emit_count / k_cg_emit_write: the final level of every coarse
//       cell written as a fine table and point copies (x, y, z, position).
// Lookup: k_cell_lookup (kernels.hip), one query per lane.
#include <hip/hip_runtime.h>

#include "cellgrid.hpp"
#include "search.hpp"

namespace ddlo {

namespace {

constexpr int kCgWaves = 4;          // waves per block (independent cells)
constexpr int kCgShards = kCgShardsHost;   // pool allocation counters (one contended word saturates at ~88 atomics/us)
constexpr unsigned kCgChunk = 512;   // pool entries a wave takes per allocation

__device__ __forceinline__ int mbcnt(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
__device__ __forceinline__ unsigned ufirst(unsigned v) { return (unsigned)__builtin_amdgcn_readfirstlane((int)v); }
// the kCgShards allocation counters of level l's pool (one 128-B line each)
__device__ __forceinline__ unsigned* pool_ctr(const CgBuild& b, int l) { return b.ctr + kCgCounters * 32 + l * kCgShards * 32; }

// Wave-uniform bump allocator over a pool split into kCgShards ranges, one
// allocation counter each (ctr[shard * 32], the first pool entry of each
// range at shard * cap / kCgShards).  Returns ~0u when the range is full.
struct Bump {
  unsigned cur = 0, end = 0;
  __device__ __forceinline__ unsigned take(unsigned n, unsigned* ctr, unsigned cap, int shard) {
    if (cur + n > end || end == 0) {
      const unsigned want = n > kCgChunk ? n : kCgChunk;
      const unsigned range = cap / kCgShards;
      unsigned s = 0;
      if (lane_id() == 0) s = atomicAdd(ctr + shard * 32, want);
      s = ufirst(s);
      if (s + want > range) return ~0u;
      cur = shard * range + s;
      end = cur + want;
    }
    const unsigned r = cur;
    cur += n;
    return r;
  }
};

// A cell box (expanded by delta), centre and half size in metres.
struct CgBox {
  double cx, cy, cz, hb;
};

// Coordinates relative to a box centre, in fp32: the build's tests carry
// margins (2e-5 relative) far above the fp32 rounding of these small numbers.
struct Rel {
  float x, y, z;
};
__device__ __forceinline__ Rel rel(const CgBox& B, float px, float py, float pz) {
  return Rel{(float)((double)px - B.cx), (float)((double)py - B.cy), (float)((double)pz - B.cz)};
}
// squared box distance
__device__ __forceinline__ float bd2(Rel a, float hb) {
  const float ex = fmaxf(fabsf(a.x) - hb, 0.f), ey = fmaxf(fabsf(a.y) - hb, 0.f), ez = fmaxf(fabsf(a.z) - hb, 0.f);
  return ex * ex + ey * ey + ez * ez;
}
// squared farthest-corner distance
__device__ __forceinline__ float far2(Rel a, float hb) {
  const float ex = fabsf(a.x) + hb, ey = fabsf(a.y) + hb, ez = fabsf(a.z) + hb;
  return ex * ex + ey * ey + ez * ez;
}
// p strictly beaten by d at every point of the box, by more than the fp32
// rounding of the search's squared distances (<= 4.8e-7 relative of the sum
// of the two; the margin is 2e-5 of an upper bound of it):
// min over q of |q-p|^2 - |q-d|^2 = |p|^2 - |d|^2 - 2 hb |p - d|_1  (box-centred)
__device__ __forceinline__ bool dominated(Rel p, Rel d, float hb) {
  const float p2 = p.x * p.x + p.y * p.y + p.z * p.z;
  const float d2 = d.x * d.x + d.y * d.y + d.z * d.z;
  const float l1 = fabsf(p.x - d.x) + fabsf(p.y - d.y) + fabsf(p.z - d.z);
  const float f = (p2 - d2) - 2.f * hb * l1;
  return f > 2e-5f * (p2 + d2 + 6.f * hb * hb) + 1e-12f;
}
// list radius from the dominators' farthest-corner distance: R = min(D, capm),
// widened by 1e-5 relative (every point that can be the fp32 nearest or tie)
__device__ __forceinline__ float list_radius2(float dmin2, double capm) {
  const double D = sqrt((double)dmin2) * (1.0 + 2e-6);
  const double R = (D < capm ? D : capm) * (1.0 + 1e-5) + 1e-6;
  return (float)(R * R);
}

__device__ __forceinline__ void cell_coords(const CgBuild& b, int cell, int& cx, int& cy, int& cz) {
  cz = cell % b.nz;
  const int t = cell / b.nz;
  cy = t % b.ny;
  cx = t / b.ny;
}

// box of fine cell (fx, fy, fz) at level l of coarse cell (cx, cy, cz), expanded by delta
__device__ __forceinline__ CgBox fine_box(const CgBuild& b, int cx, int cy, int cz, int l, int fx, int fy, int fz) {
  const double m = (double)(1 << l);
  const double sz = b.s / m;
  CgBox B;
  B.cx = b.ox + (double)cx * b.s + ((double)fx + 0.5) * sz;
  B.cy = b.oy + (double)cy * b.s + ((double)fy + 0.5) * sz;
  B.cz = b.oz + (double)cz * b.s + ((double)fz + 0.5) * sz;
  B.hb = 0.5 * sz + b.delta;
  return B;
}

__device__ __forceinline__ bool box_meets(float4 lo, float4 hi, float3 qlo, float3 qhi) {
  return lo.x <= qhi.x && hi.x >= qlo.x && lo.y <= qhi.y && hi.y >= qlo.y && lo.z <= qhi.z && hi.z >= qlo.z;
}

__device__ __forceinline__ unsigned long long wave_umin64(unsigned long long v) {
  v = xor_min64<32>(v);
  v = xor_min64<16>(v);
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) v = umin64(v, __shfl_xor(v, m));
  return v;
}

constexpr unsigned kHdrSkip = 0xffffffffu;       // hdr count: no list (NoMatch cell, dir final)
constexpr int kNoMatchList = -2;                 // direct_list: no target point within the bound of the box
constexpr int kRepNone = 0x7f7f7f7f;             // no representative (the host fills with bytes 0x7f)
constexpr unsigned kHdrOverflow = 0xfffffffeu;   // hdr count: more than kCgCandMax points (split directly)

// A node box entirely dominated by d over the cell box (every point of it
// strictly beaten by d with the rounding margin of dominated()): lower bounds
// of |p|^2 and upper bounds of |p - d|_1 and |p|^2 over the node, box-centred.
__device__ __forceinline__ bool node_dominated(const CgBox& B, float hb, float4 lo, float4 hi, Rel d) {
  float l[3] = {(float)((double)lo.x - B.cx), (float)((double)lo.y - B.cy), (float)((double)lo.z - B.cz)};
  float h[3] = {(float)((double)hi.x - B.cx), (float)((double)hi.y - B.cy), (float)((double)hi.z - B.cz)};
  const float dd[3] = {d.x, d.y, d.z};
  float mind2 = 0.f, maxd2 = 0.f, maxl1 = 0.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    l[k] -= 1e-6f * (1.f + fabsf(l[k]));   // outward: the node box stays a superset after rounding
    h[k] += 1e-6f * (1.f + fabsf(h[k]));
    const float e = fmaxf(fmaxf(l[k], -h[k]), 0.f);
    const float m = fmaxf(fabsf(l[k]), fabsf(h[k]));
    mind2 += e * e;
    maxd2 += m * m;
    maxl1 += fmaxf(fabsf(l[k] - dd[k]), fabsf(h[k] - dd[k]));
  }
  const float d2 = d.x * d.x + d.y * d.y + d.z * d.z;
  const float f = (mind2 - d2) - 2.f * hb * maxl1;
  return f > 2e-5f * (maxd2 + d2 + 6.f * hb * hb) + 1e-12f;
}

// Walk of the Morton hierarchy over the nodes that meet [qlo, qhi] and that
// node_ok accepts; leaf(pos, p) for every point of the accepted leaves
// (lanes 0-31 and 32-63 take one leaf each).  Wave-uniform control.
template <class NodeOk, class Leaf>
__device__ __forceinline__ void walk_region(const CloudDev& c, float3 qlo, float3 qhi, NodeOk node_ok, Leaf leaf) {
  const int lane = lane_id();
  const int T = c.nlevels - 1;
  const int Tt = T < 1 ? 1 : T;
  unsigned long long m1 = 0, m2 = 0, m3 = 0, m4 = 0;
  int b1 = 0, b2 = 0, b3 = 0;
  if (T == 0) {
    m1 = 1ull;
  } else {
    bool ov = false;
    if (lane < lvl_cnt(c, T)) {
      const int o = lvl_off(c, T) + lane;
      const float4 lo = ldg4(c.box_lo, o), hi = ldg4(c.box_hi, o);
      ov = box_meets(lo, hi, qlo, qhi) && node_ok(lo, hi);
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
    bool ov = false;
    if (lane < cnt) {
      const int o = lvl_off(c, lv - 1) + cb + lane;
      const float4 lo = ldg4(c.box_lo, o), hi = ldg4(c.box_hi, o);
      ov = box_meets(lo, hi, qlo, qhi) && node_ok(lo, hi);
    }
    unsigned long long cm = __ballot(ov);
    if (lv > 1) {
      --lv;
      if (lv == 1) { m1 = cm; b1 = cb; } else if (lv == 2) { m2 = cm; b2 = cb; } else { m3 = cm; b3 = cb; }
      continue;
    }
    while (cm) {
      const int la = __builtin_ctzll(cm);
      cm &= cm - 1;
      int lb = -1;
      if (cm) {
        lb = __builtin_ctzll(cm);
        cm &= cm - 1;
      }
      const int lf = lane < 32 ? la : lb;
      const int pos = lf >= 0 ? (cb + lf) * kLeafSize + (lane & 31) : c.n;
      const bool valid = pos < c.n;
      const float4 p = valid ? ldg4(c.pts, pos) : make_float4(0.f, 0.f, 0.f, 0.f);
      leaf(valid, pos, p);
    }
  }
}

// The list of a cell box B, straight from the target: pass 1 finds the
// target points nearest to B's 8 corners and centre (the dominators) within
// the reach of p0 (any target point, here a near one), pass 2 keeps the
// points within R = min(D, bound) of B that no dominator dominates.  Both
// walks skip nodes p0 dominates (the corners' nearest points are never
// dominated by p0, the kept points never by a dominator).  Returns the kept
// count (positions in cand[]), or -1 when more than kCgCandMax are kept.
__device__ __forceinline__ int direct_list(const CgBuild& b, const CgBox& B, float4 p0w, unsigned* cand) {
  const CloudDev& c = b.tgt;
  const int lane = lane_id();
  const float hb = (float)B.hb;
  const Rel p0 = rel(B, p0w.x, p0w.y, p0w.z);
  auto region = [&](float Rsq, float3& qlo, float3& qhi) {
    const float R = sqrtf(Rsq) * 1.0001f + 1e-4f;
    qlo = make_float3((float)(B.cx - B.hb) - R, (float)(B.cy - B.hb) - R, (float)(B.cz - B.hb) - R);
    qhi = make_float3((float)(B.cx + B.hb) + R, (float)(B.cy + B.hb) + R, (float)(B.cz + B.hb) + R);
  };
  auto not_dom_p0 = [&](float4 lo, float4 hi) { return !node_dominated(B, hb, lo, hi, p0); };
  // pass 1: the nearest points of the 8 corners (unexpanded box) and the centre
  const float R0sq = list_radius2(far2(p0, hb), b.capm);
  float3 qlo, qhi;
  region(R0sq, qlo, qhi);
  const float h0 = (float)(B.hb - b.delta);   // the unexpanded half size
  unsigned long long ck[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) ck[q] = ~0ull;
  walk_region(c, qlo, qhi, not_dom_p0, [&](bool valid, int pos, float4 p) {
    if (!valid) return;
    const Rel a = rel(B, p.x, p.y, p.z);
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const float ox = q == 8 ? 0.f : ((q & 4) ? h0 : -h0), oy = q == 8 ? 0.f : ((q & 2) ? h0 : -h0),
                  oz = q == 8 ? 0.f : ((q & 1) ? h0 : -h0);
      const float dx = a.x - ox, dy = a.y - oy, dz = a.z - oz;
      ck[q] = umin64(ck[q], dkey(dx * dx + dy * dy + dz * dz, pos));
    }
  });
  Rel dom[10];
  float dmin2 = far2(p0, hb);
  dom[9] = p0;
  float cd2 = INFINITY;   // the centre's nearest squared distance (fp32) within reach
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const unsigned long long kq = wave_umin64(ck[q]);
    Rel d = p0;
    if (kq != ~0ull) {
      const float4 p = ldg4(c.pts, (int)(unsigned)kq);
      d = rel(B, p.x, p.y, p.z);
      if (q == 8) cd2 = __uint_as_float((unsigned)(kq >> 32));
    }
    dom[q] = d;
    dmin2 = fminf(dmin2, far2(d, hb));
  }
  // every point of the box is farther than the bound from every target point:
  // the centre's nearest distance (exact within reach: pass 1 examined every
  // point p0 does not dominate, and the nearest is never dominated) minus the
  // half diagonal exceeds it
  if (sqrt((double)cd2 / (1.0 + 1e-6)) - 1.7320509 * B.hb - 1e-5 > b.capm) return kNoMatchList;
  // pass 2: the kept points
  const float Rsq = list_radius2(dmin2, b.capm);
  region(Rsq, qlo, qhi);
  int n = 0;
  walk_region(c, qlo, qhi,
              [&](float4 lo, float4 hi) {
                return !node_dominated(B, hb, lo, hi, dom[8]) && !node_dominated(B, hb, lo, hi, p0);
              },
              [&](bool valid, int pos, float4 p) {
                bool keep = false;
                if (valid) {
                  const Rel a = rel(B, p.x, p.y, p.z);
                  keep = bd2(a, hb) <= Rsq;
#pragma unroll
                  for (int q = 0; q < 10; ++q) keep = keep && !dominated(a, dom[q], hb);
                }
                const unsigned long long bal = __ballot(keep);
                const int o = n + mbcnt(bal);
                if (keep && o < kCgCandMax) cand[o] = (unsigned)pos;
                n += __popcll(bal);
              });
  (void)lane;
  __builtin_amdgcn_wave_barrier();
  return n > kCgCandMax ? -1 : n;
}

}  // namespace

// ---------------------------------------------------------------------------
// K7a: occupancy of the coarse cells, the band (Chebyshev dilation by r
// cells: a non-band cell is at least r - 1 whole cells from every target
// point), and the band cells in 4x4x4-blocked order (spatially coherent
// wavefronts for the nearest-point pass).
__global__ __launch_bounds__(256) void k_cg_occ(const CgBuild* __restrict__ bp, int n) {
  // representative of every occupied coarse cell: its lowest sorted position
  // (the Morton-sorted points of a cell form few runs: one atomic per run)
  const CgBuild& b = *bp;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  auto cell_of = [&](int j) {
    const float4 p = ldg4(b.tgt.pts, j);
    const int cx = min(max((int)floorf((p.x - b.fox) * b.inv_s), 0), b.nx - 1);
    const int cy = min(max((int)floorf((p.y - b.foy) * b.inv_s), 0), b.ny - 1);
    const int cz = min(max((int)floorf((p.z - b.foz) * b.inv_s), 0), b.nz - 1);
    return ((long)cx * b.ny + cy) * b.nz + cz;
  };
  const long c = cell_of(i);
  if (i == 0 || cell_of(i - 1) != c) atomicMin(b.rep + c, i);
}

// Separable propagation of the nearest representative along one axis within
// r cells (the three passes give every cell within Chebyshev distance r of an
// occupied cell a near target point: the band, and each band cell's first
// dominator p0; any target point is a valid dominator, so near is enough)
__global__ __launch_bounds__(256) void k_cg_prop(const CgBuild* __restrict__ bp, int axis, const int* __restrict__ in,
                                                 int* __restrict__ out, long ncells) {
  const CgBuild& b = *bp;
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncells) return;
  int cx, cy, cz;
  cell_coords(b, (int)c, cx, cy, cz);
  const int v = axis == 0 ? cx : axis == 1 ? cy : cz;
  const int nv = axis == 0 ? b.nx : axis == 1 ? b.ny : b.nz;
  const long stride = axis == 0 ? (long)b.ny * b.nz : axis == 1 ? (long)b.nz : 1;
  const float ccx = b.fox + ((float)cx + 0.5f) / b.inv_s, ccy = b.foy + ((float)cy + 0.5f) / b.inv_s,
              ccz = b.foz + ((float)cz + 0.5f) / b.inv_s;
  int best = kRepNone;
  float bd = INFINITY;
  const int lo = max(v - b.r, 0), hi = min(v + b.r, nv - 1);
  for (int k = lo; k <= hi; ++k) {
    const int r = in[c + (long)(k - v) * stride];
    if (r == kRepNone) continue;
    const float4 p = ldg4(b.tgt.pts, r);
    const float d = dist2(ccx, ccy, ccz, p.x, p.y, p.z);
    if (d < bd) {
      bd = d;
      best = r;
    }
  }
  out[c] = best;
}

__global__ __launch_bounds__(256) void k_cg_dir_fill(unsigned long long* __restrict__ dir, const int* __restrict__ band,
                                                     long ncells, unsigned long long outside) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < ncells) dir[c] = band[c] != kRepNone ? kCgFallback : outside;
}

__global__ __launch_bounds__(256) void k_cg_band_flags(const CgBuild* __restrict__ bp, const int* __restrict__ band,
                                                       unsigned char* __restrict__ flags, long nblocked) {
  const CgBuild& b = *bp;
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= nblocked) return;
  const int nbz = (b.nz + 3) / 4, nby = (b.ny + 3) / 4;
  const long blk = id >> 6;
  const int w = (int)(id & 63);
  const int bz = (int)(blk % nbz), by = (int)((blk / nbz) % nby), bx = (int)(blk / ((long)nbz * nby));
  const int cx = 4 * bx + (w >> 4), cy = 4 * by + ((w >> 2) & 3), cz = 4 * bz + (w & 3);
  unsigned char f = 0;
  if (cx < b.nx && cy < b.ny && cz < b.nz) f = band[((long)cx * b.ny + cy) * b.nz + cz] != kRepNone;
  flags[id] = f;
}

// blocked id -> cell id, and the centre query of each band cell
__global__ __launch_bounds__(256) void k_cg_centers(CgBuild* __restrict__ bp, int nband) {
  const CgBuild& b = *bp;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nband) return;
  const long id = b.band[k];
  const int nbz = (b.nz + 3) / 4, nby = (b.ny + 3) / 4;
  const long blk = id >> 6;
  const int w = (int)(id & 63);
  const int bz = (int)(blk % nbz), by = (int)((blk / nbz) % nby), bx = (int)(blk / ((long)nbz * nby));
  const int cx = 4 * bx + (w >> 4), cy = 4 * by + ((w >> 2) & 3), cz = 4 * bz + (w & 3);
  const long cell = ((long)cx * b.ny + cy) * b.nz + cz;
  b.band[k] = (int)cell;
  b.cnn[k] = b.rep_final[cell];   // sorted position of a near target point
}

// ---------------------------------------------------------------------------
// K7c: level-0 list of every band cell, one wavefront per cell (direct_list).
__global__ __launch_bounds__(64 * kCgWaves) void k_cg_coarse(const CgBuild* __restrict__ bp, int nband) {
  const CgBuild& b = *bp;
  const CloudDev& c = b.tgt;
  __shared__ unsigned cand_all[kCgWaves][kCgCandMax];
  const int wib = threadIdx.x >> 6;
  unsigned* const cand = cand_all[wib];
  const int lane = lane_id();
  const int wave = blockIdx.x * kCgWaves + wib;
  const int nwaves = gridDim.x * kCgWaves;
  const int shard = wave % kCgShards;
  const CgLevel L0 = b.lv[0];
  Bump bump;
  for (int bi = wave; bi < nband; bi += nwaves) {
    const int cell = b.band[bi];
    int cx, cy, cz;
    cell_coords(b, cell, cx, cy, cz);
    const CgBox B = fine_box(b, cx, cy, cz, 0, 0, 0, 0);
    const float4 p0 = ldg4(c.pts, b.cnn[bi]);
    const int n = direct_list(b, B, p0, cand);
    if (n == kNoMatchList) {   // no target point within the bound of any point of the cell
      if (lane == 0) {
        b.dir[cell] = kCgNoMatch;
        L0.hdr[bi] = make_uint2(0u, kHdrSkip);
      }
      continue;
    }
    if (n < 0) {   // more than kCgCandMax points: the cell is split (level 1, direct)
      if (lane == 0) {
        L0.hdr[bi] = make_uint2(0u, kHdrOverflow);
        atomicAdd(b.ctr + kCtrOverflow * 32, 1u);
      }
      continue;
    }
    unsigned off = 0;
    if (n > 0) {
      off = bump.take((unsigned)n, pool_ctr(b, 0), L0.pool_cap, shard);
      if (off == ~0u) {
        if (lane == 0) atomicOr(b.ctr + kCtrPoolFull * 32, 1u);
        continue;
      }
      for (int k = lane; k < n; k += 64) L0.pool[off + k] = cand[k];
    }
    if (lane == 0) L0.hdr[bi] = make_uint2(off, (unsigned)n);
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------------------
// K7d: level decisions.  level 0: lane per band cell (its hdr0 count);
// level l >= 1: lane per slot (cmax).  flags: 1 = final at this level,
// 2 = split one level deeper.  A band cell without any point within reach is
// NoMatch (no final).
__global__ __launch_bounds__(256) void k_cg_decide(CgBuild* __restrict__ bp, int level, int nslots,
                                                   unsigned char* __restrict__ fl_final, unsigned char* __restrict__ fl_next) {
  const CgBuild& b = *bp;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nslots) return;
  unsigned char f = 0, x = 0;
  if (level == 0) {
    const uint2 h = b.lv[0].hdr[s];
    if (h.y == kHdrSkip) {
      // NoMatch: dir already final
    } else if (h.y == kHdrOverflow) {
      x = 1;
    } else if (h.y == 0u) {
      b.dir[b.band[s]] = kCgNoMatch;
    } else if ((int)h.y <= b.lmax) {
      f = 1;
    } else {
      x = 1;
    }
  } else {
    const int cm = b.lv[level].cmax[s];
    if (cm <= b.lmax || level == kCgMaxLevel) f = 1;
    else x = 1;
  }
  fl_final[s] = f;
  fl_next[s] = x;
}

// after the select of the slots split one level deeper: each new slot's band cell
__global__ __launch_bounds__(256) void k_cg_slots(CgBuild* __restrict__ bp, int level, int nslots) {
  const CgBuild& b = *bp;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nslots) return;
  const int p = b.lv[level].slot_parent[s];
  b.lv[level].slot_band[s] = level == 1 ? p : b.lv[level - 1].slot_band[p];
  b.lv[level].cmax[s] = 0;
}

// K7d: one wavefront per (slot, parent fine cell) at level l: the parent's
// list split into its 8 children (fine cells of level l).
__global__ __launch_bounds__(64 * kCgWaves) void k_cg_refine(const CgBuild* __restrict__ bp, int level, int nslots) {
  const CgBuild& b = *bp;
  const CloudDev& c = b.tgt;
  __shared__ unsigned char msk_all[kCgWaves][kCgCandMax];
  __shared__ Rel lat_all[kCgWaves][36];
  __shared__ unsigned cand_all[kCgWaves][kCgCandMax];   // direct children (a parent with too many points)
  const int wib = threadIdx.x >> 6;
  unsigned char* const msk = msk_all[wib];
  unsigned* const cand = cand_all[wib];
  const int lane = lane_id();
  const int wave = blockIdx.x * kCgWaves + wib;
  const int nwaves = gridDim.x * kCgWaves;
  const int shard = wave % kCgShards;
  const CgLevel P = b.lv[level - 1], L = b.lv[level];
  const int mp = 1 << (level - 1), m = 1 << level;
  const int nparent = mp * mp * mp;
  const long items = (long)nslots * nparent;
  Bump bump;
  for (long it = wave; it < items; it += nwaves) {
    const int s = (int)(it / nparent), fp = (int)(it % nparent);
    const int ps = L.slot_parent[s];
    const int bi = L.slot_band[s];
    const uint2 ph = P.hdr[(size_t)ps * nparent + fp];
    const int n = (int)ph.y;
    int cx, cy, cz;
    cell_coords(b, b.band[bi], cx, cy, cz);
    const int px = fp / (mp * mp), py = (fp / mp) % mp, pz = fp % mp;
    // parent box (unexpanded half size hp) and the children's expanded half size
    const CgBox PB = fine_box(b, cx, cy, cz, level - 1, px, py, pz);
    const float hp = (float)(0.5 * b.s / mp);
    const float hc = (float)(0.25 * b.s / mp + b.delta);
    const float hq = 0.5f * hp;   // child centre offset
    if (ph.y == kHdrOverflow) {
      // the parent kept more than kCgCandMax points: each child straight from the target
      const float4 p0w = ldg4(c.pts, b.cnn[bi]);
      int cmx = 0;
#pragma unroll 1
      for (int o = 0; o < 8; ++o) {
        const int fx = 2 * px + ((o >> 2) & 1), fy = 2 * py + ((o >> 1) & 1), fz = 2 * pz + (o & 1);
        const CgBox CB = fine_box(b, cx, cy, cz, level, fx, fy, fz);
        int nk = direct_list(b, CB, p0w, cand);
        if (nk == kNoMatchList) nk = 0;   // no point within the bound: an empty list
        uint2 h = make_uint2(0u, kHdrOverflow);
        if (nk < 0) {
          cmx = 0x7fffffff;
        } else {
          unsigned off = 0;
          if (nk > 0) {
            off = bump.take((unsigned)nk, pool_ctr(b, level), L.pool_cap, shard);
            if (off == ~0u) {
              if (lane == 0) atomicOr(b.ctr + kCtrPoolFull * 32, 1u);
              break;
            }
            for (int k = lane; k < nk; k += 64) L.pool[off + k] = cand[k];
          }
          h = make_uint2(off, (unsigned)nk);
          cmx = max(cmx, nk);
        }
        if (lane == 0) L.hdr[(size_t)s * m * m * m + (fx * m + fy) * m + fz] = h;
        __builtin_amdgcn_wave_barrier();
      }
      if (lane == 0) atomicMax(L.cmax + s, cmx);
      continue;
    }
    int cnt[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) cnt[o] = 0;
    if (n > 0 && n <= kCgCandMax) {
      // nearest list point of the 27 lattice points (children's corners) and the 8 child centres
      // keys: the squared distance's bits with the low 11 replaced by the list
      // index (n <= kCgCandMax = 2^11): a dominator need not be the exact
      // nearest point, and a 32-bit key reduces with DPP
      static_assert(kCgCandMax <= 2048, "11-bit list index in the keys");
      unsigned lk[35];
#pragma unroll
      for (int q = 0; q < 35; ++q) lk[q] = 0xffffffffu;
      for (int k = lane; k < n; k += 64) {
        const float4 p = ldg4(c.pts, P.pool[ph.x + k]);
        const Rel a = rel(PB, p.x, p.y, p.z);
#pragma unroll
        for (int q = 0; q < 35; ++q) {
          float qx, qy, qz;
          if (q < 27) {
            qx = (float)(q / 9 - 1) * hp;
            qy = (float)((q / 3) % 3 - 1) * hp;
            qz = (float)(q % 3 - 1) * hp;
          } else {
            const int o = q - 27;
            qx = (o & 4) ? hq : -hq;
            qy = (o & 2) ? hq : -hq;
            qz = (o & 1) ? hq : -hq;
          }
          const float dx = a.x - qx, dy = a.y - qy, dz = a.z - qz;
          lk[q] = min(lk[q], (__float_as_uint(dx * dx + dy * dy + dz * dz) & ~0x7ffu) | (unsigned)k);
        }
      }
      // the 35 nearest points, parent-centred, in LDS (wave-uniform reads)
      Rel* const lat = lat_all[wib];
#pragma unroll
      for (int q = 0; q < 35; ++q) {
        // non-negative float bit patterns order like unsigned ints (all ones: NaN, ignored by fminf)
        const unsigned kq = __float_as_uint(wave_min(__uint_as_float(lk[q])));
        if (lane == q) {
          const float4 p = ldg4(c.pts, P.pool[ph.x + (int)(kq & 0x7ffu)]);
          lat[q] = rel(PB, p.x, p.y, p.z);
        }
      }
      __builtin_amdgcn_wave_barrier();
      // per child: dominators (its 8 corners' and centre's nearest points), radius
      float Rsq[8];
#pragma unroll
      for (int o = 0; o < 8; ++o) {
        const float ox = (o & 4) ? hq : -hq, oy = (o & 2) ? hq : -hq, oz = (o & 1) ? hq : -hq;
        float dmin2 = INFINITY;
#pragma unroll
        for (int q = 0; q < 9; ++q) {
          int li;
          if (q == 8) {
            li = 27 + o;
          } else {
            const int ix = ((o >> 2) & 1) + ((q >> 2) & 1), iy = ((o >> 1) & 1) + ((q >> 1) & 1), iz = (o & 1) + (q & 1);
            li = ix * 9 + iy * 3 + iz;
          }
          const Rel d = Rel{lat[li].x - ox, lat[li].y - oy, lat[li].z - oz};
          dmin2 = fminf(dmin2, far2(d, hc));
        }
        Rsq[o] = list_radius2(dmin2, b.capm);
      }
      // keep masks per list point
      for (int k = lane; k < n; k += 64) {
        const float4 p = ldg4(c.pts, P.pool[ph.x + k]);
        const Rel a = rel(PB, p.x, p.y, p.z);
        unsigned mk = 0;
#pragma unroll
        for (int o = 0; o < 8; ++o) {
          const float ox = (o & 4) ? hq : -hq, oy = (o & 2) ? hq : -hq, oz = (o & 1) ? hq : -hq;
          const Rel ac = Rel{a.x - ox, a.y - oy, a.z - oz};
          bool keep = bd2(ac, hc) <= Rsq[o];
#pragma unroll
          for (int q = 0; q < 9; ++q) {
            int li;
            if (q == 8) {
              li = 27 + o;
            } else {
              const int ix = ((o >> 2) & 1) + ((q >> 2) & 1), iy = ((o >> 1) & 1) + ((q >> 1) & 1), iz = (o & 1) + (q & 1);
              li = ix * 9 + iy * 3 + iz;
            }
            const Rel d = Rel{lat[li].x - ox, lat[li].y - oy, lat[li].z - oz};
            keep = keep && !dominated(ac, d, hc);
          }
          mk |= keep ? (1u << o) : 0u;
        }
        msk[k] = (unsigned char)mk;
      }
      __builtin_amdgcn_wave_barrier();
      for (int k0 = 0; k0 < n; k0 += 64) {
        const int k = k0 + lane;
        const unsigned mk = k < n ? msk[k] : 0u;
#pragma unroll
        for (int o = 0; o < 8; ++o) cnt[o] += __popcll(__ballot((mk >> o) & 1u));
      }
    }
    int tot = 0, cm = 0;
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      tot += cnt[o];
      cm = max(cm, cnt[o]);
    }
    unsigned base = 0;
    if (tot > 0) {
      base = bump.take((unsigned)tot, pool_ctr(b, level), L.pool_cap, shard);
      if (base == ~0u) {
        if (lane == 0) atomicOr(b.ctr + kCtrPoolFull * 32, 1u);
        continue;
      }
      // children lists, one after another
      unsigned at = base;
#pragma unroll 1
      for (int o = 0; o < 8; ++o) {
        if (cnt[o] == 0) continue;
        int w = 0;
        for (int k0 = 0; k0 < n; k0 += 64) {
          const int k = k0 + lane;
          const bool keep = k < n && ((msk[k] >> o) & 1u);
          const unsigned long long bal = __ballot(keep);
          if (keep) L.pool[at + w + mbcnt(bal)] = P.pool[ph.x + k];
          w += __popcll(bal);
        }
        at += (unsigned)cnt[o];
      }
    }
    if (lane < 8) {
      const int o = lane;
      unsigned off = base;
      for (int q = 0; q < o; ++q) off += (unsigned)cnt[q];
      const int fx = 2 * px + ((o >> 2) & 1), fy = 2 * py + ((o >> 1) & 1), fz = 2 * pz + (o & 1);
      const int f = (fx * m + fy) * m + fz;
      L.hdr[(size_t)s * m * m * m + f] = make_uint2(off, (unsigned)cnt[o]);
    }
    if (lane == 0) atomicMax(L.cmax + s, cm);
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------------------
// K7e: emission.  count: one wave per final (level, slot): its list entries
// (fine cells whose list exceeds lcap store none) and fine cells.
__global__ __launch_bounds__(64 * kCgWaves) void k_cg_emit_count(const CgBuild* __restrict__ bp, int level,
                                                                  const int* __restrict__ finals, int nfinals,
                                                                  unsigned* __restrict__ ent_n, unsigned* __restrict__ fine_n) {
  const CgBuild& b = *bp;
  const int lane = lane_id();
  const int wave = blockIdx.x * kCgWaves + (threadIdx.x >> 6);
  if (wave >= nfinals) return;
  const int s = finals[wave];
  const int nf = 1 << (3 * level);
  const uint2* hdr = b.lv[level].hdr + (size_t)s * nf;
  unsigned t = 0;
  for (int f = lane; f < nf; f += 64) {
    const unsigned k = hdr[f].y;
    t += k <= (unsigned)b.lcap ? k : 0u;
  }
  for (int m = 32; m >= 1; m >>= 1) t += __shfl_xor(t, m);
  if (lane == 0) {
    ent_n[wave] = t;
    fine_n[wave] = (unsigned)nf;
  }
}

// write: dir entry, fine table and point copies of one final per wave;
// ent_off / fine_off: the exclusive scans of emit_count's outputs, + bases
__global__ __launch_bounds__(64 * kCgWaves) void k_cg_emit_write(const CgBuild* __restrict__ bp, int level,
                                                                  const int* __restrict__ finals, int nfinals,
                                                                  const unsigned* __restrict__ ent_off,
                                                                  const unsigned* __restrict__ fine_off,
                                                                  unsigned ent_base, unsigned fine_base) {
  const CgBuild& b = *bp;
  const CloudDev& c = b.tgt;
  const int lane = lane_id();
  const int wave = blockIdx.x * kCgWaves + (threadIdx.x >> 6);
  if (wave >= nfinals) return;
  const int s = finals[wave];
  const int bi = level == 0 ? s : b.lv[level].slot_band[s];
  const int nf = 1 << (3 * level);
  const CgLevel L = b.lv[level];
  const uint2* hdr = L.hdr + (size_t)s * nf;
  const unsigned fb = fine_base + fine_off[wave];
  unsigned eb = ent_base + ent_off[wave];
  // level 0: the one list inline in the directory (no fine-table load in the lookup)
  if (lane == 0 && level > 0) b.dir[b.band[bi]] = ((unsigned long long)level << 62) | fb;
  for (int f0 = 0; f0 < nf; f0 += 64) {
    const int f = f0 + lane;
    uint2 h = make_uint2(0u, 0u);
    if (f < nf) h = hdr[f];
    const bool stored = f < nf && h.y <= (unsigned)b.lcap;
    const unsigned k = stored ? h.y : 0u;
    // exclusive prefix of the counts over the 64 lanes
    unsigned incl = k;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    const unsigned ex = incl - k;
    if (f < nf) {
      b.fine[fb + f] = stored ? make_uint2(eb + ex, k) : make_uint2(0u, kCgFineFallback);
      if (!stored) atomicAdd(b.ctr + kCtrFineFb * 32, 1u);
      if (level == 0) b.dir[b.band[bi]] = stored ? (((unsigned long long)k << 32) | (eb + ex)) : kCgFallback;
    }
    // copies: this chunk's lists, one fine cell after another
    const unsigned tot = __shfl(incl, 63);
    for (int j = 0; j < 64; ++j) {
      const unsigned kj = __shfl(k, j);
      if (kj == 0u) continue;
      const unsigned srcoff = __shfl(h.x, j), dst = eb + __shfl(ex, j);
      for (unsigned t = lane; t < kj; t += 64) {
        const int pos = (int)L.pool[srcoff + t];
        const float4 p = ldg4(c.pts, pos);
        b.ent[dst + t] = make_float4(p.x, p.y, p.z, __int_as_float(pos));
      }
    }
    eb += tot;
  }
}

// ---------------------------------------------------------------------------
// launchers
static int cdiv_l(long a, long b) { return (int)((a + b - 1) / b); }

void launch_cg_occ(hipStream_t s, const CgBuild* db, int n) {
  k_cg_occ<<<cdiv_l(n, 256), 256, 0, s>>>(db, n);
}
void launch_cg_prop(hipStream_t s, const CgBuild* db, int axis, const int* in, int* out, long ncells) {
  k_cg_prop<<<cdiv_l(ncells, 256), 256, 0, s>>>(db, axis, in, out, ncells);
}
void launch_cg_dir_fill(hipStream_t s, unsigned long long* dir, const int* band, long ncells, unsigned long long outside) {
  k_cg_dir_fill<<<cdiv_l(ncells, 256), 256, 0, s>>>(dir, band, ncells, outside);
}
void launch_cg_band_flags(hipStream_t s, const CgBuild* db, const int* band, unsigned char* flags, long nblocked) {
  k_cg_band_flags<<<cdiv_l(nblocked, 256), 256, 0, s>>>(db, band, flags, nblocked);
}
void launch_cg_centers(hipStream_t s, CgBuild* db, int nband) {
  k_cg_centers<<<cdiv_l(nband, 256), 256, 0, s>>>(db, nband);
}
void launch_cg_coarse(hipStream_t s, const CgBuild* db, int nband) {
  const int blocks = std::max(1, std::min(cdiv_l(nband, kCgWaves), 2048));
  k_cg_coarse<<<blocks, 64 * kCgWaves, 0, s>>>(db, nband);
}
void launch_cg_decide(hipStream_t s, CgBuild* db, int level, int nslots, unsigned char* fl_final, unsigned char* fl_next) {
  k_cg_decide<<<cdiv_l(nslots, 256), 256, 0, s>>>(db, level, nslots, fl_final, fl_next);
}
void launch_cg_slots(hipStream_t s, CgBuild* db, int level, int nslots) {
  k_cg_slots<<<cdiv_l(nslots, 256), 256, 0, s>>>(db, level, nslots);
}
void launch_cg_refine(hipStream_t s, const CgBuild* db, int level, int nslots) {
  const long items = (long)nslots << (3 * (level - 1));
  const int blocks = std::max(1, std::min(cdiv_l(items, kCgWaves), 2048));
  k_cg_refine<<<blocks, 64 * kCgWaves, 0, s>>>(db, level, nslots);
}
void launch_cg_emit_count(hipStream_t s, const CgBuild* db, int level, const int* finals, int nfinals, unsigned* ent_n,
                          unsigned* fine_n) {
  k_cg_emit_count<<<cdiv_l(nfinals, kCgWaves), 64 * kCgWaves, 0, s>>>(db, level, finals, nfinals, ent_n, fine_n);
}
void launch_cg_emit_write(hipStream_t s, const CgBuild* db, int level, const int* finals, int nfinals,
                          const unsigned* ent_off, const unsigned* fine_off, unsigned ent_base, unsigned fine_base) {
  k_cg_emit_write<<<cdiv_l(nfinals, kCgWaves), 64 * kCgWaves, 0, s>>>(db, level, finals, nfinals, ent_off, fine_off,
                                                                       ent_base, fine_base);
}

}  // namespace ddlo
