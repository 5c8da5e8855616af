// nftree.hpp — nanoflann's own kd-tree, rebuilt on the device, and its exact
// search, used ONLY to break exact distance ties the way the reference does.
//
// The GPU searches (search.hpp, nn_tasks.hpp) return the exact k nearest
// distances with ties broken by the lower Morton position.  nanoflann breaks a
// tie by traversal order instead: KNNResultSet::addPoint shifts only past a
// strictly larger distance and a leaf inserts only below the worst distance
// (reference include/nano_gicp/impl/nanoflann_impl.hpp:205-237, :1509), so
// among equal distances the point its depth-first walk (:1495-1566) meets
// first wins.  That order is a function of nanoflann's tree: middleSplit_'s
// cut (:1045-1096), planeSplit's two in-place Hoare passes (:1107-1143) and
// the recursion of divideTree (:987-1043) with leaf_max_size 100
// (include/nano_gicp/nanoflann.hpp:119).  nftree.hip builds exactly that tree
// on the device; the kernels flag the (rare) queries whose answer contains a
// tie and only those are re-run here with the literal nanoflann search.
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>

#include "gicp_types.hpp"

namespace ddlo {

constexpr int kNfLeafMax = 100;   // KDTreeSingleIndexAdaptorParams(100), nanoflann.hpp:119
constexpr int kNfStack = 192;     // search / build recursion depth bound (a deeper tree fails the build)

// KNNResultSet<float, int> (nanoflann_impl.hpp:161-242), default tie rule
// (NANOFLANN_FIRST_MATCH undefined): strict '>' shift.
template <int KMAX>
struct NfResult {
  float d[KMAX];
  int ix[KMAX];
  int count, cap;
  __device__ __forceinline__ void init(int k) {
    cap = k;
    count = 0;
    d[k - 1] = FLT_MAX;   // (std::numeric_limits<DistanceType>::max)()
  }
  __device__ __forceinline__ float worst() const { return d[cap - 1]; }
  __device__ __forceinline__ void add(float dist, int index) {
    int i;
    for (i = count; i > 0; --i) {
      if (d[i - 1] > dist) {
        if (i < cap) {
          d[i] = d[i - 1];
          ix[i] = ix[i - 1];
        }
      } else {
        break;
      }
    }
    if (i < cap) {
      d[i] = dist;
      ix[i] = index;
    }
    if (count < cap) count++;
  }
};

// findNeighbors (:1365-1384) + computeInitialDistances (:1145-1164) +
// searchLevel (:1495-1566) with eps = 0 (epsError = 1.0f), recursion as an
// explicit stack.  Float arithmetic in the reference's order (the file is
// compiled with -ffp-contract=off): L2_Simple_Adaptor::evalMetric sums
// diff*diff from dimension 0 (:508-517), accum_dist = (a-b)*(a-b) (:520-523).
// Returns false if the tree is deeper than kNfStack (never for real clouds).
template <int KMAX>
__device__ bool nf_search(const NfTreeDev& t, float qx, float qy, float qz, NfResult<KMAX>& rs) {
  const float q[3] = {qx, qy, qz};
  const float4 rlo = t.box[0], rhi = t.box[1];
  const float lo[3] = {rlo.x, rlo.y, rlo.z}, hi[3] = {rhi.x, rhi.y, rhi.z};
  float dists[3] = {0.f, 0.f, 0.f};
  float distsq = 0.f;
  for (int i = 0; i < 3; ++i) {
    if (q[i] < lo[i]) {
      dists[i] = (q[i] - lo[i]) * (q[i] - lo[i]);
      distsq += dists[i];
    }
    if (q[i] > hi[i]) {
      dists[i] = (q[i] - hi[i]) * (q[i] - hi[i]);
      distsq += dists[i];
    }
  }
  // frame: node, its mindistsq, the saved dists[idx] (state 2), state
  int fn[kNfStack];
  float fm[kNfStack], fd[kNfStack];
  unsigned char fs[kNfStack];
  int sp = 1;
  fn[0] = 0;
  fm[0] = distsq;
  fs[0] = 0;
  while (sp > 0) {
    const int f = sp - 1;
    const NfNode nd = t.nodes[fn[f]];
    if (nd.feat < 0) {   // leaf (child1 == child2 == NULL)
      const float worst = rs.worst();
      for (int i = nd.c1; i < nd.c2; ++i) {
        const float4 p = t.vpts[i];
        float r = 0.f;
        float diff = q[0] - p.x;
        r += diff * diff;
        diff = q[1] - p.y;
        r += diff * diff;
        diff = q[2] - p.z;
        r += diff * diff;
        if (r < worst) rs.add(r, __float_as_int(p.w));
      }
      --sp;
      continue;
    }
    const int idx = nd.feat;
    const float val = q[idx];
    const float diff1 = val - nd.divlow;
    const float diff2 = val - nd.divhigh;
    int best, other;
    float cut_dist;
    if ((diff1 + diff2) < 0) {
      best = nd.c1;
      other = nd.c2;
      cut_dist = (val - nd.divhigh) * (val - nd.divhigh);
    } else {
      best = nd.c2;
      other = nd.c1;
      cut_dist = (val - nd.divlow) * (val - nd.divlow);
    }
    if (fs[f] == 0) {   // descend into the best child first
      if (sp >= kNfStack) return false;
      fs[f] = 1;
      fn[sp] = best;
      fm[sp] = fm[f];
      fs[sp] = 0;
      ++sp;
      continue;
    }
    if (fs[f] == 1) {
      const float dst = dists[idx];
      const float mind = fm[f] + cut_dist - dst;
      dists[idx] = cut_dist;
      fd[f] = dst;
      fs[f] = 2;
      if (mind * 1.0f <= rs.worst()) {
        if (sp >= kNfStack) return false;
        fn[sp] = other;
        fm[sp] = mind;
        fs[sp] = 0;
        ++sp;
        continue;
      }
    }
    dists[idx] = fd[f];   // state 2: both children done
    --sp;
  }
  return true;
}

// The same search with one wavefront per query (the tie resolvers): the walk
// is wave-uniform (frames in LDS), a leaf's points are measured 64 at a time
// and its candidates (dist < the worst distance read once at the leaf,
// :1509) inserted in leaf order; lane j < k holds the j-th result.  The
// result set is KNNResultSet's: an insertion goes after every kept entry
// of equal or smaller distance and falls off past slot k - 1.
struct NfWaveStack {
  int fn[kNfStack];
  float fm[kNfStack], fd[kNfStack];
  int fs[kNfStack];
};

__device__ __forceinline__ float nf_sel3(float a, float b, float c, int i) { return i == 0 ? a : (i == 1 ? b : c); }

__device__ inline bool nf_search_wave(const NfTreeDev& t, float qx, float qy, float qz, int k, NfWaveStack* S,
                                      float* out_d, int* out_ix) {
  const int lane = __lane_id();
  const float4 rlo = t.box[0], rhi = t.box[1];
  float d0 = 0.f, d1 = 0.f, d2 = 0.f;   // dists[3]
  float distsq = 0.f;
  if (qx < rlo.x) { d0 = (qx - rlo.x) * (qx - rlo.x); distsq += d0; }
  if (qx > rhi.x) { d0 = (qx - rhi.x) * (qx - rhi.x); distsq += d0; }
  if (qy < rlo.y) { d1 = (qy - rlo.y) * (qy - rlo.y); distsq += d1; }
  if (qy > rhi.y) { d1 = (qy - rhi.y) * (qy - rhi.y); distsq += d1; }
  if (qz < rlo.z) { d2 = (qz - rlo.z) * (qz - rlo.z); distsq += d2; }
  if (qz > rhi.z) { d2 = (qz - rhi.z) * (qz - rhi.z); distsq += d2; }
  float kd = FLT_MAX;   // this lane's result slot
  int kx = -1;
  int count = 0;
  int sp = 1;
  S->fn[0] = 0;
  S->fm[0] = distsq;
  S->fs[0] = 0;
  while (sp > 0) {
    const int f = sp - 1;
    const NfNode nd = t.nodes[S->fn[f]];
    const float worst = count < k ? FLT_MAX : __shfl(kd, k - 1);
    if (nd.feat < 0) {   // leaf
      for (int b = nd.c1; b < nd.c2; b += 64) {
        const int i = b + lane;
        float r = FLT_MAX;
        int ip = -1;
        bool cand = false;
        if (i < nd.c2) {
          const float4 p = t.vpts[i];
          r = 0.f;
          float diff = qx - p.x;
          r += diff * diff;
          diff = qy - p.y;
          r += diff * diff;
          diff = qz - p.z;
          r += diff * diff;
          ip = __float_as_int(p.w);
          cand = r < worst;
        }
        unsigned long long m = __ballot(cand);
        while (m) {
          const int bl = __ffsll((long long)m) - 1;
          m &= m - 1;
          const float dn = __shfl(r, bl);
          const int xn = __shfl(ip, bl);
          const int pos = __popcll(__ballot(lane < count && kd <= dn));
          const float ud = __shfl_up(kd, 1);
          const int ux = __shfl_up(kx, 1);
          if (pos < k && lane < k) {
            if (lane == pos) {
              kd = dn;
              kx = xn;
            } else if (lane > pos) {
              kd = ud;
              kx = ux;
            }
          }
          if (count < k) ++count;
        }
      }
      --sp;
      continue;
    }
    const int idx = nd.feat;
    const float val = nf_sel3(qx, qy, qz, idx);
    const float diff1 = val - nd.divlow;
    const float diff2 = val - nd.divhigh;
    int best, other;
    float cut_dist;
    if ((diff1 + diff2) < 0) {
      best = nd.c1;
      other = nd.c2;
      cut_dist = (val - nd.divhigh) * (val - nd.divhigh);
    } else {
      best = nd.c2;
      other = nd.c1;
      cut_dist = (val - nd.divlow) * (val - nd.divlow);
    }
    const int st = S->fs[f];
    if (st == 0) {
      if (sp >= kNfStack) {
        *out_ix = -2;
        return false;
      }
      S->fs[f] = 1;
      S->fn[sp] = best;
      S->fm[sp] = S->fm[f];
      S->fs[sp] = 0;
      ++sp;
      continue;
    }
    if (st == 1) {
      const float dst = nf_sel3(d0, d1, d2, idx);
      const float mind = S->fm[f] + cut_dist - dst;
      if (idx == 0) d0 = cut_dist;
      else if (idx == 1) d1 = cut_dist;
      else d2 = cut_dist;
      S->fd[f] = dst;
      S->fs[f] = 2;
      if (mind * 1.0f <= worst) {
        if (sp >= kNfStack) {
          *out_ix = -2;
          return false;
        }
        S->fn[sp] = other;
        S->fm[sp] = mind;
        S->fs[sp] = 0;
        ++sp;
        continue;
      }
    }
    const float rs = S->fd[f];   // state 2: both children done
    if (idx == 0) d0 = rs;
    else if (idx == 1) d1 = rs;
    else d2 = rs;
    --sp;
  }
  *out_d = kd;
  *out_ix = kx;
  return count >= k;
}

}  // namespace ddlo
