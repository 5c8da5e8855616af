// tietree.hip — a slab shard's part of the whole submap's nanoflann tree
// (DESIGN.md §5 "Slab shards"): the tie order of update_correspondences'
// 1-NN (reference include/nano_gicp/impl/nano_gicp_impl.hpp:249-258) is the
// order in which nanoflann's depth-first walk of the WHOLE submap's tree
// (nanoflann_impl.hpp:1495-1566, built by divideTree :987-1043) meets
// equidistant points.  A slab rank holds only its slab + halo of the submap.
//
// Restriction: the tree with every point outside the rank's set removed,
// subtrees left empty by that becoming empty leaves.  For a query the rank
// owns whose nearest distance d is below the correspondence bound, every
// point at distance <= d lies in the halo (it is within d of an owned query
// along the slab axis), so the restricted walk meets the same points at
// distance <= d in the same relative order, with the same cut decisions at
// every node it keeps.  Removing points only raises the worst distance seen
// at any moment, so no tied point's subtree is pruned that the whole walk
// visits, and the first tied point met -- the reference's answer -- is the
// same.  Size: O(rank's points), not O(submap).
//
// Device work (the builder's whole tree T, n points, node slots [0, cap)):
//   k_tp_mark        local_index -> mark[whole index] = local index
//   k_tp_keep        keep flag per vind position; exclusive scan -> ppos
//   k_tp_up          every leaf holding a kept point flags its ancestors
//   k_tp_emit        a node is emitted if its parent is flagged (root: if
//                    anything is kept); exclusive scan -> new node ids
//   k_tp_write       emitted nodes (flagged: children renumbered; a leaf:
//                    its kept range; else an empty leaf) and the kept
//                    points in vind order, w = local index
// Node slots a build never wrote are zero (the builder clears the node
// buffer first); a slot is a node iff its parent names it as a child.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "gicp_types.hpp"
#include "launch.hpp"

namespace ddlo {

namespace {

__device__ __forceinline__ bool tp_valid(const NfNode* __restrict__ nodes, int cap, int i) {
  if (i == 0) return true;
  const int p = nodes[i].parent;
  if (p < 0 || p >= cap || p == i) return false;
  const NfNode q = nodes[p];
  return q.feat >= 0 && (q.c1 == i || q.c2 == i);
}

__global__ __launch_bounds__(256) void k_tp_mark(const int* __restrict__ local_index, int n_local, int n,
                                                 int* __restrict__ mark, int* __restrict__ err) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_local) return;
  const int w = local_index[i];
  if (w < 0 || w >= n) {
    atomicOr(err, 1);
    return;
  }
  mark[w] = i;
}

__global__ __launch_bounds__(256) void k_tp_keep(NfTreeDev t, const int* __restrict__ mark, unsigned* __restrict__ keep) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p > t.n) return;
  keep[p] = p < t.n ? (mark[__float_as_int(t.vpts[p].w)] >= 0 ? 1u : 0u) : 0u;
}

__global__ __launch_bounds__(256) void k_tp_up(NfTreeDev t, int cap, const unsigned* __restrict__ ppos,
                                               unsigned* __restrict__ flag, int* __restrict__ err) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  const NfNode nd = t.nodes[i];
  if (nd.feat != -1 || !tp_valid(t.nodes, cap, i)) return;
  if (nd.c1 < 0 || nd.c2 > t.n || nd.c1 > nd.c2) {
    atomicOr(err, 2);
    return;
  }
  if (ppos[nd.c2] == ppos[nd.c1]) return;
  flag[i] = 1u;
  int p = i == 0 ? -1 : nd.parent;
  for (int guard = 0; p >= 0 && guard < 4096; ++guard) {
    if (atomicOr(&flag[p], 1u)) return;   // an earlier leaf flagged the rest of the path
    p = p == 0 ? -1 : t.nodes[p].parent;
  }
  if (p >= 0) atomicOr(err, 4);
}

__global__ __launch_bounds__(256) void k_tp_emit(NfTreeDev t, int cap, const unsigned* __restrict__ flag,
                                                 unsigned* __restrict__ emit) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > cap) return;
  unsigned e = 0;
  if (i < cap) e = i == 0 ? flag[0] : ((tp_valid(t.nodes, cap, i) && flag[t.nodes[i].parent]) ? 1u : 0u);
  emit[i] = e;
}

__global__ __launch_bounds__(256) void k_tp_write(NfTreeDev t, int cap, const unsigned* __restrict__ flag,
                                                  const unsigned* __restrict__ emit_pos, const unsigned* __restrict__ ppos,
                                                  NfNode* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap || emit_pos[i + 1] == emit_pos[i]) return;
  const NfNode nd = t.nodes[i];
  NfNode o = nd;
  o.parent = i == 0 ? -1 : (int)emit_pos[nd.parent];
  o.pad0 = o.pad1 = 0;
  if (nd.feat < 0) {   // a leaf: its kept points (possibly none)
    o.c1 = (int)ppos[nd.c1];
    o.c2 = (int)ppos[nd.c2];
    o.feat = -1;
  } else if (flag[i]) {
    o.c1 = (int)emit_pos[nd.c1];
    o.c2 = (int)emit_pos[nd.c2];
  } else {             // a subtree without kept points: an empty leaf
    o.c1 = o.c2 = 0;
    o.feat = -1;
  }
  out[emit_pos[i]] = o;
}

__global__ __launch_bounds__(256) void k_tp_points(NfTreeDev t, const int* __restrict__ mark,
                                                   const unsigned* __restrict__ ppos, float4* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= t.n || ppos[p + 1] == ppos[p]) return;
  float4 v = t.vpts[p];
  v.w = __int_as_float(mark[__float_as_int(v.w)]);
  out[ppos[p]] = v;
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
inline size_t al256(size_t b) { return (b + 255) / 256 * 256; }

}  // namespace

size_t tie_prune_scratch_bytes(int n, int cap) {
  size_t cub_a = 0, cub_b = 0;
  unsigned* z = nullptr;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, cub_a, z, z, n + 1);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, cub_b, z, z, cap + 1);
  return al256(sizeof(int) * (size_t)n) + al256(sizeof(unsigned) * ((size_t)n + 1)) +
         2 * al256(sizeof(unsigned) * ((size_t)cap + 1)) + al256(std::max(cub_a, cub_b)) + 256;
}

// The restriction of tree t to the points local_index names (device array,
// n_local entries).  Outputs stay on the device: out_nodes (cap entries),
// out_pts (n_local), counts[0] = kept points, counts[1] = emitted nodes,
// counts[2] = error bits.  scratch: tie_prune_scratch_bytes(t.n, cap).
hipError_t launch_tie_prune(hipStream_t s, const NfTreeDev& t, int cap, const int* local_index, int n_local,
                            void* scratch, NfNode* out_nodes, float4* out_pts, unsigned* counts) {
  const int n = t.n;
  char* u = static_cast<char*>(scratch);
  int* mark = reinterpret_cast<int*>(u);
  u += al256(sizeof(int) * (size_t)n);
  unsigned* ppos = reinterpret_cast<unsigned*>(u);
  u += al256(sizeof(unsigned) * ((size_t)n + 1));
  unsigned* flag = reinterpret_cast<unsigned*>(u);
  u += al256(sizeof(unsigned) * ((size_t)cap + 1));
  unsigned* epos = reinterpret_cast<unsigned*>(u);
  u += al256(sizeof(unsigned) * ((size_t)cap + 1));
  void* cub_tmp = u;
  size_t cub_a = 0, cub_b = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, cub_a, ppos, ppos, n + 1, s);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveSum(nullptr, cub_b, epos, epos, cap + 1, s);
  if (e != hipSuccess) return e;
  int* err = reinterpret_cast<int*>(counts + 2);
  if ((e = hipMemsetAsync(counts, 0, 4 * sizeof(unsigned), s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(mark, 0xff, sizeof(int) * (size_t)n, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(flag, 0, sizeof(unsigned) * ((size_t)cap + 1), s)) != hipSuccess) return e;
  if (n_local > 0) k_tp_mark<<<cdiv(n_local, 256), 256, 0, s>>>(local_index, n_local, n, mark, err);
  k_tp_keep<<<cdiv(n + 1, 256), 256, 0, s>>>(t, mark, ppos);
  if ((e = hipcub::DeviceScan::ExclusiveSum(cub_tmp, cub_a, ppos, ppos, n + 1, s)) != hipSuccess) return e;
  k_tp_up<<<cdiv(cap, 256), 256, 0, s>>>(t, cap, ppos, flag, err);
  k_tp_emit<<<cdiv(cap + 1, 256), 256, 0, s>>>(t, cap, flag, epos);
  if ((e = hipcub::DeviceScan::ExclusiveSum(cub_tmp, cub_b, epos, epos, cap + 1, s)) != hipSuccess) return e;
  k_tp_write<<<cdiv(cap, 256), 256, 0, s>>>(t, cap, flag, epos, ppos, out_nodes);
  k_tp_points<<<cdiv(n, 256), 256, 0, s>>>(t, mark, ppos, out_pts);
  if ((e = hipMemcpyAsync(counts, ppos + n, sizeof(unsigned), hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(counts + 1, epos + cap, sizeof(unsigned), hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
  return hipGetLastError();
}

}  // namespace ddlo
