// launch.hpp — host-callable launchers of the kernels in kernels.hip.  The
// host runtime (capi.hip) only sees these plain functions.
#pragma once
#include <hip/hip_runtime.h>

#include "gicp_types.hpp"

namespace ddlo {

void launch_pack_bbox(hipStream_t s, const unsigned char* raw, size_t stride, int n, float4* out, float* partial,
                      int* nonfinite, int nblocks);
void launch_bbox_final(hipStream_t s, const float* partial, int nparts, float* quant);
void launch_morton(hipStream_t s, const float4* pts, int n, const float* quant, unsigned long long* keys, int* vals);
void launch_gather(hipStream_t s, const float4* raw, const int* perm, int n, int npad, float4* sorted, int* inv_perm);
void launch_key_dir(hipStream_t s, const unsigned long long* keys, int n, int* dir);
// the sorted points' per-leaf SoA copy (nleaves whole leaves) and the leaves' boxes (real points only)
void launch_leaf_soa_boxes(hipStream_t s, const float4* pts, int n, int nleaves, float* soa, float4* lo, float4* hi);
void launch_level_boxes(hipStream_t s, const float4* clo, const float4* chi, int nchild, int nparent, float4* plo,
                        float4* phi);
// returns false if k is unsupported (> 64)
// redo: nullptr = every point, else only the 64-point groups flagged 1
// ties (optional): sorted positions whose k-neighbourhood has an exact
// distance tie at its boundary are appended to ties->list (nftree.hip
// resolves them in nanoflann's order)
struct TieList {
  int* list;
  int* count;
  int cap = 0;   // list capacity: an append beyond it is dropped and the resolver reports the overflow
  __device__ __forceinline__ void push(int i) const {
    const int slot = atomicAdd(count, 1);
    if (slot < cap) list[slot] = i;
  }
};
bool launch_covariances(hipStream_t s, const CloudDev& c, int k, int method, double* cov6, const unsigned char* redo,
                        TieList ties = TieList{nullptr, nullptr});
// task-based kNN-k covariances (knn_tasks.hip), k <= 32; groups it flags in
// j.redo must then be recomputed with launch_covariances(..., j.redo)
bool launch_knn_covariances(hipStream_t s, const KnnJob& j, int tgt_upper);
int knn_task_cap_per_region(int n);
// ties: query rows whose answer holds an exact distance tie (inside the k or
// at its boundary) are listed for the nanoflann-order resolver
bool launch_knn_query(hipStream_t s, const CloudDev& c, const float4* q, int nq, int k, int* out_idx, float* out_d,
                      TieList ties = TieList{nullptr, nullptr});
void launch_cov_import(hipStream_t s, const double* in, int layout, int n, const int* inv_perm, double* cov6);
void launch_cov_export(hipStream_t s, const double* cov6, int layout, int n, const int* perm, double* out);
// tietree.hip: a slab shard's restriction of the whole submap's nanoflann tree
size_t tie_prune_scratch_bytes(int n, int cap);
hipError_t launch_tie_prune(hipStream_t s, const NfTreeDev& t, int cap, const int* local_index, int n_local,
                            void* scratch, NfNode* out_nodes, float4* out_pts, unsigned* counts);
void launch_align_init(hipStream_t s, AlignJob* job, const AlignJob* job_src);
// tgt_upper: number of upper-level (>= 1) boxes of the target (LDS cache size)
// Launch geometry of one linearize (grids, upper-box LDS cache), bucketed by
// cloud size; part of the chunk-graph key.
struct LinGeom {
  int seed_blocks, collect_blocks, scan_blocks, mom_blocks, lds_boxes, lookup_blocks;
  bool fuse_lm = false;   // the LM step runs in the moment kernel's last block (no k_lm_step launch)
  AlignState* state = nullptr;   // the job's state (job->state), a kernel argument of the moment kernel
  bool grid = false;      // the target's candidate cells answer the search first (k_cell_lookup)
  bool grid_walk = true;  // ... and some of its cells have no list: the walk kernel follows the lookup
};
bool lm_fusion_enabled(bool lookup);   // unsharded aligns on the one-kernel lookup path (DDLO_FUSE_LM: dev A/B)
LinGeom linearize_geometry(int nsrc, int tgt_upper);
// publish: with g.fuse_lm, the host-mapped state slot the fused LM step publishes to (or nullptr)
void launch_linearize(hipStream_t s, const AlignJob* job, const LinGeom& g, AlignState* publish = nullptr);
int search_queries_per_wave();
int task_cap_per_region(int nsrc);   // task-list slots per region for nsrc source points
int moment_blocks(int nsrc);  // slab rows written by the moment kernel
// st / slab / nblocks / premom: the job's state, slab rows and (sharded) all-reduced moments, as
// kernel arguments (the state and slab loads then need no job load first)
void launch_lm_step(hipStream_t s, const AlignJob* job, AlignState* st, const double* slab, int nblocks,
                    const double* premom, AlignState* publish);
void launch_mom_reduce(hipStream_t s, const AlignJob* job);  // sharded align: slab -> job->mom
void launch_residuals(hipStream_t s, const AlignJob* job, int nsrc, double* out);
void launch_residual_image(hipStream_t s, const float4* pts, const int* perm, const int* inv_perm, int n,
                           const double* residual, double tmin, double tmax, int W, int H, int* winner, float* img,
                           float* xyz);
void launch_transform(hipStream_t s, const float4* pts, int n, const int* perm, const float* T16, float* out,
                      size_t stride_floats);
void launch_export_corr(hipStream_t s, const AlignJob* job, int nsrc, int* corr, float* sqd);

// nftree.hip: nanoflann's kd-tree on the device (tie order) and the tie resolvers
NfSizes nf_sizes(int n);
// sorted_pts: the cloud's Morton-sorted points (w = original index)
// stop >= 0: run only that many big levels (diagnostics)
void launch_nf_build(hipStream_t s, const NfBuild& hb, const NfBuild* db, int stop = -1);
// *db = b on the stream (the descriptor the build kernels read)
void launch_nf_set_desc(hipStream_t s, const NfBuild& b, NfBuild* db);
// status = {build error bits, node count}; nodes: 4 ints per node (c1, c2, feat, parent), f: divlow, divhigh
void launch_nf_export(hipStream_t s, const NfTreeDev& t, const int* status, int cap, int* vind, int* nodes, float* f);
// re-run the listed (tied) queries with nanoflann's search; status: the
// tree build's error bits (nonzero: nothing resolved, *err |= 2); *err |= 1
// on a failed search
bool launch_nf_resolve_cov(hipStream_t s, const NfTreeDev& t, const CloudDev& c, TieList ties, int k, int method,
                           double* cov6, const int* status, int* err);
bool launch_nf_resolve_knn(hipStream_t s, const NfTreeDev& t, const float4* q, TieList ties, int k, int* out_idx,
                           float* out_d, const int* status, int* err);
// the same re-run on the cloud's partial tree (nftree_build partial_levels):
// each listed query's nanoflann search walks the built top levels and splits
// the stubs it enters lazily, on a private copy of their vind ranges (one
// workgroup per query, wgs workgroups; scratch: nf_lazy_bytes(c.n, wgs)).
// cov6 != nullptr: the cloud's own tied points get their covariances; else
// rows of q their (out_idx, out_d).  *err |= 1 depth, 2 build, 4 fewer than k,
// 16 pairing check.
size_t nf_lazy_bytes(int n, int wgs);
bool launch_nf_lazy(hipStream_t s, const NfTreeDev& t, const CloudDev& c, const float4* q, TieList ties, int k,
                    int method, double* cov6, int* out_idx, float* out_d, void* scratch, int wgs, const int* status,
                    int* err);
void launch_cov_remap(hipStream_t s, const double* old_cov6, const int* old_inv_perm, const int* new_perm, int n,
                      double* cov6);

// preprocess.hip (odometry driver): see the kernels there for the reference
// filters they restate.  Scratch sizes: *_tmp_bytes (hipcub temporaries).
void launch_pack4(hipStream_t s, const unsigned char* raw, size_t stride, int n, float4* out);
// pin: pinned host ints for the count read-back (crop_box 2, voxel_grid 16)
int crop_box(hipStream_t s, const float4* in, int n, float size, float4* out, int* keep, int* pos, void* tmp,
             size_t tmp_bytes, int* count_host, int* pin);
size_t crop_box_tmp_bytes(int n);
// crop > 0: the crop box (points inside [-crop, crop]^3 removed) folded into the same pass
int voxel_grid(hipStream_t s, const float4* in, int n, float leaf, float4* out, int* scratch, void* tmp, size_t tmp_bytes,
               int* count_host, float crop, int* pin);
size_t voxel_tmp_bytes(int n);
constexpr size_t voxel_scratch_ints(int n) { return 7 * (size_t)n + 16 + 6 * 64; }
void median_range_async(hipStream_t s, const float4* in, int n, float* d, float* result, void* tmp, size_t tmp_bytes,
                        float* out);
size_t median_tmp_bytes(int n);
void launch_transform4(hipStream_t s, const float4* pts, const int* perm, int n, const float* T12, float4* out);
void launch_gather_cov6(hipStream_t s, const double* cov_sorted, const int* perm, int n, double* out);

}  // namespace ddlo
