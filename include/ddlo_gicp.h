/*
 * ddlo_gicp.h — C-ABI of the MI355X-native GICP scan-matching core.
 *
 * This is the drop-in boundary for the reference's NanoGICP registration core
 * (nano_gicp::NanoGICP<PointXYZI,PointXYZI>, reference
 * dynamic_direct_lidar_odometry/include/nano_gicp/nano_gicp.hpp:58-148 and
 * lsq_registration.hpp:60-128).  Plain pointers and sizes only; no exceptions
 * cross it; every entry point returns a gicp_status and sets a thread-local
 * message readable with gicp_last_error().
 *
 * One gicp_ctx == one NanoGICP instance (OdomNode owns two: gicp_s2s_ and
 * gicp_s2m_, reference include/odometry/odom.h:159-160).  A ctx owns one HIP
 * stream on its device and needs external synchronisation (like the reference,
 * which is driven from one ROS callback thread, odom_node.cc:43).  Distinct
 * ctxs may be used concurrently.
 *
 * Host buffers passed in are copied (H2D) before the call returns; the caller
 * may free them afterwards.  Clouds live on the device as ref-counted objects,
 * so gicp_swap_source_target / gicp_share_source are O(1) and never re-upload.
 */
#ifndef DDLO_GICP_H
#define DDLO_GICP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DDLO_GICP_ABI_VERSION 4

typedef enum gicp_status {
  GICP_OK = 0,
  GICP_EINVAL = 1,      /* bad argument (null pointer, size mismatch, bad enum) */
  GICP_ENOTARGET = 2,   /* align/linearize without a target cloud            */
  GICP_ENOSOURCE = 3,   /* align/linearize without a source cloud            */
  GICP_ETOOFEW = 4,     /* cloud has fewer points than k_correspondences      */
  GICP_EHIP = 5,        /* HIP runtime error (message in gicp_last_error)     */
  GICP_ENOMEM = 6,      /* device allocation failed                          */
  GICP_ESTATE = 7,      /* call not valid in the current state (e.g. residuals
                           requested before any align)                       */
  GICP_ENONFINITE = 8,  /* cloud contains NaN/Inf coordinates                 */
  GICP_ECOMM = 9        /* RCCL missing or a collective failed (sharded align) */
} gicp_status;

/* Same order as nano_gicp::RegularizationMethod (gicp/gicp_settings.hpp:47-54). */
typedef enum gicp_regularization {
  GICP_REG_NONE = 0,
  GICP_REG_MIN_EIG = 1,
  GICP_REG_NORMALIZED_MIN_EIG = 2,
  GICP_REG_PLANE = 3,
  GICP_REG_FROBENIUS = 4
} gicp_regularization;

/* Same order as nano_gicp::LSQ_OPTIMIZER_TYPE (lsq_registration.hpp:54-58). */
typedef enum gicp_optimizer { GICP_OPT_GAUSS_NEWTON = 0, GICP_OPT_LEVENBERG_MARQUARDT = 1 } gicp_optimizer;

typedef enum gicp_side { GICP_SIDE_SOURCE = 0, GICP_SIDE_TARGET = 1 } gicp_side;

/* Covariance layouts accepted/produced at the boundary.
 * MAT4D: 16 doubles per point, row-major Eigen::Matrix4d as the reference
 *        stores them (nano_gicp.hpp:136-137); only the 3x3 block is read.
 * SYM6:  6 doubles per point (xx, xy, xz, yy, yz, zz). */
typedef enum gicp_cov_layout { GICP_COV_MAT4D = 0, GICP_COV_SYM6 = 1 } gicp_cov_layout;

/* All GICP knobs.  gicp_default_params() fills the reference defaults:
 * k=20 (nano_gicp_impl.hpp:58), max_corr=FLT_MAX (:60), PLANE (:62),
 * max_iterations=64, rotation_eps=2e-3, transformation_eps=5e-4, LM,
 * lm_max_iterations=10, lm_init_lambda_factor=1e-9
 * (lsq_registration_impl.hpp:53-60). */
typedef struct gicp_params {
  int32_t k_correspondences;            /* setCorrespondenceRandomness        */
  int32_t max_iterations;               /* setMaximumIterations               */
  double max_correspondence_distance;   /* setMaxCorrespondenceDistance       */
  double transformation_epsilon;        /* setTransformationEpsilon           */
  double rotation_epsilon;              /* setRotationEpsilon                 */
  double lm_init_lambda_factor;         /* setInitialLambdaFactor             */
  int32_t regularization;               /* gicp_regularization                */
  int32_t optimizer;                    /* gicp_optimizer (reference: LM only,
                                           no setter; GN exposed for cfg 2)   */
  int32_t lm_max_iterations;            /* hard-coded 10 in the reference     */
  int32_t fixed_iterations;             /* 0 = reference convergence logic;
                                           >0 = run exactly this many outer
                                           iterations (benchmarks, cfg 2)     */
} gicp_params;

/* Outcome of one align (reference: converged_, nr_iterations_,
 * final_hessian_, the "lm not converged!!" branch at
 * lsq_registration_impl.hpp:115-119). */
typedef struct gicp_result {
  int32_t converged;          /* hasConverged()                                  */
  int32_t nr_iterations;      /* last outer loop index (reference semantics)     */
  int32_t iterations_run;     /* number of linearize() calls executed            */
  int32_t lm_failed;          /* 1 if step_lm exhausted lm_max_iterations        */
  int32_t lm_trials;          /* total compute_error evaluations                 */
  int32_t num_correspondences;/* matched source points at the last linearize     */
  double final_cost;          /* sum e^T M e at the last linearize               */
  double final_hessian[36];   /* getFinalHessian(), row-major                    */
  double lm_lambda;           /* lambda after the last step                      */
  double device_ms;           /* device time of the align (HIP events; only when
                                 profiling is enabled, else 0)                   */
  double linearize_ms;        /* summed device time of the linearize kernels
                                 (only when profiling is enabled, else 0)       */
  int32_t ties_resolved;      /* correspondences whose nearest distance was an
                                 exact tie, re-run in nanoflann's order          */
  int32_t tie_reruns;         /* 1 if a tie appeared before the target had its
                                 nanoflann tree: the tree was built and the
                                 align run again (the result is the second run) */
} gicp_result;

/* ---- library / context --------------------------------------------------- */
int32_t gicp_abi_version(void);
const char* gicp_last_error(void);
gicp_status gicp_default_params(gicp_params* out);

/* replaces constructing nano_gicp::NanoGICP (nano_gicp_impl.hpp:49-65) */
gicp_status gicp_ctx_create(int device, struct gicp_ctx** out);
gicp_status gicp_ctx_destroy(struct gicp_ctx* ctx);

/* replaces the setters called at odom.cc:92-112 */
gicp_status gicp_set_params(struct gicp_ctx* ctx, const gicp_params* p);
gicp_status gicp_get_params(const struct gicp_ctx* ctx, gicp_params* out);

/* ---- clouds ---------------------------------------------------------------
 * xyz points at float x,y,z of point 0; consecutive points are stride_bytes
 * apart (32 for pcl::PointXYZI, 12 for packed xyz).
 *
 * gicp_set_source(build_index=1) replaces NanoGICP::setInputSource
 *   (nano_gicp_impl.hpp:132-143: sets input_, builds the source kd-tree,
 *   clears source covariances);
 * gicp_set_source(build_index=0) replaces registerInputSource (:122-130):
 *   no covariance reset — existing source covariances stay attached to the
 *   same point indices (dropped only if the point count changes: the
 *   reference then recomputes them at align, :186-189).  The device index is
 *   built either way (it is cheap and the sorted cloud is the storage).
 * gicp_set_target replaces setInputTarget (:145-155). */
gicp_status gicp_set_source(struct gicp_ctx* ctx, const float* xyz, size_t n, size_t stride_bytes, int build_index);
gicp_status gicp_set_target(struct gicp_ctx* ctx, const float* xyz, size_t n, size_t stride_bytes);
gicp_status gicp_clear_source(struct gicp_ctx* ctx); /* clearSource (:108-113) */
gicp_status gicp_clear_target(struct gicp_ctx* ctx); /* clearTarget (:115-120) */
gicp_status gicp_get_size(const struct gicp_ctx* ctx, int side, size_t* n);

/* calculateSourceCovariances / calculateTargetCovariances (:171-181 ->
 * calculate_covariances :373-441): exact kNN-k (self included), biased
 * covariance, regularisation per params. */
gicp_status gicp_compute_covariances(struct gicp_ctx* ctx, int side);
/* setSourceCovariances / setTargetCovariances (:157-169) — copied. */
gicp_status gicp_set_covariances(struct gicp_ctx* ctx, int side, const double* cov, size_t n, int layout);
/* getSourceCovariances / getTargetCovariances (nano_gicp.hpp:106-114). */
gicp_status gicp_get_covariances(const struct gicp_ctx* ctx, int side, double* cov, size_t n, int layout);
/* 1 if the side's covariances are present (size == cloud size). */
gicp_status gicp_has_covariances(const struct gicp_ctx* ctx, int side, int* has);

/* swapSourceAndTarget (:97-106): swaps clouds, indices and covariances,
 * clears correspondences.  O(1). */
gicp_status gicp_swap_source_target(struct gicp_ctx* ctx);
/* Replaces the public-member aliasing the caller does at odom.cc:530
 * (gicp_s2m_.source_kdtree_ = gicp_s2s_.source_kdtree_) and :765
 * (gicp_s2m_.source_covs_ = gicp_s2s_.source_covs_): dst's source becomes
 * src's source cloud, device index and covariances (copy-on-write). */
gicp_status gicp_share_source(struct gicp_ctx* dst, const struct gicp_ctx* src);

/* ---- registration -------------------------------------------------------- */
/* pcl::Registration::align(output, guess) -> NanoGICP::computeTransformation
 * (:183-196) -> LsqRegistration::computeTransformation
 * (lsq_registration_impl.hpp:95-126).  guess/out: row-major 4x4 float
 * (Eigen::Matrix4f).  guess may be NULL (identity, as align(output)).
 * Missing covariances are computed first, as the reference does. */
gicp_status gicp_align(struct gicp_ctx* ctx, const float* guess16, float* out16, gicp_result* res);

/* getResiduals(std::vector<double>&, trans) (:225-232): sqrt of the squared
 * 1-NN distance of every source point (original order) from the LAST
 * update_correspondences; the trans argument is ignored there too. */
gicp_status gicp_get_residuals(struct gicp_ctx* ctx, double* out, size_t n);
/* Residual image for the dynamic-object detection:
 * the projection OdomNode does after getResiduals (odom.cc:804-827; the
 * reference uses theta in [-60, 60] deg and 512 x 512) feeding
 * DetectionModule::projectResiduals (detection.cpp:203-252).  Source point i
 * (sensor frame) goes to u = int((atan2(x, z) - tmin) / (tmax - tmin) * W),
 * v = int((atan2(y, hypot(x, z)) - tmin) / (tmax - tmin) * H); the highest
 * original index landing on a pixel wins (the reference's write order).
 * img: H*W floats, the residual (0 where no point); xyz (optional): H*W*3,
 * the winning point (0 where none). */
gicp_status gicp_residual_image(struct gicp_ctx* ctx, double theta_min, double theta_max, int width, int height,
                                float* img, float* xyz);
/* correspondences_ / sq_distances_ of the last linearization, original
 * indices (-1 = no correspondence within max_correspondence_distance).
 * sq_dist is the unbounded 1-NN squared distance of every point, as
 * sq_distances_ (nano_gicp_impl.hpp:255-257), matched or not. */
gicp_status gicp_get_correspondences(struct gicp_ctx* ctx, int32_t* corr, float* sq_dist, size_t n);
/* pcl::transformPointCloud(*input_, output, final_transformation_)
 * (lsq_registration_impl.hpp:125); writes xyz with the given stride. */
gicp_status gicp_transform_source(struct gicp_ctx* ctx, float* out_xyz, size_t n, size_t stride_bytes);

/* ---- kernel-level entry points (parity tests, benchmarks) ----------------- */
/* linearize(trans, &H, &b) (:277-342) at a given pose (row-major 4x4 double):
 * runs update_correspondences + the H/b/cost reduction once.  H row-major. */
gicp_status gicp_linearize(struct gicp_ctx* ctx, const double* pose16, double* H36, double* b6, double* cost,
                           int32_t* num_correspondences);
/* Exact k-NN of query points against the TARGET index (nanoflann
 * nearestKSearch, nanoflann.hpp:145-156).  Indices are original target
 * indices, ascending by squared distance; equal distances in the order
 * nanoflann's own tree meets them (see gicp_set_tie_order). */
gicp_status gicp_knn_target(struct gicp_ctx* ctx, const float* q, size_t nq, size_t stride_bytes, int k,
                            int32_t* idx, float* sq_dist);
/* Exact distance ties (equidistant points at the k-th neighbour, or inside
 * the k of gicp_knn_target): 1 (default) = nanoflann's answer, the point its
 * depth-first walk of its own kd-tree meets first (KNNResultSet::addPoint
 * keeps the earlier of equal distances, nanoflann_impl.hpp:205-237,1509);
 * the device builds that tree (nftree.hip) and re-runs only the tied queries
 * through it.  0 = the lower position in the device's Morton order (no tree
 * is built).  Distances are identical either way.  Applies to covariances
 * and gicp_knn_target. */
gicp_status gicp_set_tie_order(struct gicp_ctx* ctx, int nanoflann_order);
gicp_status gicp_get_tie_order(const struct gicp_ctx* ctx, int* nanoflann_order);

/* Options of a context.  gicp_set_default_option sets the value contexts
 * created afterwards start with (process-wide; also the contexts the
 * odometry driver and gicp_s2s_batch create inside).  Results are identical
 * under every value; only the work differs. */
enum gicp_option {
  GICP_OPT_TIE_ORDER = 1,           /* 1 (default): nanoflann's tie order; 0: Morton (= gicp_set_tie_order) */
  GICP_OPT_TIE_LAZY = 2,            /* 1 (default): covariance ties searched on the partial tree, splitting
                                       lazily; 0: on the whole tree */
  GICP_OPT_TIE_PARTIAL_LEVELS = 3,  /* big levels of that partial tree (0..24, default 3) */
  GICP_OPT_COV_TASKS = 4,           /* 1: the task-based k-NN for covariances (default 0: a lane per query) */
  GICP_OPT_GRID_MAX_MB = 5,         /* device MiB a target's candidate cells may hold (0, the default: no
                                       cap); a build that would exceed it is abandoned and the target stays
                                       on the walk (gicp_grid_info.build_status = GICP_ENOMEM) */
  GICP_OPT_COUNT = 6
};
gicp_status gicp_set_option(struct gicp_ctx* ctx, int option, int value);
gicp_status gicp_get_option(const struct gicp_ctx* ctx, int option, int* value);
gicp_status gicp_set_default_option(int option, int value);
gicp_status gicp_get_default_option(int option, int* value);

/* Candidate cells of the target (DESIGN.md §4 "Candidate cells"): a
 * per-target structure built once per (target cloud, max correspondence
 * distance) that answers update_correspondences' bounded 1-NN
 * (nano_gicp_impl.hpp:249-258, the nanoflann knnSearch it calls) by a cell
 * lookup and a short list scan instead of a walk of the index, on every
 * outer iteration of every align against that target.  Results are
 * identical with or without it (same correspondences, distances and tie
 * order); only the time differs.  It pays for a target that is aligned
 * against several times (the S2M submap: OdomNode keeps a submap for many
 * scans, odom.cc:1215-1315).  mode: 0 = off; 1 = auto (default): built at the
 * 32nd align against the same target and bound (a long-lived target; the
 * build costs about a hundred aligns' savings); 2 = built at the next align.  The structure belongs to the target cloud (it follows
 * gicp_swap_source_target). */
#define GICP_GRID_OFF 0
#define GICP_GRID_AUTO 1
#define GICP_GRID_ON 2
gicp_status gicp_set_target_grid(struct gicp_ctx* ctx, int mode);
typedef struct gicp_grid_info {
  int32_t built;             /* 1 = the target has candidate cells for the ctx's bound */
  float build_ms;            /* device time of the build (HIP events)                 */
  float cell_size;           /* coarse cell edge (m); fine cells are 1/2..1/8 of it  */
  int64_t bytes;             /* device memory held by the structure                   */
  int64_t coarse_cells;      /* cells of the grid box                                 */
  int64_t band_cells;        /* coarse cells within reach of the target               */
  int64_t nomatch_cells;     /* ... of which no point is within the bound             */
  int64_t overflow_cells;    /* ... whose candidates overflowed kCgCandMax at level 0
                                (their children's lists come from a direct walk)     */
  int64_t level_cells[4];    /* coarse cells finished at fine level 0..3              */
  int64_t fine_cells;        /* fine cells with a list                                */
  int64_t fallback_fine;     /* fine cells whose list exceeded the cap (the walk)     */
  int64_t entries;           /* list entries (16 B each)                              */
  int64_t uses_walk;         /* 1: some queries still take the walk (a fine cell
                                without a list, or the bound's reach beyond the grid);
                                0: the linearize is one kernel (lookup fused into the
                                moments)                                              */
  int64_t build_status;      /* 0, or the gicp_status of a build that failed (pool or
                                table limits, GICP_OPT_GRID_BUDGET_MB, device memory):
                                the target then stays on the walk for this bound and
                                the align itself succeeds                             */
  int64_t scratch_bytes;     /* the build's transient device scratch at its peak (not
                                held afterwards; not in gicp_get_device_bytes)       */
} gicp_grid_info;
gicp_status gicp_get_target_grid_info(struct gicp_ctx* ctx, gicp_grid_info* out);
/* Queries the last align's final linearize answered from the candidate cells
 * and sub-groups of 16 it left to the walk (diagnostics). */
gicp_status gicp_get_lookup_stats(struct gicp_ctx* ctx, int64_t* walk_groups);

/* nanoflann's kd-tree of a side's cloud as the device built it (tests):
 * vind[n]; per node (c1, c2, divfeat, parent) with divfeat -1 for a leaf
 * whose vind range is [c1, c2), and (divlow, divhigh).  With all three
 * outputs NULL only *nnodes is returned. */
gicp_status gicp_debug_nftree(struct gicp_ctx* ctx, int side, int32_t* vind, int32_t* nodes4, float* div2, size_t cap,
                              size_t* nnodes);
/* Build diagnostics (development): a fresh build of a side's tree that stops
 * after `stop` big levels (-1 = complete), returning vind[n] as it stands,
 * info16 = {Lmax, max_task, max_pend, max_small, max_chunks, scratch offsets
 * of tasks, pend, small, chunk map, cA, cAE, cE2, tables, total bytes, n,
 * node capacity}, status2 = {error bits, nodes}, and the first scratch_cap
 * bytes of the build's scratch (control word, task lists, counts). */
gicp_status gicp_debug_nfbuild(struct gicp_ctx* ctx, int side, int stop, int32_t* vind, int64_t* info16,
                               int32_t* status2, void* scratch, size_t scratch_cap);
/* The 74 reduced normal-equation moments of the last linearize (80 doubles,
 * layout in DESIGN.md "Normal-equation moments"); test/debug entry. */
gicp_status gicp_get_moments(const struct gicp_ctx* ctx, double* out80);
/* Device time accounting of the linearize kernel inside align (HIP events
 * captured in the align graph).  Off by default. */
gicp_status gicp_set_profiling(struct gicp_ctx* ctx, int enable);
/* With profiling on: device time (HIP events, on the streams the kernels run
 * on) of the last gicp_compute_covariances on this ctx: the k-NN covariance
 * kernel, nanoflann's tree build (tie order; 0 if the cloud already had its
 * tree) and the tie resolvers.  Measurement entry (bench.py's roofline). */
typedef struct gicp_stage_times {
  double cov_ms;
  double tree_ms;
  double resolve_ms;
} gicp_stage_times;
gicp_status gicp_get_stage_times(struct gicp_ctx* ctx, gicp_stage_times* out);
/* Diagnostics (development): enable per 64-query-group search counters for
 * subsequent linearize launches and/or read those of the last launch. */
gicp_status gicp_debug_stats(struct gicp_ctx* ctx, int enable, unsigned int* out, size_t max_words, size_t* nwords);
/* Blocks until all work queued on the ctx's stream(s) has finished. */
gicp_status gicp_synchronize(struct gicp_ctx* ctx);
/* The ctx's HIP stream (hipStream_t) for callers that interleave their own work. */
gicp_status gicp_get_stream(const struct gicp_ctx* ctx, void** stream);

/* ---- spatially sharded align (no reference counterpart:
 * the reference aligns on one host, nano_gicp_impl.hpp:277-342 summing
 * per-thread H/b partials, which here become per-GPU partials) ------------
 * Rank r of N holds the target points of its slab [lo, hi) along `axis`
 * plus a halo of max_correspondence_distance on both sides (and their
 * covariances, computed on the full cloud), and the whole source.  Each
 * outer iteration it searches only the source points whose transformed
 * coordinate falls in its slab, reduces their moments, all-reduces the 80
 * moment doubles over RCCL (ncclSum, fp64) and runs the identical LM step,
 * so every rank returns the same pose.  Exact: any target point within
 * max_corr of an owned query lies in the slab + halo. */
/* Ownership slab of this ctx; axis -1 removes it. */
gicp_status gicp_set_shard(struct gicp_ctx* ctx, int axis, float lo, float hi);
/* Exact ties for a slab shard (DESIGN.md §5 "Slab shards"): a slab's target
 * is a subset of the submap, and nanoflann orders equidistant points by ITS
 * tree, which differs from the whole submap's (nanoflann_impl.hpp:1045-1143
 * cut the subset's boxes).  A slab rank resolves its tied correspondences
 * through the whole submap's tree RESTRICTED to its own points (every point
 * outside the slab + halo removed, emptied subtrees as empty leaves): for a
 * matched owned query every equidistant point lies in the halo and the walk
 * meets them in the whole tree's order.  The restriction is O(slab + halo);
 * the rank never holds the whole submap.  gicp_set_target,
 * gicp_clear_target and gicp_swap_source_target drop it.
 *
 * Builder (one rank, e.g. rank 0, once per submap): gicp_tie_builder_set
 * uploads the whole submap and builds its nanoflann tree (n = 0 frees them);
 * gicp_tie_builder_export returns the restriction to one rank's points
 * (local_index[i] = the whole-cloud index of that rank's local target point
 * i; one-to-one) as a blob owned by the ctx, valid until its next builder
 * call.  Rank: gicp_set_tie_tree installs a blob (bytes = 0 removes it); it
 * is checked against the local target (same size, a tree whose leaves
 * partition the points, each point the local target's point of that index:
 * GICP_EINVAL otherwise).  gicp_set_tie_trees_from_root does the transport
 * over the ctx's communicator (collective: the root passes every rank's
 * blob, the others NULL; one broadcast of the sizes, then root -> rank
 * point-to-point).  gicp_set_tie_target = builder + export + install on one
 * ctx, the whole cloud released before it returns (single-process use). */
gicp_status gicp_tie_builder_set(struct gicp_ctx* ctx, const float* xyz, size_t n, size_t stride_bytes);
gicp_status gicp_tie_builder_export(struct gicp_ctx* ctx, const int32_t* local_index, size_t n_local,
                                    const void** blob, size_t* bytes);
gicp_status gicp_set_tie_tree(struct gicp_ctx* ctx, const void* blob, size_t bytes);
gicp_status gicp_set_tie_trees_from_root(struct gicp_ctx* ctx, int root, const void* const* blobs,
                                         const size_t* sizes);
gicp_status gicp_set_tie_target(struct gicp_ctx* ctx, const float* xyz, size_t n, size_t stride_bytes,
                                const int32_t* local_index, size_t n_local);
/* Device bytes the ctx holds (pool size classes): out[0] total, [1] target
 * cloud (points, index, trees, candidate cells), [2] source cloud (0 when
 * shared with the target), [3] covariances, [4] slab tie tree, [5] tie
 * builder, [6] scratch.  nout entries are written (up to 7). */
gicp_status gicp_get_device_bytes(const struct gicp_ctx* ctx, int64_t* out, int nout);
/* Interleaved sharding, for a target that fits every GPU (it is replicated):
 * rank `part` of `nparts` owns the source points whose 16-point group in the
 * device's spatial (Morton) order is congruent to part mod nparts, so every
 * rank searches the same number of points spread over the whole scan.
 * Combines with gicp_set_shard (both predicates must hold); nparts <= 1
 * removes it.  Exact for the same reason as the slabs: every owned point
 * sees the whole target. */
gicp_status gicp_set_shard_groups(struct gicp_ctx* ctx, int nparts, int part);
/* ncclGetUniqueId (128 bytes) — call on one rank and broadcast. */
gicp_status gicp_comm_unique_id(uint8_t* out, size_t nbytes);
/* ncclCommInitRank on the ctx's device (collective over the nranks ranks);
 * nranks = 0 detaches.  With a communicator, align / linearize all-reduce
 * the moments and get_residuals all-reduces (min) the residuals. */
gicp_status gicp_set_comm(struct gicp_ctx* ctx, const uint8_t* id, size_t nbytes, int nranks, int rank);
/* nranks (0 = no communicator), rank, and whether the collective is captured
 * in the align graphs (1) or launched eagerly (0). */
gicp_status gicp_get_comm_info(const struct gicp_ctx* ctx, int* nranks, int* rank, int* graphs);

/* ---- frame-parallel scan-to-scan batch (SURVEY.md §8(e) cfg 5) ----------
 * The S2S half of OdomNode::scanMatching over a recorded sequence
 * (odom.cc:754-768: align(guess = I), getFinalTransformation, then
 * swapSourceAndTarget so scan t becomes the target of scan t+1 with its
 * index and covariances).  S2S pairs are independent (each uses only scans
 * t-1 and t), so the sequence is cut into nstreams contiguous chunks, each
 * chained on its own ctx / HIP stream / host thread; a chunk's first pair
 * builds scan t-1 once more.  out16[t] (row-major 4x4) = the transform
 * aligning scan t onto scan t-1 (out16[0] = identity); res[t] (optional)
 * its result.  clouds[t] points to sizes[t] points with the given stride. */
gicp_status gicp_s2s_batch(int device, const gicp_params* p, const float* const* clouds, const size_t* sizes,
                           size_t stride_bytes, int nframes, int nstreams, float* out16, gicp_result* res);

#ifdef __cplusplus
}
#endif

#endif /* DDLO_GICP_H */
