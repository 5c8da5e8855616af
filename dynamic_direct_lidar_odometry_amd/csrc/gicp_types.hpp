// gicp_types.hpp — plain data shared by the host runtime (capi.cpp) and the
// HIP kernels.  Everything here is POD so it can be memcpy'd into device
// memory as a job descriptor.
#pragma once
#include <stdint.h>

namespace ddlo {

// Search hierarchy geometry (see DESIGN.md "Cloud index"):
//   points sorted by 63-bit Morton key, leaves = 32 consecutive points,
//   every internal level groups 64 consecutive nodes of the level below, so a
//   wavefront tests one node's 64 children with one lane each.
constexpr int kLeafSize = 32;
constexpr int kFanout = 64;
constexpr int kMaxLevels = 5;   // leaves + 4 internal levels: n <= 32*64^4
constexpr int kDirBits = 18;    // key directory: top 18 of the 63 Morton-key bits (1 MB per cloud)
// Fine directory (search.hpp seed_pos): a coarse bucket holding more than
// kFineMin keys gets a slot of 2^kFineBits 16-bit offsets, the lower bound of
// each 6-bit refinement of its prefix.  Layout after dir's 2^kDirBits + 1
// entries: [slot counter][slot per coarse bucket, -1: none][slots].
constexpr int kFineBits = 6;
constexpr int kFineMin = 32;
__host__ __device__ constexpr long fine_dir_ints(int n) {   // ints of the whole directory buffer
  return (1L << kDirBits) + 2 + (1L << kDirBits) + ((long)(n / (kFineMin + 1) + 1) << kFineBits) / 2;
}

// Number of moment slots the linearize kernel reduces per source point
// (see DESIGN.md "Normal-equation moments"): 6 (sum M) + 18 (sum q_k M) +
// 36 (sum q_k q_l M) + 12 (sum (M e) qtilde^T) + cost + count = 74, padded to
// 96 for the 6-step in-register transpose reduction.
constexpr int kMoments = 74;
constexpr int kMomentSlots = 96;
constexpr int kSlabStride = 80;   // doubles per block partial in the slab
constexpr int kStatFields = 8;    // per-wave diagnostic counters (DDLO_STATS)

// Task list of the correspondence search (nn_tasks.hpp): kTaskRegions
// append counters, kCtrStride words apart (one 128-B line each), and
// kTasksPerGroup task slots per 16-query sub-group on average.
constexpr int kTaskRegions = 64;
constexpr int kTaskCounters = kTaskRegions + 1;   // + the hard sub-group list's length
constexpr int kCtrStride = 32;
constexpr int kHardMax = 1024;    // hard sub-groups walked first (longest walks first)
constexpr int kTasksPerGroup = 48;

struct CloudDev {
  const float4* pts;              // n sorted points; w = original index (int bits)
  const unsigned long long* keys; // n sorted Morton keys
  const int* perm;                // sorted position -> original index
  const int* inv_perm;            // original index -> sorted position
  const float4* box_lo;           // all levels, level 0 = leaves
  const float4* box_hi;
  const float* quant;             // device [lo.x, lo.y, lo.z, scale]
  const float* soa;               // per leaf: x[32], y[32], z[32] (sorted, sentinel-padded)
  const int* dir;                 // key directory [2^kDirBits + 1] + the fine directory (kFineBits)
  int n;
  int nlevels;
  // per-level node offset/count, kept as scalars (no array => no scratch
  // when a kernel holds a CloudDev in registers); use lvl_off()/lvl_cnt()
  int off0, off1, off2, off3, off4;
  int cnt0, cnt1, cnt2, cnt3, cnt4;
};

__host__ __device__ inline int lvl_off(const CloudDev& c, int l) {
  return l == 0 ? c.off0 : l == 1 ? c.off1 : l == 2 ? c.off2 : l == 3 ? c.off3 : c.off4;
}
__host__ __device__ inline int lvl_cnt(const CloudDev& c, int l) {
  return l == 0 ? c.cnt0 : l == 1 ? c.cnt1 : l == 2 ? c.cnt2 : l == 3 ? c.cnt3 : c.cnt4;
}

// ---------------------------------------------------------------------------
// nanoflann's kd-tree on the device (nftree.hpp / nftree.hip): only used to
// resolve exact distance ties in nanoflann's traversal order.
// nanoflann Node (reference impl/nanoflann_impl.hpp:876-894): a leaf holds the
// vind range [c1, c2); an inner node its children and divfeat / divlow / divhigh.
struct NfNode {
  int c1, c2;
  int feat;            // divfeat; -1 = leaf
  float divlow, divhigh;
  int parent;          // -1 at the root (build bookkeeping)
  int pad0, pad1;
};

struct NfTreeDev {
  const float4* vpts;  // [n] points in vind order: x, y, z, original index (int bits)
  const NfNode* nodes; // node 0 = root
  const float4* box;   // [2]: root_bbox (lo, hi), computeInitialDistances
  int n;
  int partial;         // the top levels only: a node with feat == -2 is an unsplit subtree (vind range [c1, c2),
  const float4* sbox;  // the box divideTree passes it: sbox[2 id], sbox[2 id + 1]); the lazy search splits it
};

// ---------------------------------------------------------------------------
// Candidate cells of a target (cellgrid.hip, DESIGN.md §4 "Candidate cells"):
// built once per target and bound, they answer the bounded 1-NN of
// update_correspondences (nano_gicp_impl.hpp:249-258) for a query in cell C
// from C's list: every target point that can be the fp32-nearest (or tie
// with it) for some point of C.  Coarse cells of size s tile the target's
// box plus the bound; a coarse cell is split uniformly into (2^level)^3 fine
// cells.
// Directory entry (u64) of a coarse cell: kCgNoMatch, kCgFallback, a
// level-0 list inline (bits 62-63 = 0: entry offset in bits 0-31, count in
// 32-61: no fine-table load on the lookup's dependent chain), or a refined
// cell (bits 62-63 = level 1..3, fine-table base in bits 0-31).
constexpr unsigned long long kCgNoMatch = ~0ull;       // no target point within the bound of any point of the cell
constexpr unsigned long long kCgFallback = ~0ull - 1;  // no list (the walk searches the cell's queries)
constexpr unsigned kCgFineFallback = 0xffffffffu;   // fine entry count: no list (the walk)
constexpr int kCgMaxLevel = 3;

struct CellGridDev {
  const unsigned long long* dir;   // [nx * ny * nz] directory entries (above)
  const uint2* fine;       // per fine cell: (first entry, count)
  const float4* ent;       // list entries: x, y, z, sorted target position (int bits)
  float ox, oy, oz, inv_s; // grid origin, 1 / coarse cell size
  int nx, ny, nz;
  int outside_nomatch;     // a query outside the grid box has no target point within the bound (else the walk)
  int has_fallback;        // some cell has no list (or outside_nomatch is 0): the walk kernel stays in the graph
};

// The list of the cell holding a query at grid coordinates (tx, ty, tz) (in
// range): 0 = no target point within the bound, 1 = the list (off, cnt),
// 2 = no list (the walk).
__device__ __forceinline__ int cg_cell_list(const CellGridDev& G, float tx, float ty, float tz, unsigned& off,
                                            unsigned& cnt) {
  const int cx = min((int)tx, G.nx - 1), cy = min((int)ty, G.ny - 1), cz = min((int)tz, G.nz - 1);
  const unsigned long long d = G.dir[((long)cx * G.ny + cy) * G.nz + cz];
  if (d == kCgNoMatch) return 0;
  if (d == kCgFallback) return 2;
  const int lvl = (int)(d >> 62);
  unsigned long long e = d;
  if (lvl != 0) {
    const int m = 1 << lvl;
    const int fx = min((int)((tx - (float)cx) * (float)m), m - 1);
    const int fy = min((int)((ty - (float)cy) * (float)m), m - 1);
    const int fz = min((int)((tz - (float)cz) * (float)m), m - 1);
    e = reinterpret_cast<const unsigned long long*>(G.fine)[(unsigned)d + (unsigned)((fx * m + fy) * m + fz)];
  }
  if ((unsigned)(e >> 32) == kCgFineFallback) return 2;
  off = (unsigned)e;
  cnt = (unsigned)(e >> 32) & 0x3fffffffu;
  return 1;
}

// Per-align device state (one per ctx, lives in device memory).
struct AlignState {
  double R[9];           // x0 (current estimate), row-major
  double t[3];
  double lambda;         // lm_lambda_
  double final_hessian[36];
  double final_cost;     // y0 of the last linearize
  double last_lin_R[9];  // pose of the last linearization (getResiduals)
  double last_lin_t[3];
  double last_b[6];      // b of the last linearize
  double last_mom[kSlabStride];  // reduced moments of the last linearize
  int iter;              // outer iterations executed so far
  int done;              // converged or failed: remaining kernels are no-ops
  int converged;
  int nr_iterations;
  int lm_failed;
  int lm_trials;
  int num_corr;
  int have_prev;         // correspondences of a previous linearize are valid
  int rec;               // the next search records reuse references (AlignJob::ref)
  float src_radius;      // max |p| over the source cloud's root boxes (reuse step bound)
  int any_rec;           // an iteration of this align recorded references
  // exact distance ties in the correspondences (nanoflann's order, k_moments):
  int tie_pending;       // a matched query's nearest distance is tied and the target has no nanoflann tree yet
                         // (the host builds it and runs the align again)
  int ties_resolved;     // tied queries re-run through the target's nanoflann tree (this align)
  int tie_err;           // a re-run failed (bits as k_nf_resolve_*: 1 depth, 2 tree build, 16 distance mismatch)
  // publication word (pinned copies only; 0 in the device state): k_lm_step
  // writes (ticket << 17 | done << 16 | iter) after the rest of the copy and a
  // system-scope fence, so the host that sees its align's ticket and the
  // chunk's iteration reads a complete state without waiting on a HIP event
  unsigned long long pub;
};

// Everything a kernel needs for one align, written by the host before launch.
struct AlignJob {
  CloudDev src;
  CloudDev tgt;
  const double* src_cov;   // sym6 per sorted source point
  const double* tgt_cov;   // sym6 per sorted target point
  int* corr;               // per sorted source point: sorted target pos or -1
  float* sqd;              // per sorted source point: squared 1-NN distance
  double* slab;            // [nblocks][kSlabStride] partial moments
  AlignState* state;
  unsigned int* stats;     // optional per-wave diagnostics [wave][kStatFields] (nullptr = off)
  double guess_R[9];
  double guess_t[3];
  long long job_full;      // k_align_init copies the whole job (1) or, when nothing else changed since the
                           // previous align of the ctx, only guess_R / guess_t, this word and the ticket (0)
  unsigned long long ticket;   // the align's sequence number on its ctx (AlignState::pub)
  double max_corr2;        // max_correspondence_distance^2 (double compare)
  float cap2;              // nextafter(float(max_corr2), +inf), the search bound
  // fp64 copies of the seed kernel's float knobs (scalar loads where they are
  // compared: a device-side conversion holds them in vector registers)
  double cap2_d, tri_mv_d, reuse_gap_d, reuse_gap0_d;
  int nblocks;             // linearize grid size (blocks)
  int max_iterations;      // outer loop bound (max or fixed iterations)
  int fixed_iterations;
  int optimizer;           // 0 GN, 1 LM
  int lm_max_iterations;
  double lm_init_lambda_factor;
  double transformation_epsilon;
  double rotation_epsilon;
  // Spatial sharding: this rank owns the source points
  // whose transformed coordinate q[own_axis] lies in [own_lo, own_hi); its
  // target holds that slab plus a max_corr halo.  own_axis < 0: unsharded.
  int own_axis;
  float own_lo, own_hi;
  // Interleaved sharding (the target replicated on every rank): this rank
  // owns the source points whose 16-point group of the device's spatial
  // (Morton) order is = own_rem mod own_mod.  own_mod = 0: off.
  int own_mod, own_rem;
  // premom = 1: k_mom_reduce writes this rank's reduced moments to mom, the
  // host's collective sums them across ranks in place, and k_lm_step reads
  // mom instead of reducing the slab itself.
  int premom;
  double* mom;             // [kSlabStride]
  float split_extent;      // sub-range split threshold of a wave's union box (m)
  // task-based correspondence search (nn_tasks.hpp)
  float4* qstate;                // [n_src] transformed query (x, y, z) + seed bound (< 0: inactive)
  unsigned long long* key;       // [n_src] (squared distance, sorted target position) of the best match
  unsigned long long* tasks;     // [kTaskRegions][task_cap_r]
  unsigned* task_ctr;            // [kTaskRegions * kCtrStride]
  int task_cap_r;
  int* hard_list;                // [kHardMax] sub-groups with a wide union box
  unsigned char* hard_flag;      // [n_src / 16] 1 = listed (walked by the first waves)
  float hard_extent;             // union-box extent (m) above which a sub-group is hard (first iteration)
  unsigned short* grp_blocks;    // [n_src / 16] blocks the last collect walked per sub-group
  int hard_blocks;               // later iterations: hard if the last walk took more blocks
  int xcd_scan;                  // scan: one spatial eighth of the tasks per XCD (speed only)
  int pf_ratio;                  // collect: lane-per-leaf pair tests below this queries / leaf-rounds ratio (speed only)
  int prev_window;         // seed after a large pose step: 0 previous match only, 1 + Morton window around it,
                           // 2 + Morton window at the new position (default)
  float probe2;            // fused seed: a sub-group with a windowed query still above this (squared m) probes the
                           // Morton windows of 8 points around its centre (0 = off)
  float probe_d;           // their offset from the centre (m)
  float tri_mv;            // a query that moved less than this (m) since the last linearize seeds from the
                           // triangle bound alone (no load); else from the previous match / Morton window
  // Verified match reuse across outer iterations: per query
  // the position q_ref of its last search, its match p1 there and a lower
  // bound B^2 on the fp32 squared distance from q_ref to every OTHER target
  // point.  At a later iteration, with the query moved by eps, p1 is still
  // the exact nearest point if d(q, p1) < B - eps (with fp32 rounding
  // margins); then no walk or scan runs for the query.
  int reuse;                     // 1 = check / record references (task search only)
  float reuse_gap;               // walk-radius inflation (m) at iterations >= 1: widens B beyond d1
  float reuse_gap0;              // the same at iteration 0
  int reuse_rec0;                // iteration 0 records references
  float reuse_rec_eps;           // later iterations record them only after an LM step that moved
                                 // every source point by less than this (m): the next one is smaller
  float reuse_rec_conv;          // ... and (convergence test on) whose is_converged measure exceeds this
  float4* ref;                   // [n_src] q_ref (x, y, z) + B^2 (< 0: no reference)
  float4* ref_p;                 // [n_src] p1 (x, y, z) + its sorted target position as int bits (-1: none within the bound)
  unsigned* sec;                 // [n_src] fp32 bits: smallest squared distance of an examined non-best point
                                 // (tie_scan 3: 0 = an equal-distance merge flagged the query)
  unsigned long long* key2;      // [n_src] tie_scan 3: the search's minimum of (squared distance, ~position), the
                                 // mirror of `key`: the same distance with a different point = a tie across runs
  // Exact ties of update_correspondences' 1-NN (nano_gicp_impl.hpp:255 ->
  // nanoflann_impl.hpp:205-237,1509: the first equidistant point of
  // nanoflann's walk wins).  tie_detect: k_moments flags a matched query whose
  // examined points hold another one at its nearest distance (sec == the
  // key's distance) and re-runs it through the target's nanoflann tree
  // (tgt_nf.nodes != nullptr), else sets AlignState::tie_pending.
  int tie_detect;
  int tie_ab;                    // A/B only (DDLO_TIE_AB bits, inexact): 1 no mirrored-key atomic, 2 no slice-merge
                                 // records, 4 no winner-slice check
  int tie_scan;                  // the scan's tie test: 1 second distance over every examined point, 2 the 8-point
                                 // slices' losing bests + k_moments' check of the winner's slice, 3 equal-distance
                                 // flags at the merges + the mirrored key + the winner's slice check, 4 as 3 with
                                 // the key atomic's return instead of the mirrored key, 0 none (A/B)
  const int* tgt_nf_status;      // the tree build's error bits (device int; 0 = usable)
  NfTreeDev tgt_nf;              // nodes == nullptr: no tree (yet); a slab shard's: its restriction of the
                                 // whole submap's tree (tietree.hip), point ids = the local target's
  // Candidate-cell lookup (k_cell_lookup, before the walk): grid_on = 1 when
  // the target has candidate cells built for this bound.  The lookup answers
  // every query whose cell has a list; the 16-query sub-groups left with an
  // unanswered owned query are listed for the walk (fb_list, fb_mask: the
  // unanswered queries of each sub-group, bit qi).
  int grid_on;
  CellGridDev grid;
  unsigned* fb_count;            // [kFbSegs * 32]: sub-groups listed for the walk per segment (zeroed by
                                 // k_align_init / k_moments; one counter per segment, 128 B apart)
  int* fb_list;                  // [kFbSegs][fb_seg_cap]
  int fb_seg_cap;
  unsigned short* fb_mask;       // [n_src / 16]
};
constexpr int kFbSegs = 8;       // walk-list segments (a wavefront appends to segment wave % kFbSegs)

constexpr int kNfMaxLevels = 40;   // big levels of the device build (deeper: the build reports a failure)
constexpr int kNfLevelSpare = 2;   // big levels a ctx's build carries beyond those its last build used

struct NfCtl {
  int nnodes, nsmall, err;   // err bits: 1 node capacity, 4 depth, 8 list capacity, 16/32 pairing checks
  int nchunks[2];
  int ntask[kNfMaxLevels + 1];
  int dbg[16];               // the first failed check's context (diagnostics)
};

// A node to split: its vind range, the box divideTree passes down (the
// middleSplit_ bbox argument) and its points' min / max (ordered uints).
struct NfTask {
  int node, begin, count, chunk0;
  float lo[3], hi[3];
  unsigned mm[6];
  int feat;
  float cut;
  int nch, pad;
};

struct NfBuild {
  float4* vpts;            // [n] in: original order (x, y, z, index); out: vind order
  NfNode* nodes;
  float4* box;             // [2] root_bbox
  int cap;                 // node capacity
  NfCtl* ctl;
  NfTask* tasks;           // [(Lmax + 1) * max_task]
  NfTask* pend;            // [(Lmax + 1) * max_pend] children produced by the level above
  NfTask* small;           // [max_small]
  int* chunk_task;         // [2 * max_chunks]
  NfTask* ctask;           // [2 * max_chunks] per chunk: a copy of its task (pad = the task index), one load
  int *cA, *cAE, *cE2;     // [max_chunks] per-chunk counts
  float4 *tblL, *tblR;     // [n] rank tables of the Hoare pairing
  const float* quant;      // the cloud's bbox: min [0..2], max [4..6]
  float4* sbox;            // partial build: the passed-down box of every unsplit node (indexed by node id)
  const float4* sorted;    // the cloud's Morton-sorted points (w = original index bits)
  const int* gate;         // optional: a count (the tied-query list's) that, when 0, makes every kernel a no-op
  int n, Lmax, max_task, max_pend, max_small, max_chunks;
  int nbucket;             // the size the grids are sized for (>= n): one captured graph per bucket
  int big_ids;             // node ids [0, big_ids) for the big levels; a small task of vind range
                           // [b, b + c) numbers its subtree in [big_ids + 2b, big_ids + 2(b + c))
};

struct NfSizes {
  int Lmax, max_task, max_pend, max_small, max_chunks, big_ids;
};

// Task-based kNN-k of a cloud's own points (covariances, knn_tasks.hip).
struct KnnJob {
  CloudDev c;
  int k;
  int method;                    // regularisation
  double* cov6;                  // [n] sym6 per sorted point (output)
  float4* qstate;                // [n] point (x, y, z) + squared ball bound (>= the k-th neighbour's)
  unsigned long long* cand;      // [cap][n] candidate (distance, position) keys, slot-major
  unsigned* cnt;                 // [n] candidates appended (> cap: overflow)
  int cap;
  unsigned long long* tasks;     // [kTaskRegions][task_cap_r]
  unsigned* task_ctr;            // [kTaskRegions * kCtrStride]
  int task_cap_r;
  unsigned char* redo;           // [ceil(n / 64)] 1 = recomputed by the lane-per-query kernel
  unsigned char* again;          // [n] 1 = second round (its candidates overflowed in the first)
  int round;                     // 1 or 2
  int* slot2;                    // [n] second-round candidate list of the point
  unsigned long long* cand2;     // [max2][cap2] second-round candidate keys
  unsigned* n2;                  // second-round lists handed out
  int cap2, max2;
  float split_extent;
  int* tie_list;                 // optional: sorted positions whose k-th distance is tied (nanoflann re-runs them)
  int* tie_count;
  int tie_cap;
};

}  // namespace ddlo
