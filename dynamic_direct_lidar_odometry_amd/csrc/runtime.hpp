// runtime.hpp — device-side objects of the GICP runtime shared by the C-ABI
// (capi.hip) and the odometry driver (odom.hip): the caching device
// allocator, ref-counted device clouds (Morton-sorted points + search
// hierarchy) and covariance sets, and the per-ctx state behind gicp_ctx.
#pragma once
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>  // types only (ncclComm_t)

#include <array>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/ddlo_gicp.h"
#include "gicp_types.hpp"
#include "launch.hpp"
#include "devknobs.hpp"

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return ::ddlo::rt::fail(_e == hipErrorOutOfMemory ? GICP_ENOMEM : GICP_EHIP,          \
                              std::string(#expr) + ": " + hipGetErrorString(_e));           \
  } while (0)

namespace ddlo {
namespace rt {


inline thread_local std::string g_last_error;

inline gicp_status fail(gicp_status s, const std::string& msg) {
  g_last_error = msg;
  return s;
}



// Caching device allocator.  hipFree synchronizes the whole device, which
// would serialize every ctx of a multi-stream batch (a new cloud index and
// covariance set per scan); released blocks go to a per-(device, size class)
// free list instead and are handed out again.  Safe because every entry
// point that enqueues work on a buffer waits for it before returning, so a
// buffer is idle whenever its owner releases it (the speculative no-op
// iteration of an align touches only ctx-owned state, freed at ctx
// destruction after a stream synchronize).
struct DevicePool {
  std::mutex m;
  std::multimap<std::pair<int, size_t>, void*> free_blocks;
  static size_t size_class(size_t b) {  // <= 12.5 % rounding, so same-shape clouds share a class
    b = std::max<size_t>(b, 256);
    size_t top = 1;
    while ((top << 1) <= b) top <<= 1;
    const size_t g = std::max<size_t>(top / 8, 256);
    return (b + g - 1) / g * g;
  }
  hipError_t alloc(size_t cls, void** p) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    {
      std::lock_guard<std::mutex> lk(m);
      auto it = free_blocks.find({dev, cls});
      if (it != free_blocks.end()) {
        *p = it->second;
        free_blocks.erase(it);
        return hipSuccess;
      }
    }
    e = hipMalloc(p, cls);
    if (e == hipErrorOutOfMemory) {  // give the cached blocks back and retry once
      trim();
      e = hipMalloc(p, cls);
    }
    return e;
  }
  void release(int dev, size_t cls, void* p) {
    std::lock_guard<std::mutex> lk(m);
    free_blocks.insert({{dev, cls}, p});
  }
  void trim() {
    std::lock_guard<std::mutex> lk(m);
    for (auto& kv : free_blocks) (void)hipFree(kv.second);
    free_blocks.clear();
  }
};
inline DevicePool& device_pool() {
  static DevicePool* pool = new DevicePool();  // never destroyed: blocks live until exit
  return *pool;
}

// HIP streams are recycled, not destroyed: a context made after others were
// destroyed gets their streams (and hardware queues) back instead of new
// ones.  The S2S batch in a fresh process: 0.42 ms per pair with recycling,
// 0.46-0.47 without; after 10 contexts made and destroyed it still runs at
// ~0.59-0.64 either way (cause not found: not the streams, not the pinned
// blocks; tools/batch_leg_alone.py).  A released stream is idle (its owner
// synchronized it); the last released is handed out first.
struct StreamPool {
  std::mutex m;
  std::vector<std::pair<int, hipStream_t>> free_streams;
  hipError_t acquire(hipStream_t* s) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    {
      std::lock_guard<std::mutex> lk(m);
      for (size_t i = free_streams.size(); i-- > 0;)
        if (free_streams[i].first == dev) {
          *s = free_streams[i].second;
          free_streams.erase(free_streams.begin() + (long)i);
          return hipSuccess;
        }
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  }
  void release(int dev, hipStream_t s) {
    std::lock_guard<std::mutex> lk(m);
    free_streams.emplace_back(dev, s);
  }
};
inline StreamPool& stream_pool() {
  static StreamPool* pool = new StreamPool();  // never destroyed: streams live until exit
  return *pool;
}

// Pinned host blocks of the contexts (job / state descriptors the device
// reads, read-back flags), recycled like the streams: freed to this list at
// context destruction and handed out again by (size, flags)
struct PinnedPool {
  std::mutex m;
  std::multimap<std::pair<size_t, unsigned>, void*> free_blocks;
  hipError_t alloc(void** p, size_t bytes, unsigned flags) {
    {
      std::lock_guard<std::mutex> lk(m);
      auto it = free_blocks.find({bytes, flags});
      if (it != free_blocks.end()) {
        *p = it->second;
        free_blocks.erase(it);
        std::memset(*p, 0, bytes);   // no state of the previous owner
        return hipSuccess;
      }
    }
    return hipHostMalloc(p, bytes, flags);
  }
  void release(void* p, size_t bytes, unsigned flags) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(m);
    free_blocks.insert({{bytes, flags}, p});
  }
};
inline PinnedPool& pinned_pool() {
  static PinnedPool* pool = new PinnedPool();  // never destroyed: blocks live until exit
  return *pool;
}

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int dev = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { reset(); }
  void reset() {
    if (p) device_pool().release(dev, bytes, p);
    p = nullptr;
    bytes = 0;
  }
  hipError_t ensure(size_t b) {
    if (b <= bytes && p) return hipSuccess;
    reset();
    const size_t cls = DevicePool::size_class(b);
    hipError_t e = device_pool().alloc(cls, &p);
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    (void)hipGetDevice(&dev);
    bytes = cls;
    return e;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// nanoflann's own kd-tree of a cloud (nftree.hip), built on first need: the
// order in which the reference's search meets equidistant points.
struct NfTreeData {
  int n = 0, cap = 0;
  DevBuf vpts, nodes, box, status;   // status: {the build's error bits, node count} (device ints)
  bool partial = false;              // the top levels only (nftree_build partial_levels): stubs below
  DevBuf sbox;                       // partial: the stubs' passed-down boxes
  hipEvent_t ready = nullptr;        // recorded after the build on the ctx's aux stream; users wait on it
  NfTreeData() = default;
  NfTreeData(const NfTreeData&) = delete;
  NfTreeData& operator=(const NfTreeData&) = delete;
  ~NfTreeData() {
    if (ready) (void)hipEventDestroy(ready);
  }
  NfTreeDev dev() const {
    NfTreeDev t;
    t.vpts = vpts.as<float4>();
    t.nodes = nodes.as<NfNode>();
    t.box = box.as<float4>();
    t.n = n;
    t.partial = partial ? 1 : 0;
    t.sbox = partial ? sbox.as<float4>() : nullptr;
    return t;
  }
};

// Candidate cells of a target cloud for one correspondence bound
// (cellgrid.hip; built by cellgrid_build in capi.hip).
struct CellGridData {
  float cap2 = 0.f;            // the bound (AlignJob::cap2) the lists were built for
  bool ok = false;             // built (else the walk answers every query)
  DevBuf dir, fine, ent;
  CellGridDev dev{};
  gicp_grid_info info{};
};

// Immutable device cloud + search hierarchy (shared between ctxs/sides).
struct CloudData {
  int n = 0;
  DevBuf pts, keys, perm, inv_perm, box_lo, box_hi, quant, soa, dir;
  std::shared_ptr<NfTreeData> nf;   // nanoflann's tree (tie order), built on first need
  std::shared_ptr<NfTreeData> nfp;  // its top levels only (the lazy covariance tie search)
  std::shared_ptr<CellGridData> grid;   // candidate cells (S2M targets), built on demand
  float grid_aligns_cap2 = -1.f;        // the bound of the aligns counted in grid_aligns
  int grid_aligns = 0;                  // aligns against this cloud as the target with that bound
  int nlevels = 0;
  int lvl_off[kMaxLevels] = {0};
  int lvl_cnt[kMaxLevels] = {0};
  int upper_count() const {
    return nlevels <= 1 ? 0 : lvl_off[nlevels - 1] + lvl_cnt[nlevels - 1] - lvl_off[1];
  }
  CloudDev dev() const {
    CloudDev c;
    c.pts = pts.as<float4>();
    c.keys = keys.as<unsigned long long>();
    c.perm = perm.as<int>();
    c.inv_perm = inv_perm.as<int>();
    c.box_lo = box_lo.as<float4>();
    c.box_hi = box_hi.as<float4>();
    c.quant = quant.as<float>();
    c.soa = soa.as<float>();
    c.dir = dir.as<int>();
    c.n = n;
    c.nlevels = nlevels;
    c.off0 = lvl_off[0]; c.off1 = lvl_off[1]; c.off2 = lvl_off[2]; c.off3 = lvl_off[3]; c.off4 = lvl_off[4];
    c.cnt0 = lvl_cnt[0]; c.cnt1 = lvl_cnt[1]; c.cnt2 = lvl_cnt[2]; c.cnt3 = lvl_cnt[3]; c.cnt4 = lvl_cnt[4];
    return c;
  }
};

struct CovData {
  int n = 0;
  DevBuf cov6;  // sym6 per SORTED point
};

struct Side {
  std::shared_ptr<CloudData> cloud;
  std::shared_ptr<CovData> cov;
  bool has_cov() const { return cloud && cov && cov->n == cloud->n; }
};

inline int levels_for(int n, int* cnt, int* off) {
  int c = (n + kLeafSize - 1) / kLeafSize;
  int L = 0, o = 0;
  for (;;) {
    if (L >= kMaxLevels) return -1;
    cnt[L] = c;
    off[L] = o;
    o += c;
    ++L;
    if (c <= kFanout) break;
    c = (c + kFanout - 1) / kFanout;
  }
  return L;
}

}  // namespace rt
}  // namespace ddlo

using namespace ddlo;
using namespace ddlo::rt;

// one captured chunk: the graph and its executable instance
struct hipExecGraphPair {
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
};

// The chunk graphs of one launch geometry: [init + n iterations] for the
// predicted iteration count n (one per n, index n - 1) and [1 iteration]
// publishing to state slot s = 0, 1; captured for: RCCL in the chunk, job
// buffer, launch geometry (LinGeom).
struct GraphSet {
  std::array<long long, 8> key{{-1, -1, -1, -1, -1, -1, -1, -1}};
  std::vector<hipExecGraphPair> first;
  hipExecGraphPair rest[2];
  long long last_use = 0;
};
constexpr int kGraphSets = 4;   // geometries a ctx keeps captured (scans straddling a size bucket alternate)
constexpr int kNfGraphs = 4;    // tree-build graphs a ctx keeps captured

constexpr int kDefaultPredictedIters = 4;

struct gicp_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  gicp_params params{};
  Side src, tgt;
  // build scratch
  DevBuf raw_bytes, raw_pts, partial, nonfinite, keys_tmp, vals_tmp, sort_tmp, knn;
  // align buffers
  DevBuf corr, sqd, slab, job_dev, state_dev, tmp_out, stats;
  bool stats_on = false;
  AlignJob* job_host = nullptr;   // pinned
  AlignJob job_last{};            // the job k_align_init last copied whole (AlignJob::job_full)
  bool job_last_valid = false;
  AlignJob* job_host_dev = nullptr;     // its device-side address (read by k_align_init)
  AlignState* state_host_dev = nullptr; // state_host's device-side address (written by k_lm_step)
  // pinned, two slots: chunk k publishes its end state to slot k % 2, so the
  // (at most one) chunk queued behind the one the host is reading never
  // writes the bytes being read (no torn pose / done / iter)
  AlignState* state_host = nullptr;
  int state_slot = 0;              // slot holding the state of the last align / linearize
  hipEvent_t tail_ev = nullptr;    // last chunk launched by the last align (may still be queued)
  bool tail_pending = false;
  int grid_max_mb = 0;             // GICP_OPT_GRID_MAX_MB (0: no cap)
  unsigned long long ticket = 0;   // aligns launched (AlignJob::ticket)
  int* flag_host = nullptr;       // pinned
  bool have_align = false;        // a linearize ran against the current src/tgt
  int last_nsrc = 0;
  // chunk graphs of the last kGraphSets launch geometries (least recently
  // used evicted)
  std::vector<GraphSet> gsets;
  long long graph_clock = 0;
  int predicted_iters = kDefaultPredictedIters;   // iterations of the previous align on this ctx
  std::vector<hipEvent_t> chunk_ev;
  // second stream: nanoflann's tree (tie order) is built here while the
  // covariance / kNN kernels run on `stream`; the resolvers wait for it
  hipStream_t aux_stream = nullptr;
  hipEvent_t aux_ev = nullptr;
  DevBuf nf_desc;                    // the build descriptor the tree kernels read
  // the build, captured per (size bucket, level count); the last kNfGraphs
  // kept (a scan size straddling a bucket boundary alternates two)
  struct NfGraph {
    long long key = -1;
    hipGraphExec_t ge = nullptr;
    long long last_use = 0;
  };
  std::vector<NfGraph> nf_graphs;
  long long nf_clock = 0;
  // Big levels the builds of this ctx need: the level counts of each build
  // (ctl->ntask, copied to pinned memory after it) set later builds of the
  // size bucket to the most levels any of them used + kNfLevelSpare, so
  // that the graph does not carry ~6 kernels per level that finds no node to
  // split.  A cloud that needs more levels is still exact (its larger nodes
  // go to k_nf_small_global, slowly) and sends the next build back to the
  // full margin.
  int* nf_ntask_host = nullptr;       // pinned [kNfMaxLevels + 1]
  hipEvent_t nf_ntask_ev = nullptr;   // the copy's completion
  int nf_ntask_bucket = -1, nf_ntask_lmax = 0;   // the build the copy belongs to
  struct NfHint {
    int used_max = 0, hint = 0;   // hint 0: the full margin
  };
  std::map<int, NfHint> nf_hints;   // per size bucket: the next build's level count
  // a copied level count is ready to read (its build completed)
  bool nf_ntask_pending_check() const {
    return nf_ntask_bucket >= 0 && nf_ntask_ev && hipEventQuery(nf_ntask_ev) == hipSuccess;
  }
  bool profiling = false;
  std::vector<hipEvent_t> prof_ev;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // spatial sharding: ownership slab + RCCL communicator
  int own_axis = -1;
  float own_lo = -INFINITY, own_hi = INFINITY;
  int own_mod = 0, own_rem = 0;   // interleaved sharding (gicp_set_shard_groups)
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  DevBuf mom;          // [kSlabStride] reduced moments, all-reduced in place
  DevBuf search;       // correspondence search: [qstate f4 x n][key u64 x n][counters][tasks]
  bool speculate = true;    // queue a follow-on chunk before the first one's flag is seen
  bool comm_graphs = true;  // RCCL captured into the chunk graphs (else eager chunks)
  long captures = 0;        // chunk graphs captured (diagnostics: DDLO_GRAPH_DEBUG)
  // exact distance ties in nanoflann's order (gicp_set_tie_order): the tree
  // build scratch, the tied-query list and the resolvers' error word
  bool tie_exact = true;
  DevBuf nf_scratch, tie_buf, nf_err;
  int* nf_err_host = nullptr;   // pinned: [0] copy of nf_err, read after the entry point's final wait;
                                // [1] the last covariance pass's tied-query count
  // covariance ties without a tree (k_nf_lazy): each tied query's search
  // splits only the nodes it walks; a cloud with many ties gets the whole
  // tree instead (lazy_heavy: the previous pass listed more than 2 x the
  // lazy kernel's workgroups)
  bool tie_lazy = true;    // GICP_OPT_TIE_LAZY 0: the whole tree for covariance ties too
  int partial_levels = 3;  // big levels of the partial tree the lazy search starts from (GICP_OPT_TIE_PARTIAL_LEVELS)
  bool cov_tasks = false;  // GICP_OPT_COV_TASKS: the task-based kNN for covariances
  bool lazy_heavy = false;
  // nanoflann's tree on the ctx's own stream, not beside it (gicp_s2s_batch's
  // workers: the other workers fill the device, and a second stream per
  // worker shares the 4 hardware queues with them -- 0.44 against 0.55 ms per
  // pair at 4 workers, tools/batch_streams.py)
  bool nf_same_stream = false;
  // ... and then builds the partial tree after the covariance kernel, into
  // this ctx-owned tree, gated on the tie count (no work for a scan without
  // ties, about half of cfg 5's)
  std::unique_ptr<NfTreeData> nf_gated;
  DevBuf lazy_buf;
  hipEvent_t tie_cnt_ev = nullptr;   // recorded after the count's copy
  bool tie_cnt_pending = false;
  int lazy_wgs_last = 0;
  bool nf_err_pending = false;
  long ties_resolved = 0;       // diagnostics
  std::weak_ptr<NfTreeData> nf_joined;   // the target tree c->stream last waited for
  // slab shard: its restriction of the whole submap's nanoflann tree
  // (tietree.hip; gicp_set_tie_tree), which orders the in-align ties
  std::shared_ptr<NfTreeData> tie_tree;
  // tie builder (gicp_tie_builder_set): the whole submap, its tree, and the
  // buffers of the restrictions exported from it
  std::shared_ptr<CloudData> tie_whole;
  DevBuf tie_scratch, tie_lidx, tie_out_nodes, tie_out_pts, tie_counts;
  std::vector<unsigned char> tie_blob;   // the last exported restriction (gicp_tie_builder_export)
  // candidate cells of the target (gicp_set_target_grid): 0 off, 1 auto, 2 on
  int grid_mode = GICP_GRID_AUTO;
  DevBuf fb;                      // the lookup's walk list: [counters][list segments][masks]
  // stage timing of compute_cov (profiling on): covariance kernel, tree build, resolvers
  hipEvent_t st_ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  bool st_tree = false;          // the last compute_cov built a tree (events 2, 3 recorded)
  bool st_resolve = false;       // ... and ran the tie resolvers (events 4, 5)
  bool st_in_cov = false;        // a profiled compute_cov is running: only its own tree build is timed
};

namespace ddlo {
namespace rt {


inline const AlignState& final_state(const gicp_ctx* c) { return c->state_host[c->state_slot]; }

// Wait for the align's trailing no-op chunk (if one is still queued) before
// a ctx-owned buffer it touches may be released to the device pool.
inline gicp_status drain_tail(gicp_ctx* c) {
  if (c->tail_pending) {
    HIP_TRY(hipEventSynchronize(c->tail_ev));
    c->tail_pending = false;
  }
  return GICP_OK;
}

inline gicp_status set_device(const gicp_ctx* c) {
  HIP_TRY(hipSetDevice(c->device));
  return GICP_OK;
}

// Grow a ctx scratch buffer; work still queued on the stream may read the
// old block, so the stream is drained before it goes back to the pool.
inline hipError_t grow(DevBuf& b, size_t bytes, hipStream_t s) {
  if (bytes <= b.bytes && b.p) return hipSuccess;
  if (b.p) {
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
  }
  return b.ensure(bytes);
}

// xyz: host memory (copied to the device first), or device memory when
// on_device (e.g. a preprocessed scan or a keyframe of the odometry driver).
// check_finite = false (device clouds known finite): no read-back, and the
// call returns without waiting for the build.
inline gicp_status ensure_nftree(gicp_ctx* c, CloudData& cd, hipStream_t s);
inline gicp_status ensure_nftree_partial(gicp_ctx* c, CloudData& cd, hipStream_t s);

// nf_early: start nanoflann's tree of the cloud (ctx's aux stream) as soon
// as its sorted points exist, beside the rest of the index build -- for a
// cloud whose covariances follow (the odometry driver's scans and keyframes)
inline gicp_status build_cloud(gicp_ctx* c, const float* xyz, size_t n, size_t stride, std::shared_ptr<CloudData>* out,
                               bool on_device = false, bool check_finite = true, bool nf_early = false) {
  if (!xyz || n == 0 || stride < 12 || (stride % 4) != 0) return fail(GICP_EINVAL, "invalid cloud (null, empty or bad stride)");
  if (n > (size_t)INT32_MAX / 2) return fail(GICP_EINVAL, "cloud too large");
  auto cd = std::make_shared<CloudData>();
  // nf_early starts nanoflann's tree of cd on the aux stream; if this call
  // then fails (non-finite input, a HIP error), cd and its buffers go back
  // to the device pool: wait for the build first, so that no other ctx gets
  // a block the aux stream still writes (DevicePool: idle when released)
  struct AuxDrain {
    gicp_ctx* c;
    bool armed = false;
    ~AuxDrain() {
      if (armed) (void)hipStreamSynchronize(c->aux_stream);
    }
  } drain{c};
  const int N = (int)n;
  cd->n = N;
  cd->nlevels = levels_for(N, cd->lvl_cnt, cd->lvl_off);
  if (cd->nlevels < 0) return fail(GICP_EINVAL, "cloud too large for the search hierarchy");
  if (cd->upper_count() > 2048)  // LDS cache of levels >= 1 (64 KB): <= 4.2M points
    return fail(GICP_EINVAL, "cloud too large for the search hierarchy's LDS cache (max ~4.2M points)");
  const int total_boxes = cd->lvl_off[cd->nlevels - 1] + cd->lvl_cnt[cd->nlevels - 1];
  hipStream_t s = c->stream;
  const size_t raw_sz = (n - 1) * stride + 12;
  const unsigned char* raw = reinterpret_cast<const unsigned char*>(xyz);
  if (!on_device) {
    HIP_TRY(grow(c->raw_bytes, raw_sz, s));
    HIP_TRY(hipMemcpyAsync(c->raw_bytes.p, xyz, raw_sz, hipMemcpyHostToDevice, s));
    raw = c->raw_bytes.as<unsigned char>();
  }
  const int nb = (N + 255) / 256;
  HIP_TRY(grow(c->raw_pts, sizeof(float4) * n, s));
  HIP_TRY(grow(c->partial, sizeof(float) * 6 * nb, s));
  HIP_TRY(grow(c->nonfinite, sizeof(int), s));
  if (check_finite) HIP_TRY(hipMemsetAsync(c->nonfinite.p, 0, sizeof(int), s));   // (else never read)
  HIP_TRY(cd->quant.ensure(sizeof(float) * 8));
  launch_pack_bbox(s, raw, stride, N, c->raw_pts.as<float4>(), c->partial.as<float>(),
                   c->nonfinite.as<int>(), nb);
  launch_bbox_final(s, c->partial.as<float>(), nb, cd->quant.as<float>());
  HIP_TRY(grow(c->keys_tmp, sizeof(unsigned long long) * n, s));
  HIP_TRY(grow(c->vals_tmp, sizeof(int) * n, s));
  HIP_TRY(cd->keys.ensure(sizeof(unsigned long long) * n));
  HIP_TRY(cd->perm.ensure(sizeof(int) * n));
  launch_morton(s, c->raw_pts.as<float4>(), N, cd->quant.as<float>(), c->keys_tmp.as<unsigned long long>(),
                c->vals_tmp.as<int>());
  size_t tmp_bytes = 0;
  HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, c->keys_tmp.as<unsigned long long>(),
                                             cd->keys.as<unsigned long long>(), c->vals_tmp.as<int>(),
                                             cd->perm.as<int>(), N, 0, 63, s));
  HIP_TRY(grow(c->sort_tmp, tmp_bytes, s));
  tmp_bytes = c->sort_tmp.bytes;
  HIP_TRY(hipcub::DeviceRadixSort::SortPairs(c->sort_tmp.p, tmp_bytes, c->keys_tmp.as<unsigned long long>(),
                                             cd->keys.as<unsigned long long>(), c->vals_tmp.as<int>(),
                                             cd->perm.as<int>(), N, 0, 63, s));
  const int npad = cd->lvl_cnt[0] * kLeafSize;  // whole leaves, sentinel-padded
  HIP_TRY(cd->pts.ensure(sizeof(float4) * npad));
  HIP_TRY(cd->inv_perm.ensure(sizeof(int) * n));
  launch_gather(s, c->raw_pts.as<float4>(), cd->perm.as<int>(), N, npad, cd->pts.as<float4>(), cd->inv_perm.as<int>());
  // (a ctx building its trees on its own stream gates the partial tree on the
  // covariance pass's tie count instead: compute_cov)
  if (nf_early && c->tie_exact && !(c->nf_same_stream && c->tie_lazy && !c->lazy_heavy)) {
    drain.armed = true;
    gicp_status st = (c->tie_lazy && !c->lazy_heavy) ? ensure_nftree_partial(c, *cd, s) : ensure_nftree(c, *cd, s);
    if (st) return st;
  }
  HIP_TRY(cd->dir.ensure(sizeof(int) * (size_t)fine_dir_ints(N)));
  launch_key_dir(s, cd->keys.as<unsigned long long>(), N, cd->dir.as<int>());
  HIP_TRY(cd->soa.ensure(sizeof(float) * 3 * (size_t)npad));
  HIP_TRY(cd->box_lo.ensure(sizeof(float4) * total_boxes));
  HIP_TRY(cd->box_hi.ensure(sizeof(float4) * total_boxes));
  launch_leaf_soa_boxes(s, cd->pts.as<float4>(), N, cd->lvl_cnt[0], cd->soa.as<float>(), cd->box_lo.as<float4>(),
                        cd->box_hi.as<float4>());
  for (int l = 1; l < cd->nlevels; ++l)
    launch_level_boxes(s, cd->box_lo.as<float4>() + cd->lvl_off[l - 1], cd->box_hi.as<float4>() + cd->lvl_off[l - 1],
                       cd->lvl_cnt[l - 1], cd->lvl_cnt[l], cd->box_lo.as<float4>() + cd->lvl_off[l],
                       cd->box_hi.as<float4>() + cd->lvl_off[l]);
  HIP_TRY(hipGetLastError());
  if (check_finite) {
    HIP_TRY(hipMemcpyAsync(c->flag_host, c->nonfinite.p, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (*c->flag_host) return fail(GICP_ENONFINITE, "cloud contains non-finite coordinates");
  }
  *out = cd;
  drain.armed = false;   // the tree's owner (cd) lives on: its users wait on nf->ready
  return GICP_OK;
}

// Build nanoflann's tree of cd into t on the given stream.  stop >= 0 (the
// diagnostics entry only) runs that many big levels and nothing after;
// off (optional, 16 entries) receives the sizes and the scratch offsets.
// partial_levels >= 0: only that many big levels, then stubs (k_nf_stub).
inline gicp_status nftree_build(gicp_ctx* c, CloudData& cd, hipStream_t s_in, NfTreeData& tr, int stop = -1,
                                long long* off = nullptr, int partial_levels = -1, const int* gate = nullptr,
                                bool zero_nodes = false) {
  NfTreeData* t = &tr;
  const int n = cd.n;
  // the cloud is ready on s_in; the build runs on the aux stream
  static const bool same_env = dev_getenv("DDLO_NF_SAME_STREAM") != nullptr;   // A/B, diagnostics
  const bool same_stream = same_env || c->nf_same_stream;
  const hipStream_t s = same_stream ? s_in : c->aux_stream;
  if (!same_stream) {
    HIP_TRY(hipEventRecord(c->aux_ev, s_in));
    HIP_TRY(hipStreamWaitEvent(s, c->aux_ev, 0));
  }
  if (!t->ready) HIP_TRY(hipEventCreateWithFlags(&t->ready, hipEventDisableTiming));
  t->n = n;
  const bool timed = c->profiling && c->st_in_cov && c->st_ev[2] && stop < 0 && !off;
  if (timed) HIP_TRY(hipEventRecord(c->st_ev[2], s));
  // grids sized for a bucket of 16k points: one captured build graph serves
  // every cloud of the bucket (the kernels read the descriptor, and n, from
  // device memory), so a build is one graph launch, not ~80 kernel launches
  const int nbucket = (int)(((long)n + 16383) / 16384 * 16384);
  const NfSizes z = nf_sizes(nbucket);
  // the level count: the full margin for diagnostics builds, else from the
  // last completed build of this bucket on this ctx
  if (c->nf_ntask_pending_check()) {
    int used = 0;
    while (used < c->nf_ntask_lmax && c->nf_ntask_host[used] > 0) ++used;
    auto& h = c->nf_hints[c->nf_ntask_bucket];
    if (used >= c->nf_ntask_lmax) {
      h.hint = 0;   // every level had nodes to split: measure again with the full margin
    } else {
      h.used_max = std::max(h.used_max, used);
      h.hint = h.used_max + kNfLevelSpare;
    }
    c->nf_ntask_bucket = -1;
  }
  int Lmax = z.Lmax;
  const bool partial = partial_levels >= 0 && stop < 0 && !off;
  if (partial) Lmax = std::min(z.Lmax, partial_levels);
  if (stop < 0 && !off && !partial) {
    const auto it = c->nf_hints.find(nbucket);
    if (it != c->nf_hints.end() && it->second.hint > 0) Lmax = std::min(z.Lmax, it->second.hint);
  }
  t->cap = z.big_ids + 2 * n;   // big-level ids, then 2 per point for the small subtrees' ranges
  HIP_TRY(t->vpts.ensure(sizeof(float4) * (size_t)n));
  HIP_TRY(t->nodes.ensure(sizeof(NfNode) * (size_t)t->cap));
  if (zero_nodes) HIP_TRY(hipMemsetAsync(t->nodes.p, 0, t->nodes.bytes, s));   // unwritten slots read as non-nodes (tietree.hip)
  HIP_TRY(t->box.ensure(2 * sizeof(float4)));   // root_bbox
  HIP_TRY(t->status.ensure(2 * sizeof(int)));
  t->partial = partial;
  if (partial) HIP_TRY(t->sbox.ensure(2 * sizeof(float4) * (size_t)z.big_ids));
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t o_ctl = 0, o_tasks = o_ctl + al(sizeof(NfCtl)),
               o_pend = o_tasks + al(sizeof(NfTask) * (size_t)(z.Lmax + 1) * z.max_task),
               o_small = o_pend + al(sizeof(NfTask) * (size_t)(z.Lmax + 1) * z.max_pend),
               o_cmap = o_small + al(sizeof(NfTask) * (size_t)z.max_small),
               o_cA = o_cmap + al(sizeof(int) * 2 * (size_t)z.max_chunks),
               o_cAE = o_cA + al(sizeof(int) * (size_t)z.max_chunks),
               o_cE2 = o_cAE + al(sizeof(int) * (size_t)z.max_chunks),
               o_tblL = o_cE2 + al(sizeof(int) * (size_t)z.max_chunks),
               o_tblR = o_tblL + al(sizeof(float4) * (size_t)nbucket),
               o_ctask = o_tblR + al(sizeof(float4) * (size_t)nbucket),
               total = o_ctask + al(sizeof(NfTask) * 2 * (size_t)z.max_chunks);
  HIP_TRY(grow(c->nf_scratch, total, s));
  char* u = c->nf_scratch.as<char>();
  NfBuild b;
  b.vpts = t->vpts.as<float4>();
  b.nodes = t->nodes.as<NfNode>();
  b.box = t->box.as<float4>();
  b.cap = t->cap;
  b.ctl = reinterpret_cast<NfCtl*>(u + o_ctl);
  b.tasks = reinterpret_cast<NfTask*>(u + o_tasks);
  b.pend = reinterpret_cast<NfTask*>(u + o_pend);
  b.small = reinterpret_cast<NfTask*>(u + o_small);
  b.chunk_task = reinterpret_cast<int*>(u + o_cmap);
  b.ctask = reinterpret_cast<NfTask*>(u + o_ctask);
  b.cA = reinterpret_cast<int*>(u + o_cA);
  b.cAE = reinterpret_cast<int*>(u + o_cAE);
  b.cE2 = reinterpret_cast<int*>(u + o_cE2);
  b.tblL = reinterpret_cast<float4*>(u + o_tblL);
  b.tblR = reinterpret_cast<float4*>(u + o_tblR);
  b.quant = cd.quant.as<float>();
  b.sbox = partial ? t->sbox.as<float4>() : nullptr;
  b.sorted = cd.pts.as<float4>();
  b.gate = gate;
  b.n = n;
  b.nbucket = nbucket;
  b.Lmax = Lmax;
  b.max_task = z.max_task;
  b.max_pend = z.max_pend;
  b.max_small = z.max_small;
  b.max_chunks = z.max_chunks;
  b.big_ids = z.big_ids;
  if (off) {
    const long long v[16] = {Lmax, z.max_task, z.max_pend, z.max_small, z.max_chunks, (long long)o_tasks,
                             (long long)o_pend, (long long)o_small, (long long)o_cmap, (long long)o_cA,
                             (long long)o_cAE, (long long)o_cE2, (long long)o_tblL, (long long)total, n, t->cap};
    for (int i = 0; i < 16; ++i) off[i] = v[i];
  }
  HIP_TRY(c->nf_desc.ensure(sizeof(NfBuild)));
  NfBuild* db = c->nf_desc.as<NfBuild>();
  launch_nf_set_desc(s, b, db);   // by value as a kernel argument: no host buffer has to outlive the call
  static const bool no_graph = dev_getenv("DDLO_NF_NO_GRAPH") != nullptr;   // A/B, diagnostics
  if (stop >= 0 || no_graph || same_env) {
    launch_nf_build(s, b, db, stop);
    HIP_TRY(hipGetLastError());
  } else {
    const long long gkey = ((long long)nbucket * 64 + Lmax) * 2 + (partial ? 1 : 0);
    ++c->nf_clock;
    gicp_ctx::NfGraph* ng = nullptr;
    for (auto& e : c->nf_graphs)
      if (e.key == gkey) ng = &e;
    if (!ng) {
      if ((int)c->nf_graphs.size() < kNfGraphs) {
        c->nf_graphs.reserve(kNfGraphs);
        c->nf_graphs.emplace_back();
        ng = &c->nf_graphs.back();
      } else {   // evict the least recently used, after the builds queued on the stream
        ng = &c->nf_graphs[0];
        for (auto& e : c->nf_graphs)
          if (e.last_use < ng->last_use) ng = &e;
        HIP_TRY(hipStreamSynchronize(s));
        if (ng->ge) HIP_TRY(hipGraphExecDestroy(ng->ge));
        ng->ge = nullptr;
        ng->key = -1;
      }
      hipGraph_t g = nullptr;
      HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      launch_nf_build(s, b, db, -1);   // (b.sbox set: the partial build)
      const hipError_t e1 = hipGetLastError();
      const hipError_t e2 = hipStreamEndCapture(s, &g);
      HIP_TRY(e1);
      HIP_TRY(e2);
      const hipError_t e3 = hipGraphInstantiate(&ng->ge, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      HIP_TRY(e3);
      ng->key = gkey;
    }
    ng->last_use = c->nf_clock;
    HIP_TRY(hipGraphLaunch(ng->ge, s));
  }
  if (stop < 0 && !off && !partial) {   // the level counts of this build, for the next one
    if (!c->nf_ntask_host) {
      HIP_TRY(pinned_pool().alloc((void**)&c->nf_ntask_host, sizeof(int) * (kNfMaxLevels + 1), hipHostMallocDefault));
      HIP_TRY(hipEventCreateWithFlags(&c->nf_ntask_ev, hipEventDisableTiming));
    }
    HIP_TRY(hipMemcpyAsync(c->nf_ntask_host, b.ctl->ntask, sizeof(int) * (kNfMaxLevels + 1), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(c->nf_ntask_ev, s));
    c->nf_ntask_bucket = nbucket;
    c->nf_ntask_lmax = Lmax;
  }
  HIP_TRY(hipMemcpyAsync(t->status.p, &b.ctl->err, sizeof(int), hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemcpyAsync(t->status.as<int>() + 1, &b.ctl->nnodes, sizeof(int), hipMemcpyDeviceToDevice, s));
  if (timed) {
    HIP_TRY(hipEventRecord(c->st_ev[3], s));
    c->st_tree = true;
  }
  HIP_TRY(hipEventRecord(t->ready, s));
  return GICP_OK;
}

// stream s waits for the tree's build (enqueued, no host wait)
inline hipError_t nftree_join(const NfTreeData& t, hipStream_t s) { return hipStreamWaitEvent(s, t.ready, 0); }

// nanoflann's tree of a cloud (once per cloud, on the given stream)
inline gicp_status ensure_nftree(gicp_ctx* c, CloudData& cd, hipStream_t s) {
  if (cd.nf) return GICP_OK;
  auto t = std::make_shared<NfTreeData>();
  gicp_status st = nftree_build(c, cd, s, *t);
  if (st) return st;
  cd.nf = t;
  return GICP_OK;
}

// the top levels of nanoflann's tree (the lazy covariance tie search), once per cloud
inline gicp_status ensure_nftree_partial(gicp_ctx* c, CloudData& cd, hipStream_t s) {
  if (cd.nfp || cd.nf) return GICP_OK;
  auto t = std::make_shared<NfTreeData>();
  gicp_status st = nftree_build(c, cd, s, *t, -1, nullptr, c->partial_levels);
  if (st) return st;
  cd.nfp = t;
  return GICP_OK;
}

// the tied-query list ([count][list n]) and the resolvers' error word, reset on the stream
inline gicp_status tie_scratch(gicp_ctx* c, int n, hipStream_t s, TieList* tl) {
  // a point is listed at most twice (the task-based kNN, then the lane-per-query kernel for its group)
  HIP_TRY(grow(c->tie_buf, sizeof(int) * (2 * (size_t)n + 64), s));
  HIP_TRY(c->nf_err.ensure(sizeof(int)));
  if (!c->nf_err_host) HIP_TRY(pinned_pool().alloc((void**)&c->nf_err_host, 2 * sizeof(int), hipHostMallocDefault));
  if (!c->nf_err_pending) {
    HIP_TRY(hipMemsetAsync(c->nf_err.p, 0, sizeof(int), s));
    c->nf_err_pending = true;
  }
  HIP_TRY(hipMemsetAsync(c->tie_buf.p, 0, sizeof(int), s));
  tl->count = c->tie_buf.as<int>();
  tl->list = c->tie_buf.as<int>() + 64;
  tl->cap = 2 * n;
  return GICP_OK;
}

// at the start of an entry point: a tie error word left pending by an
// earlier call that failed before its check belongs to that call (already
// reported as its failure), not to this one
inline void begin_ties(gicp_ctx* c) { c->nf_err_pending = false; }

// after the entry point's final wait: a failed tie resolution is an error
// (the answers would silently carry the Morton tie order instead of nanoflann's)
inline gicp_status check_ties(gicp_ctx* c) {
  if (!c->nf_err_pending) return GICP_OK;
  c->nf_err_pending = false;
  const int e = *(volatile int*)c->nf_err_host;
  if (e)
    return fail(GICP_EHIP, "nanoflann tie order: the device kd-tree build or search failed (resolver bits " +
                               std::to_string(e & 255) + ", build bits " + std::to_string(e >> 8) + ")");
  return GICP_OK;
}

// enqueue the copy of the resolvers' error word that check_ties reads
inline gicp_status publish_ties(gicp_ctx* c, hipStream_t s) {
  if (c->nf_err_pending) HIP_TRY(hipMemcpyAsync(c->nf_err_host, c->nf_err.p, sizeof(int), hipMemcpyDeviceToHost, s));
  return GICP_OK;
}

// workgroups of the lazy tie search: one tied query each at a time, a
// private copy of the cloud each (scratch bounded by ~256 MB)
inline int lazy_workgroups(int n) {
  const size_t per = nf_lazy_bytes(n, 1) - nf_lazy_bytes(n, 0);
  return (int)std::max<size_t>(1, std::min<size_t>(64, (size_t(256) << 20) / std::max<size_t>(per, 1)));
}

// k_use > 0 overrides the ctx's k (a keyframe smaller than k, odom.hip)
inline gicp_status compute_cov(gicp_ctx* c, Side& side, int k_use = 0) {
  if (!side.cloud) return fail(GICP_ESTATE, "no cloud on this side");
  const int k = k_use > 0 ? k_use : c->params.k_correspondences;
  if (k <= 0 || k > 64) return fail(GICP_EINVAL, "k_correspondences must be in [1, 64]");
  if (side.cloud->n < k) return fail(GICP_ETOOFEW, "cloud has fewer points than k_correspondences");
  auto cv = std::make_shared<CovData>();
  cv->n = side.cloud->n;
  HIP_TRY(cv->cov6.ensure(sizeof(double) * 6 * (size_t)cv->n));
  if (c->profiling && !c->st_ev[0])
    for (auto& e : c->st_ev) HIP_TRY(hipEventCreate(&e));
  // stage times: only what this pass records (a tree built earlier, e.g. with
  // the index, is not this pass's; nothing is reported from an older pass)
  c->st_tree = false;
  c->st_resolve = false;
  struct InCov {
    gicp_ctx* c;
    ~InCov() { c->st_in_cov = false; }
  } in_cov{c};
  c->st_in_cov = c->profiling;
  // GICP_OPT_COV_TASKS: the task-based kNN (knn_tasks.hip) — exact, but not
  // faster than the lane-per-query kernel on the cfg 5 clouds
  const bool tasks = c->cov_tasks;
  const CloudDev cd = side.cloud->dev();
  // exact ties: the points whose k-th neighbour distance is tied get their
  // neighbourhood from nanoflann's own search (nftree.hip)
  TieList tl{nullptr, nullptr};
  // the previous pass's tie count (once its copy has landed): many ties make
  // the whole tree cheaper than one lazy search per tied query
  if (c->tie_cnt_pending && hipEventQuery(c->tie_cnt_ev) == hipSuccess) {
    c->lazy_heavy = c->nf_err_host[1] > 2 * std::max(c->lazy_wgs_last, 1);
    c->tie_cnt_pending = false;
  }
  const bool lazy = c->tie_exact && c->tie_lazy && !c->lazy_heavy && !side.cloud->nf;
  const bool gated = lazy && c->nf_same_stream && !side.cloud->nfp;
  if (c->tie_exact) {
    gicp_status st = gated ? GICP_OK
                     : lazy ? ensure_nftree_partial(c, *side.cloud, c->stream)
                            : ensure_nftree(c, *side.cloud, c->stream);
    if (!st) st = tie_scratch(c, side.cloud->n, c->stream, &tl);
    if (st) return st;
  }
  if (c->profiling) HIP_TRY(hipEventRecord(c->st_ev[0], c->stream));
  if (tasks && k <= 32) {
    // scratch of the task-based kNN; a queued covariance launch may still
    // read the old block, so growing it waits for the stream
    const int n = cv->n;
    const int cap = std::max(64, 6 * k);
    const int cap2 = 8 * cap, max2 = std::max(256, n / 64);   // second round: ~1 % of the points, longer lists
    const int cap_r = knn_task_cap_per_region(n);
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t o_q = 0, o_cnt = o_q + al(sizeof(float4) * ((size_t)(n + 15) / 16 * 16)),
                 o_redo = o_cnt + al(sizeof(unsigned) * (size_t)n), o_again = o_redo + al((size_t)(n + 63) / 64),
                 o_slot2 = o_again + al((size_t)n), o_n2 = o_slot2 + al(sizeof(int) * (size_t)n),
                 o_ctr = o_n2 + 256,
                 o_tasks = o_ctr + al(sizeof(unsigned) * kTaskRegions * kCtrStride),
                 o_cand = o_tasks + al(sizeof(unsigned long long) * (size_t)kTaskRegions * cap_r),
                 o_cand2 = o_cand + al(sizeof(unsigned long long) * (size_t)n * cap),
                 total = o_cand2 + sizeof(unsigned long long) * (size_t)max2 * cap2;
    if (total > c->knn.bytes) {
      HIP_TRY(hipStreamSynchronize(c->stream));
      HIP_TRY(c->knn.ensure(total));
    }
    char* u = c->knn.as<char>();
    KnnJob j;
    j.c = cd;
    j.k = k;
    j.method = c->params.regularization;
    j.cov6 = cv->cov6.as<double>();
    j.qstate = reinterpret_cast<float4*>(u + o_q);
    j.cnt = reinterpret_cast<unsigned*>(u + o_cnt);
    j.redo = reinterpret_cast<unsigned char*>(u + o_redo);
    j.again = reinterpret_cast<unsigned char*>(u + o_again);
    j.round = 1;
    j.slot2 = reinterpret_cast<int*>(u + o_slot2);
    j.n2 = reinterpret_cast<unsigned*>(u + o_n2);
    j.cand2 = reinterpret_cast<unsigned long long*>(u + o_cand2);
    j.cap2 = cap2;
    j.max2 = max2;
    j.task_ctr = reinterpret_cast<unsigned*>(u + o_ctr);
    j.tasks = reinterpret_cast<unsigned long long*>(u + o_tasks);
    j.cand = reinterpret_cast<unsigned long long*>(u + o_cand);
    j.cap = cap;
    j.task_cap_r = cap_r;
    j.split_extent = 5.0f;
    j.tie_list = tl.list;
    j.tie_count = tl.count;
    j.tie_cap = tl.cap;
    if (!launch_knn_covariances(c->stream, j, side.cloud->upper_count()))
      return fail(GICP_EINVAL, "unsupported k");
    launch_covariances(c->stream, cd, k, c->params.regularization, cv->cov6.as<double>(), j.redo, tl);
    if (dev_getenv("DDLO_COV_DEBUG")) {   // development: how many groups needed the fallback
      std::vector<unsigned char> r((n + 63) / 64);
      std::vector<unsigned> cn(n);
      HIP_TRY(hipMemcpyAsync(r.data(), j.redo, r.size(), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipMemcpyAsync(cn.data(), j.cnt, sizeof(unsigned) * n, hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      size_t nr = 0, over = 0, sum = 0, mx = 0;
      for (auto v : r) nr += v;
      for (auto v : cn) { over += v > (unsigned)cap; sum += v; mx = std::max<size_t>(mx, v); }
      std::fprintf(stderr, "[cov] n %d k %d redo groups %zu / %zu, points over cap %zu, mean cand %.1f max %zu\n", n, k,
                   nr, r.size(), over, (double)sum / n, mx);
    }
  } else if (!launch_covariances(c->stream, cd, k, c->params.regularization, cv->cov6.as<double>(), nullptr, tl)) {
    return fail(GICP_EINVAL, "unsupported k");
  }
  if (c->profiling) HIP_TRY(hipEventRecord(c->st_ev[1], c->stream));
  c->st_resolve = c->tie_exact && c->profiling;
  if (c->tie_exact) {
    if (lazy) {
      const int n = side.cloud->n;
      const int wgs = lazy_workgroups(n);
      HIP_TRY(grow(c->lazy_buf, nf_lazy_bytes(n, wgs), c->stream));
      if (gated) {   // after the covariance kernel, on the stream: no work when no query is tied
        if (!c->nf_gated) c->nf_gated = std::make_unique<NfTreeData>();
        gicp_status st = nftree_build(c, *side.cloud, c->stream, *c->nf_gated, -1, nullptr, c->partial_levels, tl.count);
        if (st) return st;
      }
      const NfTreeData& tp = gated ? *c->nf_gated : *side.cloud->nfp;
      HIP_TRY(nftree_join(tp, c->stream));
      if (c->profiling) HIP_TRY(hipEventRecord(c->st_ev[4], c->stream));
      if (!launch_nf_lazy(c->stream, tp.dev(), cd, nullptr, tl, k, c->params.regularization, cv->cov6.as<double>(),
                          nullptr, nullptr, c->lazy_buf.p, wgs, tp.status.as<int>(), c->nf_err.as<int>()))
        return fail(GICP_EINVAL, "nanoflann tie order: the lazy tie search cannot run (k > 64 or no partial tree)");
      if (c->profiling) HIP_TRY(hipEventRecord(c->st_ev[5], c->stream));
      c->lazy_wgs_last = wgs;
    } else {
      HIP_TRY(nftree_join(*side.cloud->nf, c->stream));
      if (c->profiling) HIP_TRY(hipEventRecord(c->st_ev[4], c->stream));
      launch_nf_resolve_cov(c->stream, side.cloud->nf->dev(), cd, tl, k, c->params.regularization,
                            cv->cov6.as<double>(), side.cloud->nf->status.as<int>(), c->nf_err.as<int>());
      if (c->profiling) HIP_TRY(hipEventRecord(c->st_ev[5], c->stream));
      c->lazy_wgs_last = lazy_workgroups(side.cloud->n);
    }
    if (c->tie_lazy) {   // the count for the next pass's choice
      if (!c->tie_cnt_ev) HIP_TRY(hipEventCreateWithFlags(&c->tie_cnt_ev, hipEventDisableTiming));
      HIP_TRY(hipMemcpyAsync(c->nf_err_host + 1, tl.count, sizeof(int), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipEventRecord(c->tie_cnt_ev, c->stream));
      c->tie_cnt_pending = true;
    }
    gicp_status st = publish_ties(c, c->stream);
    if (st) return st;
    static const bool dbg = dev_getenv("DDLO_TIE_DEBUG") != nullptr;   // development: tied queries per cloud
    if (dbg) {
      int cnt = 0;
      HIP_TRY(hipMemcpyAsync(&cnt, tl.count, sizeof(int), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      std::fprintf(stderr, "[ties] n %d k %d tied %d\n", side.cloud->n, k, cnt);
      if (const char* path = dev_getenv("DDLO_TIE_DUMP")) {   // the tied queries' original indices, one line per cloud
        const int m = std::min(cnt, tl.cap);
        std::vector<int> pos(m), perm(side.cloud->n);
        HIP_TRY(hipMemcpyAsync(pos.data(), tl.list, sizeof(int) * m, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(perm.data(), side.cloud->perm.p, sizeof(int) * perm.size(), hipMemcpyDeviceToHost,
                               c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (FILE* f = std::fopen(path, "a")) {
          std::fprintf(f, "%d %d", side.cloud->n, k);
          for (int p : pos) std::fprintf(f, " %d", p < side.cloud->n ? perm[p] : -1);
          std::fprintf(f, "\n");
          std::fclose(f);
        }
      }
    }
  }
  HIP_TRY(hipGetLastError());
  side.cov = cv;
  return GICP_OK;
}

// A cloud, covariance or tie-tree change: no linearization to report, and the
// next align sends its whole job (k_align_init keeps per-source values such as
// st->src_radius only across aligns whose job is unchanged; a new cloud may
// reuse the old one's pool blocks, so equal pointers do not prove the same cloud)
inline void invalidate_align(gicp_ctx* c) {
  c->have_align = false;
  c->job_last_valid = false;
}

}  // namespace rt
}  // namespace ddlo
