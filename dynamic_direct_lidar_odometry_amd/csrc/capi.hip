// capi.hip — host runtime behind include/ddlo_gicp.h.
//
// Owns device clouds (ref-counted, so swap/share are O(1)), builds the
// Morton-sorted search hierarchy (K1), and runs align() as ONE hipGraph:
//   k_align_init, then max_iterations x {k_linearize, k_lm_step}
// whose kernels become no-ops once the on-device LM has converged or
// failed.  The host synchronises once per align, to read back the pose.
#include <hip/hip_runtime.h>

#include <atomic>
#include <thread>

#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>  // types only: RCCL is dlopen'ed on first gicp_set_comm

#include <dlfcn.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <thread>
#include <vector>

#include "../../include/ddlo_gicp.h"
#include "gicp_types.hpp"
#include "launch.hpp"
#include "runtime.hpp"
#include "cellgrid.hpp"
#include "nftree.hpp"   // kNfStack: the search depth a tie tree must fit
#include "devknobs.hpp"


namespace {

// RCCL entry points, resolved at run time so the single-GPU library carries
// no link dependency on RCCL.  dlopen by soname: in a process that already
// loaded torch, this returns torch's RCCL, which shares torch's HIP runtime
// with this library (same libamdhip64.so.7 soname), so streams are compatible.
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;   // gicp_set_tie_trees_from_root
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok = false;
  std::string why;
};

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      x.why = std::string("cannot load RCCL: ") + (e ? e : "?");
      return x;
    }
    x.get_unique_id = (decltype(x.get_unique_id))dlsym(h, "ncclGetUniqueId");
    x.comm_init_rank = (decltype(x.comm_init_rank))dlsym(h, "ncclCommInitRank");
    x.comm_destroy = (decltype(x.comm_destroy))dlsym(h, "ncclCommDestroy");
    x.all_reduce = (decltype(x.all_reduce))dlsym(h, "ncclAllReduce");
    x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
    x.broadcast = (decltype(x.broadcast))dlsym(h, "ncclBroadcast");
    x.send = (decltype(x.send))dlsym(h, "ncclSend");
    x.recv = (decltype(x.recv))dlsym(h, "ncclRecv");
    x.group_start = (decltype(x.group_start))dlsym(h, "ncclGroupStart");
    x.group_end = (decltype(x.group_end))dlsym(h, "ncclGroupEnd");
    x.ok = x.get_unique_id && x.comm_init_rank && x.comm_destroy && x.all_reduce && x.error_string;
    if (!x.ok) x.why = "RCCL is missing an entry point";
    return x;
  }();
  return r;
}

#define NCCL_TRY(expr)                                                                      \
  do {                                                                                      \
    ncclResult_t _r = (expr);                                                               \
    if (_r != ncclSuccess)                                                                  \
      return fail(GICP_ECOMM, std::string(#expr) + ": " + rccl().error_string(_r));         \
  } while (0)


// Tuning knob of the search (development; the default is the tuned value)
constexpr float kSplitExtentDefault = 5.0f;
float env_float(const char* name, float dflt) {
  const char* v = dev_getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  const float f = std::strtof(v, &end);
  return (end && end != v && f >= 0.f) ? f : dflt;
}

int env_int(const char* name, int dflt) {
  const char* v = dev_getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

// Options (gicp_set_option): the values new contexts take.  A -DDDLO_DEV
// build still reads the old A/B environment variables as the initial values.
static std::atomic<int> g_opt_default[GICP_OPT_COUNT] = {{0}, {1}, {1}, {3}, {0}, {0}};
static const bool g_opt_env_read = [] {
  auto rd = [](const char* name, int opt, bool flag) {
    const char* v = dev_getenv(name);
    if (v && *v) g_opt_default[opt].store(flag ? (*v != '0') : std::max(0, std::atoi(v)));
  };
  rd("DDLO_TIE_EXACT", GICP_OPT_TIE_ORDER, true);
  rd("DDLO_TIE_LAZY", GICP_OPT_TIE_LAZY, true);
  rd("DDLO_TIE_PARTIAL_LEVELS", GICP_OPT_TIE_PARTIAL_LEVELS, false);
  rd("DDLO_COV_TASKS", GICP_OPT_COV_TASKS, true);
  return true;
}();

static gicp_status check_option(int option, int value) {
  if (option <= 0 || option >= GICP_OPT_COUNT) return fail(GICP_EINVAL, "unknown option");
  const bool ok = option == GICP_OPT_TIE_PARTIAL_LEVELS ? (value >= 0 && value <= 24)
                  : option == GICP_OPT_GRID_MAX_MB        ? value >= 0
                                                          : (value == 0 || value == 1);
  if (!ok) return fail(GICP_EINVAL, "option value out of range");
  return GICP_OK;
}

// The search's development knobs, read from the environment once per
// process, not on every align (host time between aligns).
struct SearchKnobs {
  float split_extent, hard_extent, probe, probe_d, tri_mv, reuse_gap, reuse_gap0, reuse_rec_eps, reuse_rec_conv;
  int xcd_scan, pf_ratio, hard_blocks, prev_window, reuse, reuse_rec0, tie_scan, tie_ab;
};
const SearchKnobs& search_knobs() {
  static const SearchKnobs k = [] {
    SearchKnobs v;
    v.split_extent = env_float("DDLO_SPLIT_EXTENT", kSplitExtentDefault);
    v.xcd_scan = env_int("DDLO_XCD_SCAN", 1);
    v.pf_ratio = env_int("DDLO_PF_RATIO", 2);
    v.hard_extent = env_float("DDLO_HARD_EXTENT", 4.0f);
    v.hard_blocks = env_int("DDLO_HARD_BLOCKS", 10);
    v.prev_window = env_int("DDLO_PREV_WINDOW", 2);
    v.tri_mv = env_float("DDLO_TRI_MV", 0.2f);
    v.probe = env_float("DDLO_PROBE", 1.0f);
    v.probe_d = env_float("DDLO_PROBE_D", 0.5f);
    v.reuse = env_int("DDLO_REUSE", 1);
    v.reuse_gap = env_float("DDLO_REUSE_GAP", 0.05f);
    v.reuse_gap0 = env_float("DDLO_REUSE_GAP0", 0.f);
    v.reuse_rec0 = env_int("DDLO_REUSE_REC0", 0);
    v.reuse_rec_eps = env_float("DDLO_REUSE_REC_EPS", 0.05f);
    v.reuse_rec_conv = env_float("DDLO_REUSE_REC_CONV", 10.f);
    v.tie_ab = env_int("DDLO_TIE_AB", 0);
    v.tie_scan = env_int("DDLO_TIE_SCAN", 4);   // 1 / 2 / 3 / 4 (see AlignJob::tie_scan); 0 = A/B only
    return v;
  }();
  return k;
}

// byte layout of ctx->search for ns source points
struct SearchLayout {
  size_t qstate, key, ctr, hard_list, hard_flag, grp_blocks, ref, ref_p, sec, key2, tasks, total;
  int cap_r;
  explicit SearchLayout(int ns) {
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    cap_r = task_cap_per_region(ns);
    qstate = 0;
    key = al(sizeof(float4) * (size_t)ns);
    ctr = key + al(sizeof(unsigned long long) * (size_t)ns);
    hard_list = ctr + al(sizeof(unsigned) * (kTaskCounters + 1) * kCtrStride);   // + the moment kernel's arrival counter
    hard_flag = hard_list + al(sizeof(int) * kHardMax);
    grp_blocks = hard_flag + al((size_t)ns / 16 + 16);
    ref = grp_blocks + al(sizeof(unsigned short) * ((size_t)ns / 16 + 16));
    ref_p = ref + al(sizeof(float4) * (size_t)ns);
    sec = ref_p + al(sizeof(float4) * (size_t)ns);
    key2 = sec + al(sizeof(unsigned) * (size_t)ns);
    tasks = key2 + al(sizeof(unsigned long long) * (size_t)ns);
    total = tasks + sizeof(unsigned long long) * (size_t)kTaskRegions * cap_r;
  }
};

// the search bound of an align: nextafter(float(max_corr^2), +inf) (AlignJob::cap2)
float search_cap2(const gicp_params& p) {
  const double r = p.max_correspondence_distance;
  float f = (float)(r * r);
  if (!std::isfinite(f)) f = FLT_MAX;
  return std::nextafter(f, INFINITY);
}

// The target's candidate cells answer this ctx's searches (same bound)
bool grid_active(const gicp_ctx* c) {
  if (!c->grid_mode || !c->tgt.cloud) return false;
  const auto& g = c->tgt.cloud->grid;
  return g && g->ok && g->cap2 == search_cap2(c->params);
}

// byte layout of ctx->fb (the lookup's walk list) for ns source points
struct FbLayout {
  size_t ctr, list, mask, total;
  int seg_cap;
  explicit FbLayout(int ns) {
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    seg_cap = (ns + 15) / 16 + 1;
    ctr = 0;
    list = al(sizeof(unsigned) * (kFbSegs + 1) * 32);   // + the align's total
    mask = list + al(sizeof(int) * (size_t)kFbSegs * seg_cap);
    total = mask + al(sizeof(unsigned short) * (size_t)seg_cap);
  }
};

// ---------------------------------------------------------------------------
// Candidate cells of a target (cellgrid.hip): coarse cells of
// kGridCell metres over the target's box plus the bound's reach, split up to
// 3 times where lists are longer than kGridListMax points.
constexpr double kGridCell = 0.4;
constexpr double kGridMaxReach = 4.0;     // bounds beyond this: cells farther than it use the walk
constexpr int kGridListMax = 32;
constexpr int kGridAutoAligns = 32;       // GICP_GRID_AUTO: built at this align against the same target and bound
constexpr int kGridListCap = kCgCandMax;  // finest level: longer lists are not stored (the walk)
constexpr long kGridMaxCells = 48L << 20; // coarse cells (the directory is 8 B per cell)

gicp_status cellgrid_build(gicp_ctx* c, CloudData& cd, float cap2, std::shared_ptr<CellGridData>* out) {
  hipStream_t s = c->stream;
  auto g = std::make_shared<CellGridData>();
  g->cap2 = cap2;
  *out = g;
  float q[8];
  HIP_TRY(hipMemcpyAsync(q, cd.quant.p, sizeof(float) * 7, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const double S = kGridCell;
  const double capm = std::sqrt((double)cap2) * (1.0 + 1e-5) + 1e-6;
  const double reach = std::min(capm, kGridMaxReach);
  const int r = (int)std::ceil(reach / S) + 1;
  const double M = (r + 1) * S;   // the box: the target's bbox plus M on every side
  double lo[3], ext[3];
  long dims[3];
  double amax = 0.0;
  for (int a = 0; a < 3; ++a) {
    lo[a] = (double)q[a] - M;
    ext[a] = (double)q[4 + a] - (double)q[a] + 2 * M;
    dims[a] = (long)std::ceil(ext[a] / S) + 1;
    amax = std::max({amax, std::fabs((double)q[a]), std::fabs((double)q[4 + a])});
  }
  const long ncells = dims[0] * dims[1] * dims[2];
  if (ncells > kGridMaxCells || !std::isfinite(ext[0] + ext[1] + ext[2])) return GICP_OK;   // not built: the walk
  const size_t cap_bytes = c->grid_max_mb > 0 ? ((size_t)c->grid_max_mb << 20) : ~(size_t)0;
  if ((size_t)ncells * sizeof(unsigned long long) > cap_bytes)
    return fail(GICP_ENOMEM, "candidate cells: the directory exceeds GICP_OPT_GRID_MAX_MB");
  hipEvent_t e0, e1;
  HIP_TRY(hipEventCreate(&e0));
  HIP_TRY(hipEventCreate(&e1));
  struct EvGuard {
    hipEvent_t a, b;
    ~EvGuard() {
      (void)hipEventDestroy(a);
      (void)hipEventDestroy(b);
    }
  } evg{e0, e1};
  HIP_TRY(hipEventRecord(e0, s));
  CgBuild b{};
  b.tgt = cd.dev();
  // the build's geometry is the lookup's fp32 origin and scale, exactly
  b.fox = (float)lo[0]; b.foy = (float)lo[1]; b.foz = (float)lo[2];
  b.inv_s = (float)(1.0 / S);
  b.ox = b.fox; b.oy = b.foy; b.oz = b.foz;
  b.s = 1.0 / (double)b.inv_s;
  b.nx = (int)dims[0]; b.ny = (int)dims[1]; b.nz = (int)dims[2];
  b.r = r;
  // the lookup maps a query to its cell in fp32: |error| <~ 3 ulp of the
  // coordinate; every box is widened by delta to cover it
  b.delta = 1e-4 + 4e-6 * (amax + M + S);
  b.capm = capm;
  b.nomatch_dist = (r - 1) * S - 1e-3;
  static const int lmax_env = [] {   // development A/B of the list length (DDLO_GRID_LMAX)
    const char* v = dev_getenv("DDLO_GRID_LMAX");
    return v && *v ? std::atoi(v) : 0;
  }();
  b.lmax = lmax_env > 0 ? lmax_env : kGridListMax;
  b.lcap = kGridListCap;
  const bool outside_nomatch = capm <= b.nomatch_dist;
  // scratch
  const long nbx = (dims[0] + 3) / 4, nby = (dims[1] + 3) / 4, nbz = (dims[2] + 3) / 4;
  const long nblocked = nbx * nby * nbz * 64;
  {   // the per-cell scratch and directory (~21 B per coarse cell) must fit in free device memory with room
      // for the lists; otherwise the build is not attempted (the walk answers: maybe_build_grid)
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && (size_t)ncells * 21 + ((size_t)256 << 20) > fr)
      return fail(GICP_ENOMEM, "candidate cells: not enough free device memory for the build");
  }
  DevBuf rep, rep_tmp, flags, ctr, band, dnum, cub_tmp, cnn, db_buf;
  HIP_TRY(rep.ensure(sizeof(int) * (size_t)ncells));
  HIP_TRY(rep_tmp.ensure(sizeof(int) * (size_t)ncells));
  HIP_TRY(flags.ensure((size_t)std::max(nblocked, ncells)));
  HIP_TRY(ctr.ensure(sizeof(unsigned) * kCgCtrWords));
  HIP_TRY(band.ensure(sizeof(int) * (size_t)ncells));
  HIP_TRY(dnum.ensure(sizeof(int) * 8));
  HIP_TRY(db_buf.ensure(sizeof(CgBuild)));
  HIP_TRY(g->dir.ensure(sizeof(unsigned long long) * (size_t)ncells));
  b.rep = rep.as<int>();
  b.rep_tmp = rep_tmp.as<int>();
  b.rep_final = rep.as<int>();   // x: rep -> tmp, y: tmp -> rep, z: rep -> tmp; see below
  b.dir = g->dir.as<unsigned long long>();
  b.band = band.as<int>();
  b.ctr = ctr.as<unsigned>();
  CgBuild* db = db_buf.as<CgBuild>();
  auto upload = [&]() -> hipError_t { return hipMemcpyAsync(db, &b, sizeof(CgBuild), hipMemcpyHostToDevice, s); };
  b.rep_final = rep_tmp.as<int>();
  HIP_TRY(upload());
  HIP_TRY(hipMemsetAsync(rep.p, 0x7f, sizeof(int) * (size_t)ncells, s));   // 0x7f7f7f7f: none (> any position)
  HIP_TRY(hipMemsetAsync(ctr.p, 0, sizeof(unsigned) * kCgCtrWords, s));
  launch_cg_occ(s, db, cd.n);
  launch_cg_prop(s, db, 0, b.rep, b.rep_tmp, ncells);
  launch_cg_prop(s, db, 1, b.rep_tmp, b.rep, ncells);
  launch_cg_prop(s, db, 2, b.rep, b.rep_tmp, ncells);   // band: rep_tmp != none
  launch_cg_dir_fill(s, b.dir, b.rep_tmp, ncells, outside_nomatch ? kCgNoMatch : kCgFallback);
  launch_cg_band_flags(s, db, b.rep_tmp, flags.as<unsigned char>(), nblocked);
  HIP_TRY(hipGetLastError());
  // band cells in blocked order (selected blocked ids; k_cg_centers turns them into cell ids)
  auto select = [&](const unsigned char* fl, long n, int* outp, int* nsel) -> gicp_status {
    size_t tb = 0;
    hipcub::CountingInputIterator<int> it(0);
    HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, it, fl, outp, dnum.as<int>(), (int)n, s));
    HIP_TRY(cub_tmp.ensure(std::max<size_t>(tb, 256)));
    tb = cub_tmp.bytes;
    HIP_TRY(hipcub::DeviceSelect::Flagged(cub_tmp.p, tb, it, fl, outp, dnum.as<int>(), (int)n, s));
    HIP_TRY(hipMemcpyAsync(c->flag_host, dnum.p, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *nsel = *c->flag_host;
    return GICP_OK;
  };
  int nband = 0;
  gicp_status st = select(flags.as<unsigned char>(), nblocked, b.band, &nband);
  if (st) return st;
  g->info.coarse_cells = ncells;
  g->info.band_cells = nband;
  g->info.cell_size = (float)S;
  // level-0 lists
  DevBuf hdr[4], pool[4], cmax[4], sband[4], sparent[4], fin_sel[4], fl_final, fl_next;
  int nfin[4] = {0, 0, 0, 0}, nslot[4] = {0, 0, 0, 0};
  if (nband > 0) {
    HIP_TRY(cnn.ensure(sizeof(int) * (size_t)nband));
    b.cnn = cnn.as<int>();
    HIP_TRY(upload());
    launch_cg_centers(s, db, nband);
    HIP_TRY(hdr[0].ensure(sizeof(uint2) * (size_t)nband));
    HIP_TRY(fl_final.ensure((size_t)nband));
    HIP_TRY(fl_next.ensure((size_t)nband));
    nslot[0] = nband;
  }
  std::vector<unsigned> counters(kCgCtrWords);
  auto read_counters = [&]() -> gicp_status {
    HIP_TRY(hipMemcpyAsync(counters.data(), ctr.p, sizeof(unsigned) * kCgCtrWords, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return GICP_OK;
  };
  for (int l = 0; l <= kCgMaxLevel && nslot[l] > 0; ++l) {
    const long nf = 1L << (3 * l);
    // the level's lists: pools sized from the parent level, doubled on overflow
    // (a wave's chunks leave at most kCgChunk unused entries per shard range)
    size_t used_above = 0;
    if (l > 0)
      for (int k = 0; k < kCgShardsHost; ++k) used_above += counters[(kCgCounters + (l - 1) * kCgShardsHost + k) * 32];
    size_t pcap = l == 0 ? (size_t)nband * 64 + (1u << 23) : 3 * used_above + (size_t)nslot[l] * nf * 4 + (1u << 23);
    for (int attempt = 0;; ++attempt) {
      pcap = std::min<size_t>(pcap, 0xfff00000u);
      HIP_TRY(pool[l].ensure(sizeof(unsigned) * pcap));
      b.lv[l].pool = pool[l].as<unsigned>();
      b.lv[l].pool_cap = (unsigned)(pcap / kCgShardsHost * kCgShardsHost);
      if (l > 0) {
        HIP_TRY(hdr[l].ensure(sizeof(uint2) * (size_t)nslot[l] * nf));
        b.lv[l].hdr = hdr[l].as<uint2>();
      } else {
        b.lv[0].hdr = hdr[0].as<uint2>();
      }
      HIP_TRY(upload());
      HIP_TRY(hipMemsetAsync(ctr.as<unsigned>() + (kCgCounters + l * kCgShardsHost) * 32, 0,
                             sizeof(unsigned) * kCgShardsHost * 32, s));
      HIP_TRY(hipMemsetAsync(ctr.as<unsigned>() + kCtrPoolFull * 32, 0, sizeof(unsigned), s));
      if (l == 0) launch_cg_coarse(s, db, nband);
      else launch_cg_refine(s, db, l, nslot[l]);
      HIP_TRY(hipGetLastError());
      st = read_counters();
      if (st) return st;
      if (!counters[kCtrPoolFull * 32]) break;
      if (attempt >= 4 || pcap >= 0xfff00000u) return fail(GICP_ENOMEM, "candidate cells: list pool overflow");
      pcap *= 2;
    }
    // decisions: final at this level, or split once more
    HIP_TRY(fl_final.ensure((size_t)nslot[l]));
    HIP_TRY(fl_next.ensure((size_t)nslot[l]));
    launch_cg_decide(s, db, l, nslot[l], fl_final.as<unsigned char>(), fl_next.as<unsigned char>());
    HIP_TRY(fin_sel[l].ensure(sizeof(int) * (size_t)nslot[l]));
    st = select(fl_final.as<unsigned char>(), nslot[l], fin_sel[l].as<int>(), &nfin[l]);
    if (st) return st;
    if (l < kCgMaxLevel) {
      HIP_TRY(sparent[l + 1].ensure(sizeof(int) * (size_t)nslot[l] + 64));
      int nn = 0;
      st = select(fl_next.as<unsigned char>(), nslot[l], sparent[l + 1].as<int>(), &nn);
      if (st) return st;
      nslot[l + 1] = nn;
      if (nn > 0) {
        HIP_TRY(sband[l + 1].ensure(sizeof(int) * (size_t)nn));
        HIP_TRY(cmax[l + 1].ensure(sizeof(int) * (size_t)nn));
        b.lv[l + 1].slot_parent = sparent[l + 1].as<int>();
        b.lv[l + 1].slot_band = sband[l + 1].as<int>();
        b.lv[l + 1].cmax = cmax[l + 1].as<int>();
        b.lv[l + 1].slot_cap = nn;
        HIP_TRY(upload());
        launch_cg_slots(s, db, l + 1, nn);
      }
    }
  }
  // emission: per level, list entries and fine cells of each final, scanned
  DevBuf ent_n[4], fine_n[4];
  unsigned ent_base[5] = {0, 0, 0, 0, 0}, fine_base[5] = {0, 0, 0, 0, 0};
  for (int l = 0; l <= kCgMaxLevel; ++l) {
    ent_base[l + 1] = ent_base[l];
    fine_base[l + 1] = fine_base[l];
    g->info.level_cells[l] = nfin[l];
    if (nfin[l] == 0) continue;
    HIP_TRY(ent_n[l].ensure(sizeof(unsigned) * ((size_t)nfin[l] + 1)));
    HIP_TRY(fine_n[l].ensure(sizeof(unsigned) * ((size_t)nfin[l] + 1)));
    launch_cg_emit_count(s, db, l, fin_sel[l].as<int>(), nfin[l], ent_n[l].as<unsigned>(), fine_n[l].as<unsigned>());
    for (DevBuf* v : {&ent_n[l], &fine_n[l]}) {
      // exclusive scan in place over nfin + 1 entries (the last one = the total)
      HIP_TRY(hipMemsetAsync(v->as<unsigned>() + nfin[l], 0, sizeof(unsigned), s));
      size_t tb = 0;
      HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, v->as<unsigned>(), v->as<unsigned>(), nfin[l] + 1, s));
      HIP_TRY(cub_tmp.ensure(std::max<size_t>(tb, 256)));
      tb = cub_tmp.bytes;
      HIP_TRY(hipcub::DeviceScan::ExclusiveSum(cub_tmp.p, tb, v->as<unsigned>(), v->as<unsigned>(), nfin[l] + 1, s));
    }
    unsigned tot[2];
    HIP_TRY(hipMemcpyAsync(&tot[0], ent_n[l].as<unsigned>() + nfin[l], sizeof(unsigned), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&tot[1], fine_n[l].as<unsigned>() + nfin[l], sizeof(unsigned), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    ent_base[l + 1] += tot[0];
    fine_base[l + 1] += tot[1];
  }
  if ((size_t)fine_base[4] >= 0x3ffffffeu) return fail(GICP_ENOMEM, "candidate cells: fine table too large");
  if ((size_t)ncells * sizeof(unsigned long long) + sizeof(uint2) * (size_t)fine_base[4] +
          sizeof(float4) * (size_t)ent_base[4] > cap_bytes)
    return fail(GICP_ENOMEM, "candidate cells: the lists exceed GICP_OPT_GRID_MAX_MB");
  HIP_TRY(g->fine.ensure(sizeof(uint2) * std::max<size_t>(fine_base[4], 1)));
  HIP_TRY(g->ent.ensure(sizeof(float4) * std::max<size_t>(ent_base[4], 1)));
  b.fine = g->fine.as<uint2>();
  b.ent = g->ent.as<float4>();
  HIP_TRY(upload());
  for (int l = 0; l <= kCgMaxLevel; ++l)
    if (nfin[l] > 0)
      launch_cg_emit_write(s, db, l, fin_sel[l].as<int>(), nfin[l], ent_n[l].as<unsigned>(), fine_n[l].as<unsigned>(),
                           ent_base[l], fine_base[l]);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(e1, s));
  st = read_counters();   // (waits for the build)
  if (st) return st;
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
  g->info.build_ms = ms;
  g->info.nomatch_cells = nband - nfin[0] - nslot[1];   // band cells neither final at level 0 nor split
  g->info.overflow_cells = counters[kCtrOverflow * 32];
  g->info.fallback_fine = counters[kCtrFineFb * 32];
  g->info.fine_cells = (int64_t)fine_base[4] - g->info.fallback_fine;
  g->info.entries = ent_base[4];
  g->info.bytes = (int64_t)(g->dir.bytes + g->fine.bytes + g->ent.bytes);
  {   // the build's transient scratch at its peak (released on return)
    size_t sb = rep.bytes + rep_tmp.bytes + flags.bytes + ctr.bytes + band.bytes + dnum.bytes + cub_tmp.bytes +
                cnn.bytes + db_buf.bytes + fl_final.bytes + fl_next.bytes;
    for (int l = 0; l <= kCgMaxLevel; ++l)
      sb += hdr[l].bytes + pool[l].bytes + cmax[l].bytes + sband[l].bytes + sparent[l].bytes + fin_sel[l].bytes +
            ent_n[l].bytes + fine_n[l].bytes;
    g->info.scratch_bytes = (int64_t)sb;
  }
  g->info.built = 1;
  CellGridDev& d = g->dev;
  d.dir = g->dir.as<unsigned long long>();
  d.fine = g->fine.as<uint2>();
  d.ent = g->ent.as<float4>();
  d.ox = b.fox;
  d.oy = b.foy;
  d.oz = b.foz;
  d.inv_s = b.inv_s;
  d.nx = b.nx;
  d.ny = b.ny;
  d.nz = b.nz;
  d.outside_nomatch = outside_nomatch ? 1 : 0;
  d.has_fallback = (g->info.fallback_fine > 0 || !outside_nomatch) ? 1 : 0;
  g->info.uses_walk = d.has_fallback;
  g->ok = true;
  return GICP_OK;
}

// gicp_set_target_grid policy: build the target's candidate cells for this
// ctx's bound (auto: at the kGridAutoAligns-th (32nd) align against the same
// target and bound)
gicp_status maybe_build_grid(gicp_ctx* c) {
  if (!c->grid_mode || !c->tgt.cloud) return GICP_OK;
  CloudData& t = *c->tgt.cloud;
  const float cap2 = search_cap2(c->params);
  if (t.grid && t.grid->cap2 == cap2) return GICP_OK;   // built (or found too large) for this bound
  if (t.grid_aligns_cap2 != cap2) {
    t.grid_aligns_cap2 = cap2;
    t.grid_aligns = 0;
  }
  ++t.grid_aligns;
  // auto: only a target aligned against many times pays for its cells (a
  // ~16 ms build for a 500k-point submap against ~0.15 ms saved per align);
  // OdomNode's submaps live ~20 scans (DESIGN.md §4 "Candidate cells")
  if (c->grid_mode == GICP_GRID_AUTO && t.grid_aligns < kGridAutoAligns) return GICP_OK;
  std::shared_ptr<CellGridData> g;
  const gicp_status s = cellgrid_build(c, t, cap2, &g);
  if (s) {
    // The cells are an optional speed-up: a build that fails (pool or table
    // limits, the byte budget, device memory) leaves this target on the walk
    // for this bound and is not retried.  Only a device fault (the stream no
    // longer synchronizes) is the align's error.
    g.reset();   // its partial buffers are released (nothing queued reads them)
    (void)hipGetLastError();
    if (hipStreamSynchronize(c->stream) != hipSuccess) return s;
    auto none = std::make_shared<CellGridData>();
    none->cap2 = cap2;
    none->info.build_status = s;
    t.grid = none;
    g_last_error.clear();
    return GICP_OK;
  }
  t.grid = g;
  return GICP_OK;
}

// Just before k_align_init reads the pinned job: whole (job_full = 1) unless
// only the guess changed since the job it last copied whole, whose device copy
// is still in place (k_align_init alone writes the device job).
// finalize_job records the job as the device's copy before anything is
// launched; an error return before the launch has happened must forget it,
// or the next align would send only its guess to a device job that never
// received this one (JobCommit: armed after finalize_job, done() once the
// launch succeeded).
struct JobCommit {
  gicp_ctx* c;
  bool ok = false;
  explicit JobCommit(gicp_ctx* ctx) : c(ctx) {}
  void done() { ok = true; }
  ~JobCommit() {
    if (!ok) c->job_last_valid = false;
  }
};

void finalize_job(gicp_ctx* c) {
  AlignJob& j = *c->job_host;
  j.job_full = 0;
  AlignJob probe = j;
  std::memcpy(probe.guess_R, c->job_last.guess_R, sizeof(probe.guess_R));
  std::memcpy(probe.guess_t, c->job_last.guess_t, sizeof(probe.guess_t));
  probe.job_full = c->job_last.job_full;
  probe.ticket = c->job_last.ticket;
  if (!c->job_last_valid || std::memcmp(&probe, &c->job_last, sizeof(AlignJob)) != 0) {
    j.job_full = 1;
    c->job_last = j;
    c->job_last_valid = true;
  }
}

gicp_status fill_job(gicp_ctx* c, const float* guess16, int nblocks) {
  const SearchKnobs& kn = search_knobs();
  AlignJob& j = *c->job_host;
  std::memset(&j, 0, sizeof(j));
  j.src = c->src.cloud->dev();
  j.tgt = c->tgt.cloud->dev();
  j.src_cov = c->src.cov->cov6.as<double>();
  j.tgt_cov = c->tgt.cov->cov6.as<double>();
  j.corr = c->corr.as<int>();
  j.sqd = c->sqd.as<float>();
  j.slab = c->slab.as<double>();
  j.state = c->state_dev.as<AlignState>();
  j.ticket = (++c->ticket) & ((1ull << 47) - 1);
  j.stats = c->stats_on ? c->stats.as<unsigned int>() : nullptr;
  for (int r = 0; r < 3; ++r) {
    for (int cc = 0; cc < 3; ++cc) j.guess_R[3 * r + cc] = guess16 ? (double)guess16[4 * r + cc] : (r == cc ? 1.0 : 0.0);
    j.guess_t[r] = guess16 ? (double)guess16[4 * r + 3] : 0.0;
  }
  const double r = c->params.max_correspondence_distance;
  j.max_corr2 = r * r;
  float f = (float)j.max_corr2;
  if (!std::isfinite(f)) f = FLT_MAX;
  j.cap2 = std::nextafter(f, INFINITY);
  j.nblocks = nblocks;
  j.fixed_iterations = c->params.fixed_iterations;
  j.max_iterations = c->params.fixed_iterations > 0 ? c->params.fixed_iterations : c->params.max_iterations;
  j.optimizer = c->params.optimizer;
  j.lm_max_iterations = c->params.lm_max_iterations;
  j.lm_init_lambda_factor = c->params.lm_init_lambda_factor;
  j.transformation_epsilon = c->params.transformation_epsilon;
  j.rotation_epsilon = c->params.rotation_epsilon;
  j.own_axis = c->own_axis;
  j.own_lo = c->own_lo;
  j.own_hi = c->own_hi;
  j.own_mod = c->own_mod;
  j.own_rem = c->own_rem;
  j.split_extent = kn.split_extent;
  j.premom = c->comm ? 1 : 0;
  j.mom = c->mom.as<double>();
  {
    const SearchLayout sl(c->src.cloud->n);
    char* u = c->search.as<char>();
    j.qstate = reinterpret_cast<float4*>(u + sl.qstate);
    j.key = reinterpret_cast<unsigned long long*>(u + sl.key);
    j.task_ctr = reinterpret_cast<unsigned*>(u + sl.ctr);
    j.tasks = reinterpret_cast<unsigned long long*>(u + sl.tasks);
    j.task_cap_r = sl.cap_r;
    j.hard_list = reinterpret_cast<int*>(u + sl.hard_list);
    j.hard_flag = reinterpret_cast<unsigned char*>(u + sl.hard_flag);
    j.grp_blocks = reinterpret_cast<unsigned short*>(u + sl.grp_blocks);
    j.ref = reinterpret_cast<float4*>(u + sl.ref);
    j.ref_p = reinterpret_cast<float4*>(u + sl.ref_p);
    j.sec = reinterpret_cast<unsigned*>(u + sl.sec);
    j.key2 = reinterpret_cast<unsigned long long*>(u + sl.key2);
  }
  j.xcd_scan = kn.xcd_scan;
  j.pf_ratio = kn.pf_ratio;
  j.hard_extent = kn.hard_extent;
  j.hard_blocks = kn.hard_blocks;
  j.prev_window = kn.prev_window;
  j.tri_mv = kn.tri_mv;
  j.probe2 = kn.probe * kn.probe;
  j.probe_d = kn.probe_d;
  j.reuse = kn.reuse;
  j.reuse_gap = kn.reuse_gap;
  j.reuse_gap0 = kn.reuse_gap0;
  j.cap2_d = (double)j.cap2;
  j.tri_mv_d = (double)j.tri_mv;
  j.reuse_gap_d = (double)j.reuse_gap;
  j.reuse_gap0_d = (double)j.reuse_gap0;
  j.reuse_rec0 = kn.reuse_rec0;
  j.reuse_rec_eps = kn.reuse_rec_eps;
  j.reuse_rec_conv = kn.reuse_rec_conv;
  // exact correspondence ties in nanoflann's order (k_moments): the task
  // search tracks the examined points' second distance; the target's tree,
  // when it exists, re-runs the tied queries.  Slab shards hold a subset of
  // the target, whose tree orders ties differently: Morton order there.
  j.tie_detect = (c->tie_exact && (c->own_axis < 0 || c->tie_tree)) ? 1 : 0;
  j.tgt_nf = NfTreeDev{nullptr, nullptr, nullptr, 0};
  j.tgt_nf_status = nullptr;
  j.tie_scan = j.tie_detect ? kn.tie_scan : 0;
  j.tie_ab = kn.tie_ab;
  if (j.tie_detect) {
    const NfTreeData* tt = c->tie_tree ? c->tie_tree.get() : c->tgt.cloud->nf.get();
    if (tt) {
      j.tgt_nf = tt->dev();
      j.tgt_nf_status = tt->status.as<int>();
    }
  }
  // the target's candidate cells answer the search first (k_cell_lookup)
  j.grid_on = grid_active(c) ? 1 : 0;
  if (j.grid_on) {
    j.task_cap_r = 0;   // the walk's few sub-groups scan their leaves inline (no k_nn_scan launch)
    j.grid = c->tgt.cloud->grid->dev;
    const FbLayout fl(c->src.cloud->n);
    char* u = c->fb.as<char>();
    j.fb_count = reinterpret_cast<unsigned*>(u + fl.ctr);
    j.fb_list = reinterpret_cast<int*>(u + fl.list);
    j.fb_seg_cap = fl.seg_cap;
    j.fb_mask = reinterpret_cast<unsigned short*>(u + fl.mask);
  }
  // no copy here: k_align_init reads the pinned job and writes the device one
  return GICP_OK;
}

int linearize_blocks(int nsrc) { return linearize_geometry(nsrc, 0).mom_blocks; }   // slab rows
LinGeom geometry(const gicp_ctx* c) {
  LinGeom g = linearize_geometry(c->src.cloud->n, c->tgt.cloud->upper_count());
  g.state = c->state_dev.as<AlignState>();
  g.grid = grid_active(c);
  g.grid_walk = !g.grid || c->tgt.cloud->grid->dev.has_fallback != 0;
  // the LM step in the moment kernel's last block: a sharded align all-reduces
  // between the two, so never there; on by default for the one-kernel lookup
  // linearize (DDLO_FUSE_LM: development A/B for every path)
  g.fuse_lm = !c->comm && lm_fusion_enabled(g.grid && !g.grid_walk);
  return g;
}

gicp_status prepare_align(gicp_ctx* c) {
  if (!c->src.cloud) return fail(GICP_ENOSOURCE, "no source cloud");
  if (!c->tgt.cloud) return fail(GICP_ENOTARGET, "no target cloud");
  // NanoGICP::computeTransformation (:186-193): compute missing covariances
  if (!c->src.has_cov()) {
    gicp_status s = compute_cov(c, c->src);
    if (s) return s;
  }
  if (!c->tgt.has_cov()) {
    gicp_status s = compute_cov(c, c->tgt);
    if (s) return s;
  }
  const int ns = c->src.cloud->n;
  // a growing buffer goes back to the pool: the queued no-op chunk of the
  // previous align must not still reference it
  const size_t need_corr = sizeof(int) * ns, need_sqd = sizeof(float) * ns,
               need_slab = sizeof(double) * kSlabStride * linearize_blocks(ns),
               need_search = SearchLayout(ns).total, need_fb = grid_active(c) ? FbLayout(ns).total : 0;
  if (need_corr > c->corr.bytes || need_sqd > c->sqd.bytes || need_slab > c->slab.bytes ||
      need_search > c->search.bytes || need_fb > c->fb.bytes ||
      (c->stats_on && sizeof(unsigned int) * kStatFields * (ns + 15) > c->stats.bytes)) {
    gicp_status s = drain_tail(c);
    if (s) return s;
  }
  HIP_TRY(c->corr.ensure(sizeof(int) * ns));
  HIP_TRY(c->sqd.ensure(sizeof(float) * ns));
  HIP_TRY(c->slab.ensure(sizeof(double) * kSlabStride * linearize_blocks(ns)));
  HIP_TRY(c->mom.ensure(sizeof(double) * kSlabStride));
  HIP_TRY(c->search.ensure(need_search));
  if (need_fb) HIP_TRY(c->fb.ensure(need_fb));
  // the target's nanoflann tree (tie order): a sharded align builds it up
  // front (every rank the same tree, so no rank ever re-runs alone and the
  // collectives stay matched); otherwise it is built only when an align
  // meets a tie (gicp_align).  The stream waits once for a tree's build.
  if (c->tie_exact && (c->own_axis < 0 || c->tie_tree)) {
    CloudData& tc = *c->tgt.cloud;
    if (c->comm && !c->tie_tree && !tc.nf) {
      gicp_status s = ensure_nftree(c, tc, c->stream);
      if (s) return s;
    }
    const auto& nf = c->tie_tree ? c->tie_tree : tc.nf;
    if (nf && c->nf_joined.lock() != nf) {
      HIP_TRY(nftree_join(*nf, c->stream));
      c->nf_joined = nf;
    }
  }
  if (c->stats_on) {
    HIP_TRY(c->stats.ensure(sizeof(unsigned int) * kStatFields * (ns + 15)));
    HIP_TRY(hipMemsetAsync(c->stats.p, 0, c->stats.bytes, c->stream));
  }
  return GICP_OK;
}

// Build the target's nanoflann tree (the tie order of the correspondences)
// and make the ctx stream wait for it.
gicp_status ensure_tie_tree(gicp_ctx* c) {
  gicp_status s = drain_tail(c);
  if (s) return s;
  s = ensure_nftree(c, *c->tgt.cloud, c->stream);
  if (s) return s;
  HIP_TRY(nftree_join(*c->tgt.cloud->nf, c->stream));
  c->nf_joined = c->tgt.cloud->nf;
  return GICP_OK;
}

constexpr int kMaxFirstChunk = 8;  // largest predicted first chunk (iterations)
// With fixed_iterations the count is known, so the whole align is one graph
// (up to this many iterations): every later chunk is a separate graph launch
// and a host round trip (cfg 2: 20 iterations were 1 + 12 chunks)
constexpr int kMaxFixedChunk = 64;

// One outer iteration: linearize (search + moments), then — on a sharded ctx —
// this rank's reduced moments all-reduced across ranks (80 doubles over
// RCCL: H, b, cost and the LM trial-cost moments in one collective), then
// the LM/GN step, replicated bit-identically on every rank.
// publish: host-mapped state slot the LM step copies the new state to (the
// last iteration of a chunk), or nullptr.
gicp_status enqueue_iteration(gicp_ctx* c, const AlignJob* jd, int nblocks, AlignState* publish) {
  (void)nblocks;   // = geometry(c).mom_blocks (fill_job)
  const LinGeom g = geometry(c);
  launch_linearize(c->stream, jd, g, publish);   // (fused LM step: the moment kernel's last block publishes)
  if (c->comm) {
    launch_mom_reduce(c->stream, jd);
    NCCL_TRY(rccl().all_reduce(c->mom.p, c->mom.p, kSlabStride, ncclFloat64, ncclSum, c->comm, c->stream));
  }
  if (!g.fuse_lm)
    launch_lm_step(c->stream, jd, c->state_dev.as<AlignState>(), c->slab.as<double>(), g.mom_blocks,
                   c->comm ? c->mom.as<double>() : nullptr, publish);
  return GICP_OK;
}

gicp_status enqueue_chunk(gicp_ctx* c, bool with_init, int iters, int nblocks, int slot) {
  AlignJob* jd = c->job_dev.as<AlignJob>();
  if (with_init) launch_align_init(c->stream, jd, c->job_host_dev);
  // the chunk's last LM step publishes the whole state to pinned host
  // memory: the host polls {iter, done} from it, and once done it already
  // holds the final pose, so no read-back round trip (and no copy kernel)
  // follows convergence (a speculative no-op chunk behind it rewrites the
  // same bytes)
  for (int i = 0; i < iters; ++i) {
    gicp_status s = enqueue_iteration(c, jd, nblocks, i == iters - 1 ? c->state_host_dev + slot : nullptr);
    if (s) return s;
  }
  return GICP_OK;
}

gicp_status capture_chunk(gicp_ctx* c, bool with_init, int iters, int nblocks, int slot, hipExecGraphPair* out) {
  ++c->captures;
  HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
  const gicp_status s = enqueue_chunk(c, with_init, iters, nblocks, slot);
  const hipError_t e = hipStreamEndCapture(c->stream, &out->g);  // always leave capture mode
  if (s) return s;
  HIP_TRY(e);
  HIP_TRY(hipGraphInstantiate(&out->ge, out->g, nullptr, nullptr, 0));
  return GICP_OK;
}

void drop_pair(hipExecGraphPair& p) {
  if (p.ge) (void)hipGraphExecDestroy(p.ge);
  if (p.g) (void)hipGraphDestroy(p.g);
  p.ge = nullptr;
  p.g = nullptr;
}

void drop_set(GraphSet& gs) {
  for (auto& p : gs.first) drop_pair(p);
  gs.first.clear();
  drop_pair(gs.rest[0]);
  drop_pair(gs.rest[1]);
  gs.key.fill(-1);
}

void drop_graphs(gicp_ctx* c) {
  for (auto& gs : c->gsets) drop_set(gs);
  c->gsets.clear();
}

// The graph set of a launch geometry: a cached one, else captured (its two
// single-iteration graphs now, first chunks on demand), evicting the least
// recently used set -- after the stream's queued chunk, which may be one of
// its graphs, has run.
gicp_status graph_set(gicp_ctx* c, const std::array<long long, 8>& key, int nblocks, GraphSet** out);

// Launch the align as a first chunk of n outer iterations (n = the previous
// align's iteration count on this ctx: aligns of consecutive scans converge
// in similar counts) followed by single-iteration chunks, keeping one
// speculative single-iteration chunk queued ahead while the host checks the
// previous chunk's done flag (from the first chunk on only when the previous
// align needed more than its first chunk).  After convergence at most that
// one no-op iteration (three early-exiting kernels) runs.  Returns the index
// of the chunk after which the state is final.
gicp_status run_align_graph(gicp_ctx* c, int max_it, int nblocks, int* final_chunk) {
  const void* jd = c->job_dev.p;
  // key: whether RCCL is in the chunk, the job buffer and the launch geometry
  const LinGeom g = geometry(c);
  (void)nblocks;   // = g.mom_blocks
  // (the slab buffer: k_lm_step takes it as an argument; pool blocks are 256-B aligned, bit 0 = RCCL)
  const std::array<long long, 8> key{{(long long)(uintptr_t)c->slab.p | (c->comm ? 1 : 0), (long long)(uintptr_t)jd,
                                      g.seed_blocks, g.collect_blocks,
                                      g.scan_blocks, g.mom_blocks, g.lds_boxes,
                                      g.grid ? (g.grid_walk ? 2L : 1L) * g.lookup_blocks : 0}};
  const bool use_graph = !c->comm || c->comm_graphs;
  const int first = c->params.fixed_iterations > 0
                        ? std::max(1, std::min(max_it, kMaxFixedChunk))
                        : std::max(1, std::min({c->predicted_iters, max_it, kMaxFirstChunk}));
  GraphSet* gs = nullptr;
  if (use_graph) {
    gicp_status s = graph_set(c, key, nblocks, &gs);
    if (s) {
      drop_graphs(c);
      (void)hipGetLastError();
      if (!c->comm) return s;
      c->comm_graphs = false;  // RCCL refused stream capture: launch chunks eagerly
      return run_align_graph(c, max_it, nblocks, final_chunk);
    }
  }
  if (use_graph && !gs->first[first - 1].ge) {
    gicp_status s = capture_chunk(c, true, first, nblocks, 0, &gs->first[first - 1]);
    if (s) {
      drop_graphs(c);
      return s;
    }
  }
  // chunk k publishes to slot k % 2 (chunk 0: the first-chunk graph, slot 0)
  auto launch_chunk = [&](int k) -> gicp_status {
    const bool is_first = k == 0;
    if (use_graph) {
      HIP_TRY(hipGraphLaunch(is_first ? gs->first[first - 1].ge : gs->rest[k & 1].ge, c->stream));
      return GICP_OK;
    }
    return enqueue_chunk(c, is_first, is_first ? first : 1, nblocks, k & 1);
  };
  const int nchunks = 1 + (max_it - first);
  while ((int)c->chunk_ev.size() < nchunks) {
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));  // timed: the last one ends the align's device time
    c->chunk_ev.push_back(e);
  }
  gicp_status s = launch_chunk(0);
  if (s) return s;
  HIP_TRY(hipEventRecord(c->chunk_ev[0], c->stream));
  int launched = 1;
  if (nchunks > 1 && c->speculate) {
    s = launch_chunk(1);
    if (s) return s;
    HIP_TRY(hipEventRecord(c->chunk_ev[1], c->stream));
    launched = 2;
  }
  // The number of chunks launched depends only on the done flags, which the
  // replicated LM step makes identical on every rank of a sharded align, so
  // every rank issues the same sequence of collectives.  When chunk k is
  // read, at most chunk k + 1 (the other slot) is queued behind it; chunk
  // k + 2 (same slot as k) is launched only after the read.
  int k = 0;
  // the host polls the chunk's event (hipEventQuery) instead of blocking in
  // hipEventSynchronize: 2 us less per align at cfg 3 (DDLO_SPIN_WAIT=0: block)
  static const bool spin = [] {
    const char* v = dev_getenv("DDLO_SPIN_WAIT");
    return !(v && *v == '0');
  }();
  const unsigned long long ticket = c->job_host->ticket;
  for (;;) {
    if (spin) {
      // chunk k's last LM step writes its publication word (ticket, done,
      // iter) after the state (AlignState::pub): the host polls that word in
      // pinned memory, which lands as the kernel stores it, instead of the
      // chunk's event, which completes only after the command processor has
      // retired the kernel.  The event is still queried every 64 polls (an
      // error, or a word that never comes, ends the wait).
      static std::atomic<int> waiters{0};
      waiters.fetch_add(1, std::memory_order_relaxed);
      const volatile unsigned long long* pw = &(c->state_host + (k & 1))->pub;
      const int expect = first + k;   // iterations after chunk k unless done earlier
      hipError_t q = hipErrorNotReady;
      for (unsigned n = 1;; ++n) {
        const unsigned long long w = *pw;
        if ((w >> 17) == ticket && (((w >> 16) & 1ull) || (int)(w & 0xffffu) >= expect)) {
          q = hipSuccess;
          break;
        }
        if ((n & 63) == 0) {
          q = hipEventQuery(c->chunk_ev[k]);
          if (q != hipErrorNotReady) {
            const unsigned long long w2 = *pw;   // the event completed: the word has landed
            if (q == hipSuccess && !((w2 >> 17) == ticket && (((w2 >> 16) & 1ull) || (int)(w2 & 0xffffu) >= expect)))
              q = hipErrorUnknown;
            break;
          }
        }
        if (waiters.load(std::memory_order_relaxed) > 1) std::this_thread::yield();
      }
      waiters.fetch_sub(1, std::memory_order_relaxed);
      if (q == hipErrorUnknown) return fail(GICP_EHIP, "align chunk completed without its state publication");
      HIP_TRY(q);
    } else {
      HIP_TRY(hipEventSynchronize(c->chunk_ev[k]));
    }
    const volatile AlignState* st = c->state_host + (k & 1);
    if (st->done || k == nchunks - 1) break;
    while (launched < nchunks && launched <= k + 2) {  // keep one chunk queued ahead of k+1
      s = launch_chunk(launched);
      if (s) return s;
      HIP_TRY(hipEventRecord(c->chunk_ev[launched], c->stream));
      ++launched;
    }
    ++k;
  }
  *final_chunk = k;
  c->state_slot = k & 1;
  c->tail_ev = c->chunk_ev[launched - 1];
  // (a published chunk may still be retiring its last kernel: the tail covers it too)
  c->tail_pending = launched - 1 > k || spin;
  // Speculate next time only if this align outran its predicted first chunk:
  // when the prediction held, the queued no-op chunk only delays the next
  // align (A/B at cfg 3: 0.466 -> 0.459 ms/scan without it).
  c->speculate = k > 0;
  c->predicted_iters = std::max(1, (int)((const volatile AlignState*)(c->state_host + (k & 1)))->iter);
  return GICP_OK;
}

gicp_status graph_set(gicp_ctx* c, const std::array<long long, 8>& key, int nblocks, GraphSet** out) {
  ++c->graph_clock;
  for (auto& gs : c->gsets)
    if (gs.key == key) {
      gs.last_use = c->graph_clock;
      *out = &gs;
      return GICP_OK;
    }
  GraphSet* slot = nullptr;
  if ((int)c->gsets.size() < kGraphSets) {
    c->gsets.reserve(kGraphSets);   // no reallocation: the sets stay where their pointers point
    c->gsets.emplace_back();
    slot = &c->gsets.back();
  } else {
    slot = &c->gsets[0];
    for (auto& gs : c->gsets)
      if (gs.last_use < slot->last_use) slot = &gs;
    gicp_status s = drain_tail(c);   // the queued speculative chunk may be one of its graphs
    if (s) return s;
    drop_set(*slot);
  }
  slot->first.resize(kMaxFixedChunk);
  gicp_status s = capture_chunk(c, false, 1, nblocks, 0, &slot->rest[0]);
  if (!s) s = capture_chunk(c, false, 1, nblocks, 1, &slot->rest[1]);
  if (s) return s;
  slot->key = key;
  slot->last_use = c->graph_clock;
  *out = slot;
  return GICP_OK;
}

gicp_status run_align_eager_profiled(gicp_ctx* c, int max_it, int nblocks) {
  AlignJob* jd = c->job_dev.as<AlignJob>();
  const size_t need = 2 * (size_t)max_it;
  while (c->prof_ev.size() < need) {
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));
    c->prof_ev.push_back(e);
  }
  launch_align_init(c->stream, jd, c->job_host_dev);
  for (int i = 0; i < max_it; ++i) {
    HIP_TRY(hipEventRecord(c->prof_ev[2 * i], c->stream));
    LinGeom g = geometry(c);
    g.fuse_lm = false;   // profiled aligns time the linearize on its own
    launch_linearize(c->stream, jd, g);
    HIP_TRY(hipEventRecord(c->prof_ev[2 * i + 1], c->stream));
    if (c->comm) {
      launch_mom_reduce(c->stream, jd);
      NCCL_TRY(rccl().all_reduce(c->mom.p, c->mom.p, kSlabStride, ncclFloat64, ncclSum, c->comm, c->stream));
    }
    launch_lm_step(c->stream, jd, c->state_dev.as<AlignState>(), c->slab.as<double>(), g.mom_blocks,
                   c->comm ? c->mom.as<double>() : nullptr, nullptr);
  }
  HIP_TRY(hipGetLastError());
  return GICP_OK;
}

}  // namespace

namespace ddlo {
bool lm_fusion_enabled(bool lookup) {
  static const int on = [] {   // -1: the default (fused on the lookup path only)
    const char* v = dev_getenv("DDLO_FUSE_LM");
    return v && *v ? std::atoi(v) : -1;
  }();
  return on < 0 ? lookup : on != 0;
}
}  // namespace ddlo

extern "C" {

int32_t gicp_abi_version(void) { return DDLO_GICP_ABI_VERSION; }
const char* gicp_last_error(void) { return g_last_error.c_str(); }

gicp_status gicp_default_params(gicp_params* p) {
  if (!p) return fail(GICP_EINVAL, "null params");
  p->k_correspondences = 20;
  p->max_iterations = 64;
  p->max_correspondence_distance = FLT_MAX;
  p->transformation_epsilon = 5e-4;
  p->rotation_epsilon = 2e-3;
  p->lm_init_lambda_factor = 1e-9;
  p->regularization = GICP_REG_PLANE;
  p->optimizer = GICP_OPT_LEVENBERG_MARQUARDT;
  p->lm_max_iterations = 10;
  p->fixed_iterations = 0;
  return GICP_OK;
}

gicp_status gicp_ctx_create(int device, gicp_ctx** out) {
  if (!out) return fail(GICP_EINVAL, "null out");
  *out = nullptr;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(GICP_EINVAL, "invalid device ordinal");
  HIP_TRY(hipSetDevice(device));
  auto c = std::make_unique<gicp_ctx>();
  c->device = device;
  gicp_default_params(&c->params);
  HIP_TRY(stream_pool().acquire(&c->stream));
  HIP_TRY(stream_pool().acquire(&c->aux_stream));
  HIP_TRY(hipEventCreateWithFlags(&c->aux_ev, hipEventDisableTiming));
  HIP_TRY(pinned_pool().alloc((void**)&c->job_host, sizeof(AlignJob), hipHostMallocMapped));
  HIP_TRY(pinned_pool().alloc((void**)&c->state_host, 2 * sizeof(AlignState), hipHostMallocMapped));
  HIP_TRY(hipHostGetDevicePointer((void**)&c->job_host_dev, c->job_host, 0));
  HIP_TRY(hipHostGetDevicePointer((void**)&c->state_host_dev, c->state_host, 0));
  HIP_TRY(pinned_pool().alloc((void**)&c->flag_host, sizeof(int) * 4, hipHostMallocDefault));
  HIP_TRY(c->job_dev.ensure(sizeof(AlignJob)));
  HIP_TRY(c->state_dev.ensure(sizeof(AlignState)));
  std::memset(c->state_host, 0, 2 * sizeof(AlignState));
  for (int i = 0; i < 6; ++i) c->state_host->final_hessian[7 * i] = 1.0;  // final_hessian_.setIdentity()
  // stream-ordered (never the legacy stream: another ctx's thread may be
  // capturing its align graph at this moment)
  HIP_TRY(hipMemcpyAsync(c->state_dev.p, c->state_host, sizeof(AlignState), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipEventCreate(&c->ev0));
  HIP_TRY(hipEventCreate(&c->ev1));
  // options (gicp_set_default_option: the process-wide values new contexts take)
  c->tie_exact = g_opt_default[GICP_OPT_TIE_ORDER].load() != 0;
  c->tie_lazy = g_opt_default[GICP_OPT_TIE_LAZY].load() != 0;
  c->partial_levels = g_opt_default[GICP_OPT_TIE_PARTIAL_LEVELS].load();
  c->cov_tasks = g_opt_default[GICP_OPT_COV_TASKS].load() != 0;
  c->grid_max_mb = g_opt_default[GICP_OPT_GRID_MAX_MB].load();
  {
    // DDLO_NF_OWN_STREAM=1 (development): every ctx builds its trees on its
    // own stream, the partial tree gated on the tie count (the S2S batch's
    // workers always do)
    const char* os = dev_getenv("DDLO_NF_OWN_STREAM");
    c->nf_same_stream = os && *os == '1';
  }
  *out = c.release();
  return GICP_OK;
}

gicp_status gicp_ctx_destroy(gicp_ctx* c) {
  if (!c) return GICP_OK;
  if (dev_getenv("DDLO_GRAPH_DEBUG")) std::fprintf(stderr, "[graphs] ctx %p: %ld chunk captures\n", (void*)c, c->captures);
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  (void)hipStreamSynchronize(c->aux_stream);
  drop_graphs(c);
  if (c->comm) (void)rccl().comm_destroy(c->comm);
  for (auto e : c->prof_ev) (void)hipEventDestroy(e);
  for (auto e : c->st_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto e : c->chunk_ev) (void)hipEventDestroy(e);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  pinned_pool().release(c->job_host, sizeof(AlignJob), hipHostMallocMapped);
  pinned_pool().release(c->state_host, 2 * sizeof(AlignState), hipHostMallocMapped);
  pinned_pool().release(c->flag_host, sizeof(int) * 4, hipHostMallocDefault);
  pinned_pool().release(c->nf_err_host, 2 * sizeof(int), hipHostMallocDefault);
  if (c->tie_cnt_ev) (void)hipEventDestroy(c->tie_cnt_ev);
  c->src = Side();
  c->tgt = Side();
  (void)hipStreamSynchronize(c->aux_stream);
  for (auto& e : c->nf_graphs)
    if (e.ge) (void)hipGraphExecDestroy(e.ge);
  pinned_pool().release(c->nf_ntask_host, sizeof(int) * (kNfMaxLevels + 1), hipHostMallocDefault);
  if (c->nf_ntask_ev) (void)hipEventDestroy(c->nf_ntask_ev);
  stream_pool().release(c->device, c->aux_stream);   // (both synchronized above)
  stream_pool().release(c->device, c->stream);
  (void)hipEventDestroy(c->aux_ev);
  delete c;
  return GICP_OK;
}

gicp_status gicp_set_params(gicp_ctx* c, const gicp_params* p) {
  if (!c || !p) return fail(GICP_EINVAL, "null argument");
  if (p->regularization < 0 || p->regularization > 4) return fail(GICP_EINVAL, "invalid regularization method");
  if (p->optimizer < 0 || p->optimizer > 1) return fail(GICP_EINVAL, "invalid optimizer");
  if (p->k_correspondences < 1 || p->k_correspondences > 64) return fail(GICP_EINVAL, "k_correspondences must be in [1, 64]");
  if (p->lm_max_iterations < 1 || p->max_iterations < 0 || p->fixed_iterations < 0)
    return fail(GICP_EINVAL, "invalid iteration limits");
  if (!(p->max_correspondence_distance > 0) || !(p->transformation_epsilon > 0) || !(p->rotation_epsilon > 0))
    return fail(GICP_EINVAL, "distances/epsilons must be positive");
  c->params = *p;
  // per-ctx launch history restarts with the parameters: every rank of a
  // sharded align then derives the same chunk sequence (same collectives)
  c->speculate = true;
  c->predicted_iters = kDefaultPredictedIters;
  return GICP_OK;
}

gicp_status gicp_get_params(const gicp_ctx* c, gicp_params* out) {
  if (!c || !out) return fail(GICP_EINVAL, "null argument");
  *out = c->params;
  return GICP_OK;
}

namespace {
// nf_early: the caller computes the source covariances next (gicp_s2s_batch),
// so nanoflann's tree starts with the index build
gicp_status set_source_impl(gicp_ctx* c, const float* xyz, size_t n, size_t stride, int build_index, bool nf_early) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  gicp_status s = set_device(c);
  if (s) return s;
  std::shared_ptr<CloudData> cd;
  s = build_cloud(c, xyz, n, stride, &cd, false, true, nf_early);   // the device cloud is always sorted + indexed (cheap)
  if (s) return s;
  const Side old = c->src;
  c->src.cloud = cd;
  c->src.cov.reset();  // setInputSource clears source covariances (:142)
  if (!build_index && old.has_cov() && old.cloud->n == (int)n) {
    // registerInputSource (:122-130) keeps source_covs_: covariance i stays
    // with point i of the new cloud (a size mismatch is recomputed at align,
    // :186-189, so it is dropped here)
    auto cv = std::make_shared<CovData>();
    cv->n = (int)n;
    HIP_TRY(cv->cov6.ensure(sizeof(double) * 6 * n));
    launch_cov_remap(c->stream, old.cov->cov6.as<double>(), old.cloud->inv_perm.as<int>(), cd->perm.as<int>(), (int)n,
                     cv->cov6.as<double>());
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->src.cov = cv;
  }
  invalidate_align(c);
  return GICP_OK;
}
}  // namespace

gicp_status gicp_set_source(gicp_ctx* c, const float* xyz, size_t n, size_t stride, int build_index) {
  return set_source_impl(c, xyz, n, stride, build_index, false);
}

gicp_status gicp_set_target(gicp_ctx* c, const float* xyz, size_t n, size_t stride) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  gicp_status s = set_device(c);
  if (s) return s;
  std::shared_ptr<CloudData> cd;
  s = build_cloud(c, xyz, n, stride, &cd);
  if (s) return s;
  c->tgt.cloud = cd;
  c->tgt.cov.reset();  // (:154)
  c->tie_tree.reset();  // a slab's tie order belongs to the previous target
  invalidate_align(c);
  return GICP_OK;
}

gicp_status gicp_clear_source(gicp_ctx* c) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  c->src = Side();
  invalidate_align(c);
  return GICP_OK;
}
gicp_status gicp_clear_target(gicp_ctx* c) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  c->tgt = Side();
  c->tie_tree.reset();   // a slab's tie order belongs to the cleared target
  invalidate_align(c);
  return GICP_OK;
}

gicp_status gicp_get_size(const gicp_ctx* c, int side, size_t* n) {
  if (!c || !n) return fail(GICP_EINVAL, "null argument");
  const Side& sd = side == GICP_SIDE_SOURCE ? c->src : c->tgt;
  *n = sd.cloud ? (size_t)sd.cloud->n : 0;
  return GICP_OK;
}

gicp_status gicp_compute_covariances(gicp_ctx* c, int side) {
  if (!c || (side != 0 && side != 1)) return fail(GICP_EINVAL, "invalid argument");
  begin_ties(c);
  gicp_status s = set_device(c);
  if (s) return s;
  s = compute_cov(c, side == GICP_SIDE_SOURCE ? c->src : c->tgt);
  if (s) return s;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return check_ties(c);
}

gicp_status gicp_set_covariances(gicp_ctx* c, int side, const double* cov, size_t n, int layout) {
  if (!c || !cov || (side != 0 && side != 1) || (layout != 0 && layout != 1)) return fail(GICP_EINVAL, "invalid argument");
  Side& sd = side == GICP_SIDE_SOURCE ? c->src : c->tgt;
  if (!sd.cloud) return fail(GICP_ESTATE, "set the cloud before its covariances");
  if ((int)n != sd.cloud->n) return fail(GICP_EINVAL, "covariance count != cloud size");
  gicp_status s = set_device(c);
  if (s) return s;
  const size_t w = layout == GICP_COV_MAT4D ? 16 : 6;
  HIP_TRY(c->tmp_out.ensure(sizeof(double) * w * n));
  HIP_TRY(hipMemcpyAsync(c->tmp_out.p, cov, sizeof(double) * w * n, hipMemcpyHostToDevice, c->stream));
  auto cv = std::make_shared<CovData>();  // copy semantics (:161,168): never mutate a shared CovData
  cv->n = (int)n;
  HIP_TRY(cv->cov6.ensure(sizeof(double) * 6 * n));
  launch_cov_import(c->stream, c->tmp_out.as<double>(), layout, (int)n, sd.cloud->inv_perm.as<int>(), cv->cov6.as<double>());
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  sd.cov = cv;
  return GICP_OK;
}

gicp_status gicp_get_covariances(const gicp_ctx* cc, int side, double* cov, size_t n, int layout) {
  gicp_ctx* c = const_cast<gicp_ctx*>(cc);
  if (!c || !cov || (side != 0 && side != 1) || (layout != 0 && layout != 1)) return fail(GICP_EINVAL, "invalid argument");
  Side& sd = side == GICP_SIDE_SOURCE ? c->src : c->tgt;
  if (!sd.has_cov()) return fail(GICP_ESTATE, "no covariances on this side");
  if ((int)n != sd.cloud->n) return fail(GICP_EINVAL, "n != cloud size");
  gicp_status s = set_device(c);
  if (s) return s;
  const size_t w = layout == GICP_COV_MAT4D ? 16 : 6;
  HIP_TRY(c->tmp_out.ensure(sizeof(double) * w * n));
  launch_cov_export(c->stream, sd.cov->cov6.as<double>(), layout, (int)n, sd.cloud->perm.as<int>(), c->tmp_out.as<double>());
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(cov, c->tmp_out.p, sizeof(double) * w * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GICP_OK;
}

gicp_status gicp_has_covariances(const gicp_ctx* c, int side, int* has) {
  if (!c || !has || (side != 0 && side != 1)) return fail(GICP_EINVAL, "invalid argument");
  *has = (side == GICP_SIDE_SOURCE ? c->src : c->tgt).has_cov() ? 1 : 0;
  return GICP_OK;
}

gicp_status gicp_swap_source_target(gicp_ctx* c) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  std::swap(c->src, c->tgt);  // clouds, indices and covariances (:100-102)
  c->tie_tree.reset();        // a slab's tie order belonged to the old target
  invalidate_align(c);        // correspondences_.clear() (:104-105)
  return GICP_OK;
}

gicp_status gicp_share_source(gicp_ctx* dst, const gicp_ctx* src) {
  if (!dst || !src) return fail(GICP_EINVAL, "null ctx");
  if (dst->device != src->device) return fail(GICP_EINVAL, "contexts live on different devices");
  dst->src = src->src;
  invalidate_align(dst);
  return GICP_OK;
}

gicp_status gicp_align(gicp_ctx* c, const float* guess16, float* out16, gicp_result* res) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  begin_ties(c);
  gicp_status s = set_device(c);
  if (s) return s;
  s = maybe_build_grid(c);
  if (s) return s;
  s = prepare_align(c);
  if (s) return s;
  const int ns = c->src.cloud->n;
  const int nblocks = linearize_blocks(ns);
  hipEvent_t end_ev = c->ev1;
  int reruns = 0;
  for (;;) {
    s = fill_job(c, guess16, nblocks);
    if (s) return s;
    finalize_job(c);
    JobCommit commit(c);
    const int max_it = c->job_host->max_iterations;
    end_ev = c->ev1;
    HIP_TRY(hipEventRecord(c->ev0, c->stream));
    if (c->profiling || max_it <= 0) {
      s = max_it > 0 ? run_align_eager_profiled(c, max_it, nblocks) : GICP_OK;
      if (s) return s;
      if (max_it <= 0) launch_align_init(c->stream, c->job_dev.as<AlignJob>(), c->job_host_dev);
      HIP_TRY(hipGetLastError());
      commit.done();
      HIP_TRY(hipEventRecord(c->ev1, c->stream));
      HIP_TRY(hipMemcpyAsync(c->state_host, c->state_dev.p, sizeof(AlignState), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      c->state_slot = 0;
      c->tail_pending = false;
    } else {
      int fc = 0;
      s = run_align_graph(c, max_it, nblocks, &fc);
      if (s) return s;
      commit.done();
      // chunk fc's end-of-chunk copy already put the final state in its
      // slot; the (at most one) speculative no-op chunk still queued writes
      // the other slot and does not delay the return
      end_ev = c->chunk_ev[fc];
    }
    // a correspondence met an exact tie before the target had nanoflann's
    // tree: build it and run the align again, so every correspondence is
    // nanoflann's (the tree stays with the target cloud for later aligns)
    if (!final_state(c).tie_pending || reruns > 0) break;
    s = ensure_tie_tree(c);
    if (s) return s;
    ++reruns;
  }
  const AlignState& st = final_state(c);
  c->have_align = st.iter > 0;
  c->last_nsrc = ns;
  if (out16) {
    for (int r = 0; r < 3; ++r) {
      for (int cc = 0; cc < 3; ++cc) out16[4 * r + cc] = (float)st.R[3 * r + cc];
      out16[4 * r + 3] = (float)st.t[r];
    }
    out16[12] = out16[13] = out16[14] = 0.f;
    out16[15] = 1.f;
  }
  if (res) {
    std::memset(res, 0, sizeof(*res));
    res->converged = st.converged;
    res->nr_iterations = st.nr_iterations;
    res->iterations_run = st.iter;
    res->lm_failed = st.lm_failed;
    res->lm_trials = st.lm_trials;
    res->num_correspondences = st.num_corr;
    res->final_cost = st.final_cost;
    std::memcpy(res->final_hessian, st.final_hessian, sizeof(res->final_hessian));
    res->lm_lambda = st.lambda;
    res->ties_resolved = st.ties_resolved;
    res->tie_reruns = reruns;
    if (c->profiling) {
      // (profiled aligns only: a graph align returns as soon as its state is
      // published, before its end event has completed)
      float ms = 0.f;
      HIP_TRY(hipEventSynchronize(end_ev));
      HIP_TRY(hipEventElapsedTime(&ms, c->ev0, end_ev));
      res->device_ms = ms;
      double tot = 0.0;
      for (int i = 0; i < st.iter; ++i) {
        float m = 0.f;
        HIP_TRY(hipEventElapsedTime(&m, c->prof_ev[2 * i], c->prof_ev[2 * i + 1]));
        tot += m;
      }
      res->linearize_ms = tot;
    }
  }
  s = check_ties(c);
  if (s) return s;
  if (st.tie_err || st.tie_pending)
    return fail(GICP_EHIP, "nanoflann tie order: a tied correspondence could not be re-run (bits " +
                               std::to_string(st.tie_err) + (st.tie_pending ? ", no tree" : "") + ")");
  if (st.lm_failed) g_last_error = "lm not converged!!";
  return GICP_OK;
}

gicp_status gicp_get_residuals(gicp_ctx* c, double* out, size_t n) {
  if (!c || !out) return fail(GICP_EINVAL, "null argument");
  if (!c->have_align || !c->src.cloud || !c->tgt.cloud) return fail(GICP_ESTATE, "no linearization to report residuals of");
  if ((int)n != c->src.cloud->n) return fail(GICP_EINVAL, "n != source size");
  gicp_status s = set_device(c);
  if (s) return s;
  HIP_TRY(c->tmp_out.ensure(sizeof(double) * n));
  launch_residuals(c->stream, c->job_dev.as<AlignJob>(), (int)n, c->tmp_out.as<double>());
  HIP_TRY(hipGetLastError());
  // sharded: every rank holds the exact nearest distance within its tile +
  // halo for every source point (owned matches, unbounded search otherwise);
  // the tiles cover the whole target, so the minimum over ranks is the
  // global 1-NN distance (nano_gicp_impl.hpp:255-257,225-232)
  if (c->comm)
    NCCL_TRY(rccl().all_reduce(c->tmp_out.p, c->tmp_out.p, n, ncclFloat64, ncclMin, c->comm, c->stream));
  HIP_TRY(hipMemcpyAsync(out, c->tmp_out.p, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GICP_OK;
}

gicp_status gicp_residual_image(gicp_ctx* c, double theta_min, double theta_max, int width, int height, float* img,
                                float* xyz) {
  if (!c || !img) return fail(GICP_EINVAL, "null argument");
  if (width <= 0 || height <= 0 || (long)width * height > (1L << 28) || !(theta_max > theta_min))
    return fail(GICP_EINVAL, "invalid image geometry");
  if (!c->have_align || !c->src.cloud || !c->tgt.cloud) return fail(GICP_ESTATE, "no linearization to report residuals of");
  gicp_status s = set_device(c);
  if (s) return s;
  const int n = c->src.cloud->n;
  const size_t npix = (size_t)width * height;
  HIP_TRY(c->tmp_out.ensure(sizeof(double) * n));
  launch_residuals(c->stream, c->job_dev.as<AlignJob>(), n, c->tmp_out.as<double>());
  if (c->comm)  // sharded: global residual = min over ranks (see gicp_get_residuals)
    NCCL_TRY(rccl().all_reduce(c->tmp_out.p, c->tmp_out.p, n, ncclFloat64, ncclMin, c->comm, c->stream));
  DevBuf winner, dimg, dxyz;
  HIP_TRY(winner.ensure(sizeof(int) * npix));
  HIP_TRY(dimg.ensure(sizeof(float) * npix));
  if (xyz) HIP_TRY(dxyz.ensure(sizeof(float) * 3 * npix));
  HIP_TRY(hipMemsetAsync(winner.p, 0xff, sizeof(int) * npix, c->stream));  // -1: no point
  const CloudData& cd = *c->src.cloud;
  launch_residual_image(c->stream, cd.pts.as<float4>(), cd.perm.as<int>(), cd.inv_perm.as<int>(), n,
                        c->tmp_out.as<double>(), theta_min, theta_max, width, height, winner.as<int>(),
                        dimg.as<float>(), xyz ? dxyz.as<float>() : nullptr);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(img, dimg.p, sizeof(float) * npix, hipMemcpyDeviceToHost, c->stream));
  if (xyz) HIP_TRY(hipMemcpyAsync(xyz, dxyz.p, sizeof(float) * 3 * npix, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GICP_OK;
}

gicp_status gicp_get_correspondences(gicp_ctx* c, int32_t* corr, float* sq_dist, size_t n) {
  if (!c || (!corr && !sq_dist)) return fail(GICP_EINVAL, "null argument");
  if (!c->have_align || !c->src.cloud) return fail(GICP_ESTATE, "no linearization");
  if ((int)n != c->src.cloud->n) return fail(GICP_EINVAL, "n != source size");
  gicp_status s = set_device(c);
  if (s) return s;
  HIP_TRY(c->tmp_out.ensure((sizeof(int) + sizeof(float)) * n + 64));
  int* dcorr = c->tmp_out.as<int>();
  float* dsqd = reinterpret_cast<float*>(c->tmp_out.as<char>() + ((sizeof(int) * n + 63) / 64) * 64);
  // sq_distances_ holds the unbounded 1-NN distance of EVERY point
  // (nano_gicp_impl.hpp:255-257); the bounded search left +inf for points
  // without a match, so complete those first (same kernel as getResiduals)
  if (sq_dist && c->tgt.cloud) launch_residuals(c->stream, c->job_dev.as<AlignJob>(), (int)n, nullptr);
  launch_export_corr(c->stream, c->job_dev.as<AlignJob>(), (int)n, dcorr, dsqd);
  HIP_TRY(hipGetLastError());
  if (corr) HIP_TRY(hipMemcpyAsync(corr, dcorr, sizeof(int) * n, hipMemcpyDeviceToHost, c->stream));
  if (sq_dist) HIP_TRY(hipMemcpyAsync(sq_dist, dsqd, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GICP_OK;
}

gicp_status gicp_transform_source(gicp_ctx* c, float* out_xyz, size_t n, size_t stride) {
  if (!c || !out_xyz || stride < 12 || stride % 4) return fail(GICP_EINVAL, "invalid argument");
  if (!c->src.cloud) return fail(GICP_ENOSOURCE, "no source");
  if ((int)n != c->src.cloud->n) return fail(GICP_EINVAL, "n != source size");
  gicp_status s = set_device(c);
  if (s) return s;
  // final_transformation_ = x0.cast<float>() of the last align
  float T[16];
  const AlignState& st = final_state(c);
  for (int r = 0; r < 3; ++r) {
    for (int cc = 0; cc < 3; ++cc) T[4 * r + cc] = (float)st.R[3 * r + cc];
    T[4 * r + 3] = (float)st.t[r];
  }
  T[12] = T[13] = T[14] = 0.f;
  T[15] = 1.f;
  const size_t bytes = (n - 1) * stride + 12;
  HIP_TRY(c->tmp_out.ensure(bytes + 256));
  float* dT = reinterpret_cast<float*>(c->tmp_out.as<char>() + ((bytes + 63) / 64) * 64);
  HIP_TRY(hipMemcpyAsync(dT, T, sizeof(T), hipMemcpyHostToDevice, c->stream));
  // keep the caller's other fields (e.g. intensity): start from their buffer
  HIP_TRY(hipMemcpyAsync(c->tmp_out.p, out_xyz, bytes, hipMemcpyHostToDevice, c->stream));
  launch_transform(c->stream, c->src.cloud->pts.as<float4>(), (int)n, c->src.cloud->perm.as<int>(), dT,
                   c->tmp_out.as<float>(), stride / 4);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out_xyz, c->tmp_out.p, bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GICP_OK;
}

gicp_status gicp_linearize(gicp_ctx* c, const double* pose16, double* H36, double* b6, double* cost, int32_t* ncorr) {
  if (!c || !pose16) return fail(GICP_EINVAL, "null argument");
  begin_ties(c);
  gicp_status s = set_device(c);
  if (s) return s;
  s = maybe_build_grid(c);
  if (s) return s;
  s = prepare_align(c);
  if (s) return s;
  const int ns = c->src.cloud->n;
  const int nblocks = linearize_blocks(ns);
  for (int rerun = 0;; ++rerun) {
    float g[16];
    for (int i = 0; i < 16; ++i) g[i] = 0.f;
    s = fill_job(c, g, nblocks);
    if (s) return s;
    // exact double pose (not the float guess path)
    for (int r = 0; r < 3; ++r) {
      for (int cc = 0; cc < 3; ++cc) c->job_host->guess_R[3 * r + cc] = pose16[4 * r + cc];
      c->job_host->guess_t[r] = pose16[4 * r + 3];
    }
    c->job_host->optimizer = GICP_OPT_GAUSS_NEWTON;
    c->job_host->max_iterations = 1;
    c->job_host->fixed_iterations = 1;
    finalize_job(c);
    JobCommit commit(c);
    AlignJob* jd = c->job_dev.as<AlignJob>();
    launch_align_init(c->stream, jd, c->job_host_dev);
    s = enqueue_iteration(c, jd, nblocks, nullptr);
    if (s) return s;
    HIP_TRY(hipGetLastError());
    commit.done();
    HIP_TRY(hipMemcpyAsync(c->state_host, c->state_dev.p, sizeof(AlignState), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->state_slot = 0;
    c->tail_pending = false;
    if (!final_state(c).tie_pending || rerun > 0) break;
    s = ensure_tie_tree(c);   // a tie met before the target had its nanoflann tree (see gicp_align)
    if (s) return s;
  }
  const AlignState& st = final_state(c);
  if (st.tie_err || st.tie_pending)
    return fail(GICP_EHIP, "nanoflann tie order: a tied correspondence could not be re-run (bits " +
                               std::to_string(st.tie_err) + ")");
  if (H36) std::memcpy(H36, st.final_hessian, sizeof(double) * 36);
  if (cost) *cost = st.final_cost;
  if (ncorr) *ncorr = st.num_corr;
  if (b6) std::memcpy(b6, st.last_b, sizeof(double) * 6);
  c->have_align = true;
  c->last_nsrc = ns;
  return GICP_OK;
}

gicp_status gicp_knn_target(gicp_ctx* c, const float* q, size_t nq, size_t stride, int k, int32_t* idx, float* sqd) {
  if (!c || !q || !idx || !sqd || nq == 0 || stride < 12 || stride % 4) return fail(GICP_EINVAL, "invalid argument");
  if (!c->tgt.cloud) return fail(GICP_ENOTARGET, "no target");
  if (k < 1 || k > 64) return fail(GICP_EINVAL, "k must be in [1, 64]");
  if (c->tgt.cloud->n < k) return fail(GICP_ETOOFEW, "target has fewer than k points");
  begin_ties(c);
  gicp_status s = set_device(c);
  if (s) return s;
  const size_t raw = (nq - 1) * stride + 12;
  HIP_TRY(c->raw_bytes.ensure(raw));
  HIP_TRY(hipMemcpyAsync(c->raw_bytes.p, q, raw, hipMemcpyHostToDevice, c->stream));
  const int nb = (int)((nq + 255) / 256);
  HIP_TRY(c->raw_pts.ensure(sizeof(float4) * nq));
  HIP_TRY(c->partial.ensure(sizeof(float) * 6 * nb));
  HIP_TRY(c->nonfinite.ensure(sizeof(int)));
  launch_pack_bbox(c->stream, c->raw_bytes.as<unsigned char>(), stride, (int)nq, c->raw_pts.as<float4>(),
                   c->partial.as<float>(), c->nonfinite.as<int>(), nb);
  HIP_TRY(c->tmp_out.ensure((sizeof(int) + sizeof(float)) * nq * k + 64));
  int* didx = c->tmp_out.as<int>();
  float* dd = reinterpret_cast<float*>(c->tmp_out.as<char>() + ((sizeof(int) * nq * k + 63) / 64) * 64);
  TieList tl{nullptr, nullptr};
  if (c->tie_exact) {   // tied answers are re-run in nanoflann's order (nftree.hip)
    s = ensure_nftree(c, *c->tgt.cloud, c->stream);
    if (!s) s = tie_scratch(c, (int)nq, c->stream, &tl);
    if (s) return s;
  }
  if (!launch_knn_query(c->stream, c->tgt.cloud->dev(), c->raw_pts.as<float4>(), (int)nq, k, didx, dd, tl))
    return fail(GICP_EINVAL, "unsupported k");
  if (c->tie_exact) {
    HIP_TRY(nftree_join(*c->tgt.cloud->nf, c->stream));
    launch_nf_resolve_knn(c->stream, c->tgt.cloud->nf->dev(), c->raw_pts.as<float4>(), tl, k, didx, dd,
                          c->tgt.cloud->nf->status.as<int>(), c->nf_err.as<int>());
    s = publish_ties(c, c->stream);
    if (s) return s;
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(idx, didx, sizeof(int) * nq * k, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(sqd, dd, sizeof(float) * nq * k, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return check_ties(c);
}

gicp_status gicp_set_tie_order(gicp_ctx* c, int nanoflann_order) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  c->tie_exact = nanoflann_order != 0;
  return GICP_OK;
}

gicp_status gicp_set_option(gicp_ctx* c, int option, int value) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  gicp_status s = check_option(option, value);
  if (s) return s;
  switch (option) {
    case GICP_OPT_TIE_ORDER: c->tie_exact = value != 0; break;
    case GICP_OPT_TIE_LAZY: c->tie_lazy = value != 0; break;
    case GICP_OPT_TIE_PARTIAL_LEVELS: c->partial_levels = value; break;
    case GICP_OPT_COV_TASKS: c->cov_tasks = value != 0; break;
    case GICP_OPT_GRID_MAX_MB: c->grid_max_mb = value; break;
  }
  return GICP_OK;
}

gicp_status gicp_get_option(const gicp_ctx* c, int option, int* value) {
  if (!c || !value) return fail(GICP_EINVAL, "null argument");
  gicp_status s = check_option(option, 0);
  if (s) return s;
  switch (option) {
    case GICP_OPT_TIE_ORDER: *value = c->tie_exact ? 1 : 0; break;
    case GICP_OPT_TIE_LAZY: *value = c->tie_lazy ? 1 : 0; break;
    case GICP_OPT_TIE_PARTIAL_LEVELS: *value = c->partial_levels; break;
    case GICP_OPT_COV_TASKS: *value = c->cov_tasks ? 1 : 0; break;
    case GICP_OPT_GRID_MAX_MB: *value = c->grid_max_mb; break;
  }
  return GICP_OK;
}

gicp_status gicp_set_default_option(int option, int value) {
  gicp_status s = check_option(option, value);
  if (s) return s;
  g_opt_default[option].store(value);
  return GICP_OK;
}

gicp_status gicp_get_default_option(int option, int* value) {
  if (!value) return fail(GICP_EINVAL, "null argument");
  gicp_status s = check_option(option, 0);
  if (s) return s;
  *value = g_opt_default[option].load();
  return GICP_OK;
}

gicp_status gicp_get_tie_order(const gicp_ctx* c, int* nanoflann_order) {
  if (!c || !nanoflann_order) return fail(GICP_EINVAL, "null argument");
  *nanoflann_order = c->tie_exact ? 1 : 0;
  return GICP_OK;
}

namespace {
int64_t tree_bytes(const std::shared_ptr<NfTreeData>& t) {
  return t ? (int64_t)(t->vpts.bytes + t->nodes.bytes + t->box.bytes + t->status.bytes + t->sbox.bytes) : 0;
}
int64_t cloud_bytes(const std::shared_ptr<CloudData>& cd) {
  if (!cd) return 0;
  const CloudData& d = *cd;
  int64_t b = (int64_t)(d.pts.bytes + d.keys.bytes + d.perm.bytes + d.inv_perm.bytes + d.box_lo.bytes +
                        d.box_hi.bytes + d.quant.bytes + d.soa.bytes + d.dir.bytes);
  b += tree_bytes(d.nf) + tree_bytes(d.nfp);
  if (d.grid) b += (int64_t)(d.grid->dir.bytes + d.grid->fine.bytes + d.grid->ent.bytes);
  return b;
}
}  // namespace

gicp_status gicp_get_device_bytes(const gicp_ctx* c, int64_t* out, int nout) {
  if (!c || !out || nout < 1) return fail(GICP_EINVAL, "null argument");
  int64_t v[7] = {0, 0, 0, 0, 0, 0, 0};
  v[1] = cloud_bytes(c->tgt.cloud);
  v[2] = c->src.cloud == c->tgt.cloud ? 0 : cloud_bytes(c->src.cloud);
  v[3] = (c->tgt.cov ? (int64_t)c->tgt.cov->cov6.bytes : 0) + (c->src.cov && c->src.cov != c->tgt.cov ? (int64_t)c->src.cov->cov6.bytes : 0);
  v[4] = tree_bytes(c->tie_tree);
  v[5] = cloud_bytes(c->tie_whole) + (int64_t)(c->tie_scratch.bytes + c->tie_lidx.bytes + c->tie_out_nodes.bytes +
                                               c->tie_out_pts.bytes + c->tie_counts.bytes);
  const DevBuf* scratch[] = {&c->raw_bytes, &c->raw_pts, &c->partial, &c->nonfinite, &c->keys_tmp, &c->vals_tmp,
                             &c->sort_tmp, &c->knn, &c->corr, &c->sqd, &c->slab, &c->job_dev, &c->state_dev,
                             &c->tmp_out, &c->stats, &c->nf_desc, &c->mom, &c->search, &c->nf_scratch, &c->tie_buf,
                             &c->nf_err, &c->lazy_buf, &c->fb};
  for (const DevBuf* b : scratch) v[6] += (int64_t)b->bytes;
  if (c->nf_gated) v[6] += (int64_t)(c->nf_gated->vpts.bytes + c->nf_gated->nodes.bytes + c->nf_gated->box.bytes +
                                     c->nf_gated->status.bytes + c->nf_gated->sbox.bytes);
  v[0] = v[1] + v[2] + v[3] + v[4] + v[5] + v[6];
  for (int i = 0; i < nout && i < 7; ++i) out[i] = v[i];
  for (int i = 7; i < nout; ++i) out[i] = 0;
  return GICP_OK;
}

gicp_status gicp_set_target_grid(gicp_ctx* c, int mode) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  if (mode < GICP_GRID_OFF || mode > GICP_GRID_ON) return fail(GICP_EINVAL, "grid mode must be 0 (off), 1 (auto) or 2 (on)");
  c->grid_mode = mode;
  return GICP_OK;
}

gicp_status gicp_get_target_grid_info(gicp_ctx* c, gicp_grid_info* out) {
  if (!c || !out) return fail(GICP_EINVAL, "null argument");
  std::memset(out, 0, sizeof(*out));
  if (!c->tgt.cloud || !c->tgt.cloud->grid) return GICP_OK;
  *out = c->tgt.cloud->grid->info;
  out->built = grid_active(c) ? 1 : 0;
  return GICP_OK;
}

gicp_status gicp_get_lookup_stats(gicp_ctx* c, int64_t* walk_groups) {
  if (!c || !walk_groups) return fail(GICP_EINVAL, "null argument");
  *walk_groups = -1;
  if (!c->fb.p || !c->src.cloud) return GICP_OK;
  gicp_status s = set_device(c);
  if (s) return s;
  unsigned v = 0;
  const FbLayout fl(c->src.cloud->n);
  HIP_TRY(hipMemcpyAsync(&v, c->fb.as<char>() + fl.ctr + sizeof(unsigned) * kFbSegs * 32, sizeof(unsigned),
                         hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  *walk_groups = v;
  return GICP_OK;
}

gicp_status gicp_debug_nftree(gicp_ctx* c, int side, int32_t* vind, int32_t* nodes4, float* div2, size_t cap,
                              size_t* nnodes) {
  if (!c || (side != 0 && side != 1) || !nnodes) return fail(GICP_EINVAL, "invalid argument");
  Side& sd = side == GICP_SIDE_SOURCE ? c->src : c->tgt;
  if (!sd.cloud) return fail(GICP_ESTATE, "no cloud on this side");
  gicp_status s = set_device(c);
  if (s) return s;
  s = ensure_nftree(c, *sd.cloud, c->stream);
  if (s) return s;
  const NfTreeData& t = *sd.cloud->nf;
  HIP_TRY(nftree_join(t, c->stream));
  int st[2] = {0, 0};
  HIP_TRY(hipMemcpyAsync(st, t.status.p, sizeof(st), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (st[0]) return fail(GICP_EHIP, "nanoflann tree build failed (error bits " + std::to_string(st[0]) + ")");
  *nnodes = (size_t)st[1];
  if (!vind && !nodes4 && !div2) return GICP_OK;
  if (cap < (size_t)st[1]) return fail(GICP_EINVAL, "node capacity too small");
  const int n = t.n;
  DevBuf dv, dn, df;
  HIP_TRY(dv.ensure(sizeof(int) * (size_t)n));
  HIP_TRY(dn.ensure(sizeof(int) * 4 * (size_t)st[1]));
  HIP_TRY(df.ensure(sizeof(float) * 2 * (size_t)st[1]));
  launch_nf_export(c->stream, t.dev(), t.status.as<int>(), st[1], dv.as<int>(), dn.as<int>(), df.as<float>());
  HIP_TRY(hipGetLastError());
  if (vind) HIP_TRY(hipMemcpyAsync(vind, dv.p, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
  if (nodes4) HIP_TRY(hipMemcpyAsync(nodes4, dn.p, sizeof(int) * 4 * (size_t)st[1], hipMemcpyDeviceToHost, c->stream));
  if (div2) HIP_TRY(hipMemcpyAsync(div2, df.p, sizeof(float) * 2 * (size_t)st[1], hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GICP_OK;
}

gicp_status gicp_debug_nfbuild(gicp_ctx* c, int side, int stop, int32_t* vind, int64_t* info16, int32_t* status2,
                               void* scratch, size_t scratch_cap) {
  if (!c || (side != 0 && side != 1) || !vind || !info16 || !status2) return fail(GICP_EINVAL, "invalid argument");
  Side& sd = side == GICP_SIDE_SOURCE ? c->src : c->tgt;
  if (!sd.cloud) return fail(GICP_ESTATE, "no cloud on this side");
  gicp_status s = set_device(c);
  if (s) return s;
  NfTreeData t;
  long long off[16];
  s = nftree_build(c, *sd.cloud, c->stream, t, stop, off);
  if (s) return s;
  HIP_TRY(nftree_join(t, c->stream));
  for (int i = 0; i < 16; ++i) info16[i] = off[i];
  HIP_TRY(hipMemcpyAsync(status2, t.status.p, 2 * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  std::vector<float4> v((size_t)t.n);
  HIP_TRY(hipMemcpyAsync(v.data(), t.vpts.p, sizeof(float4) * (size_t)t.n, hipMemcpyDeviceToHost, c->stream));
  if (scratch && scratch_cap)
    HIP_TRY(hipMemcpyAsync(scratch, c->nf_scratch.p, std::min(scratch_cap, (size_t)off[13]), hipMemcpyDeviceToHost,
                           c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (int i = 0; i < t.n; ++i) {
    int w;
    std::memcpy(&w, &v[(size_t)i].w, sizeof(int));
    vind[i] = w;
  }
  return GICP_OK;
}

gicp_status gicp_get_moments(const gicp_ctx* c, double* out80) {
  if (!c || !out80) return fail(GICP_EINVAL, "null argument");
  std::memcpy(out80, final_state(c).last_mom, sizeof(double) * kSlabStride);
  return GICP_OK;
}

// diagnostics: per 64-query group counters of the LAST linearize launch
gicp_status gicp_debug_stats(gicp_ctx* c, int enable, unsigned int* out, size_t max_words, size_t* nwords) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  c->stats_on = enable != 0;
  if (out && c->src.cloud && c->stats.p) {
    const int q = search_queries_per_wave();
    const size_t groups = (c->src.cloud->n + q - 1) / q;
    const size_t words = std::min(max_words, (size_t)kStatFields * (groups + (groups + 3) / 4));  // phase A + B rows
    HIP_TRY(hipMemcpyAsync(out, c->stats.p, sizeof(unsigned int) * words, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (nwords) *nwords = words;
  }
  return GICP_OK;
}

gicp_status gicp_set_profiling(gicp_ctx* c, int enable) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  c->profiling = enable != 0;
  return GICP_OK;
}

gicp_status gicp_get_stage_times(gicp_ctx* c, gicp_stage_times* out) {
  if (!c || !out) return fail(GICP_EINVAL, "null argument");
  std::memset(out, 0, sizeof(*out));
  if (!c->st_ev[0]) return fail(GICP_ESTATE, "no profiled compute_covariances on this ctx");
  gicp_status s = set_device(c);
  if (s) return s;
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipStreamSynchronize(c->aux_stream));
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, c->st_ev[0], c->st_ev[1]));
  out->cov_ms = ms;
  if (c->st_tree) {
    HIP_TRY(hipEventElapsedTime(&ms, c->st_ev[2], c->st_ev[3]));
    out->tree_ms = ms;
  }
  if (c->st_resolve) {
    HIP_TRY(hipEventElapsedTime(&ms, c->st_ev[4], c->st_ev[5]));
    out->resolve_ms = ms;
  }
  return GICP_OK;
}

gicp_status gicp_synchronize(gicp_ctx* c) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  gicp_status s = set_device(c);
  if (s) return s;
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipStreamSynchronize(c->aux_stream));
  return GICP_OK;
}

gicp_status gicp_set_shard(gicp_ctx* c, int axis, float lo, float hi) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  if (axis < -1 || axis > 2) return fail(GICP_EINVAL, "shard axis must be -1 (none), 0, 1 or 2");
  if (axis >= 0 && !(lo < hi)) return fail(GICP_EINVAL, "empty shard range");
  c->own_axis = axis;
  c->own_lo = axis >= 0 ? lo : -INFINITY;
  c->own_hi = axis >= 0 ? hi : INFINITY;
  invalidate_align(c);
  return GICP_OK;
}

// ---- slab shards' tie order (tietree.hip, DESIGN.md §5 "Slab shards") ----
// Blob: header, the restricted tree's nodes, its points (x, y, z, local index).
struct TieBlobHeader {
  uint32_t magic, version;
  int32_t n_local, nnodes;
  float box[8];   // root_bbox lo (x, y, z, 0), hi (x, y, z, 0): the whole submap's
};
constexpr uint32_t kTieBlobMagic = 0x31545444u;   // "DTT1"

namespace {
gicp_status check_local_index(const int32_t* local_index, size_t n_local, size_t n) {
  std::vector<unsigned char> seen(n, 0);
  for (size_t i = 0; i < n_local; ++i) {
    if (local_index[i] < 0 || (size_t)local_index[i] >= n) return fail(GICP_EINVAL, "local_index out of range");
    if (seen[(size_t)local_index[i]]++) return fail(GICP_EINVAL, "local_index is not one-to-one");
  }
  return GICP_OK;
}
}  // namespace

gicp_status gicp_tie_builder_set(gicp_ctx* c, const float* xyz, size_t n, size_t stride) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  gicp_status s = set_device(c);
  if (s) return s;
  if (n == 0) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->tie_whole.reset();
    c->tie_scratch.reset();
    c->tie_lidx.reset();
    c->tie_out_nodes.reset();
    c->tie_out_pts.reset();
    c->tie_counts.reset();
    std::vector<unsigned char>().swap(c->tie_blob);
    return GICP_OK;
  }
  if (!xyz) return fail(GICP_EINVAL, "null argument");
  std::shared_ptr<CloudData> cd;
  s = build_cloud(c, xyz, n, stride, &cd);
  if (s) return s;
  auto t = std::make_shared<NfTreeData>();
  s = nftree_build(c, *cd, c->stream, *t, -1, nullptr, -1, nullptr, /*zero_nodes=*/true);
  if (s) return s;
  HIP_TRY(nftree_join(*t, c->stream));
  cd->nf = t;
  c->tie_whole = cd;
  return GICP_OK;
}

gicp_status gicp_tie_builder_export(gicp_ctx* c, const int32_t* local_index, size_t n_local, const void** blob,
                                    size_t* bytes) {
  if (!c || !blob || !bytes) return fail(GICP_EINVAL, "null argument");
  *blob = nullptr;
  *bytes = 0;
  if (!c->tie_whole || !c->tie_whole->nf) return fail(GICP_ESTATE, "no whole cloud: gicp_tie_builder_set first");
  if (n_local == 0 || !local_index) return fail(GICP_EINVAL, "empty local_index");
  const CloudData& W = *c->tie_whole;
  const NfTreeData& T = *W.nf;
  gicp_status s = check_local_index(local_index, n_local, (size_t)W.n);
  if (s) return s;
  s = set_device(c);
  if (s) return s;
  HIP_TRY(c->tie_scratch.ensure(tie_prune_scratch_bytes(T.n, T.cap)));
  HIP_TRY(c->tie_lidx.ensure(sizeof(int) * n_local));
  HIP_TRY(c->tie_out_nodes.ensure(sizeof(NfNode) * (size_t)T.cap));
  HIP_TRY(c->tie_out_pts.ensure(sizeof(float4) * n_local));
  HIP_TRY(c->tie_counts.ensure(sizeof(unsigned) * 4 + 2 * sizeof(float4)));
  HIP_TRY(hipMemcpyAsync(c->tie_lidx.p, local_index, sizeof(int) * n_local, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(launch_tie_prune(c->stream, T.dev(), T.cap, c->tie_lidx.as<int>(), (int)n_local, c->tie_scratch.p,
                           c->tie_out_nodes.as<NfNode>(), c->tie_out_pts.as<float4>(), c->tie_counts.as<unsigned>()));
  unsigned cnt[4];
  float4 box[2];
  int bstat = 0;
  HIP_TRY(hipMemcpyAsync(cnt, c->tie_counts.p, sizeof(cnt), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(box, T.box.p, sizeof(box), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(&bstat, T.status.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (bstat) return fail(GICP_EHIP, "the whole cloud's tree build failed");
  if (cnt[2] || cnt[0] != (unsigned)n_local || cnt[1] == 0 || cnt[1] > (unsigned)T.cap)
    return fail(GICP_EHIP, "tie tree restriction failed");
  const size_t nb = sizeof(TieBlobHeader) + sizeof(NfNode) * cnt[1] + sizeof(float4) * n_local;
  c->tie_blob.resize(nb);
  TieBlobHeader h{};
  h.magic = kTieBlobMagic;
  h.version = 1;
  h.n_local = (int32_t)n_local;
  h.nnodes = (int32_t)cnt[1];
  std::memcpy(h.box, box, sizeof(h.box));
  std::memcpy(c->tie_blob.data(), &h, sizeof(h));
  unsigned char* q = c->tie_blob.data() + sizeof(h);
  HIP_TRY(hipMemcpyAsync(q, c->tie_out_nodes.p, sizeof(NfNode) * cnt[1], hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(q + sizeof(NfNode) * cnt[1], c->tie_out_pts.p, sizeof(float4) * n_local,
                         hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  *blob = c->tie_blob.data();
  *bytes = nb;
  return GICP_OK;
}

gicp_status gicp_set_tie_tree(gicp_ctx* c, const void* blob, size_t bytes) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  if (bytes == 0) {
    c->tie_tree.reset();
    invalidate_align(c);
    return GICP_OK;
  }
  if (!blob || bytes < sizeof(TieBlobHeader)) return fail(GICP_EINVAL, "tie tree blob too short");
  TieBlobHeader h;
  std::memcpy(&h, blob, sizeof(h));
  if (h.magic != kTieBlobMagic || h.version != 1) return fail(GICP_EINVAL, "not a tie tree blob");
  if (!c->tgt.cloud) return fail(GICP_ESTATE, "set the local target first");
  const int nl = c->tgt.cloud->n;
  if (h.n_local != nl) return fail(GICP_EINVAL, "tie tree is not for a target of this size");
  if (h.nnodes < 1 || bytes != sizeof(h) + sizeof(NfNode) * (size_t)h.nnodes + sizeof(float4) * (size_t)nl)
    return fail(GICP_EINVAL, "tie tree blob size mismatch");
  const unsigned char* q = static_cast<const unsigned char*>(blob) + sizeof(h);
  std::vector<NfNode> nodes((size_t)h.nnodes);
  std::vector<float4> pts((size_t)nl);
  std::memcpy(nodes.data(), q, sizeof(NfNode) * nodes.size());
  std::memcpy(pts.data(), q + sizeof(NfNode) * nodes.size(), sizeof(float4) * pts.size());
  // a tree: every node reached once from the root, within the search's depth;
  // the leaves' point ranges partition [0, n_local)
  {
    std::vector<unsigned char> seen(nodes.size(), 0);
    std::vector<std::pair<int, int>> st{{0, 0}};
    long covered = 0;
    std::vector<int> cover((size_t)nl + 1, 0);
    while (!st.empty()) {
      const auto [v, d] = st.back();
      st.pop_back();
      if (v < 0 || v >= h.nnodes || seen[(size_t)v]++ || d >= kNfStack) return fail(GICP_EINVAL, "tie tree is not a tree");
      const NfNode& nd = nodes[(size_t)v];
      if (nd.feat == -1) {
        if (nd.c1 < 0 || nd.c2 > nl || nd.c1 > nd.c2) return fail(GICP_EINVAL, "tie tree leaf range out of bounds");
        covered += nd.c2 - nd.c1;
        cover[(size_t)nd.c1] += 1;
        cover[(size_t)nd.c2] -= 1;
      } else {
        if (nd.feat < 0 || nd.feat > 2) return fail(GICP_EINVAL, "tie tree node has no cut dimension");
        st.push_back({nd.c2, d + 1});
        st.push_back({nd.c1, d + 1});
      }
    }
    int run = 0;
    for (int i = 0; i < nl; ++i)
      if ((run += cover[(size_t)i]) != 1) return fail(GICP_EINVAL, "tie tree leaves do not partition the points");
    if (covered != nl) return fail(GICP_EINVAL, "tie tree leaves do not partition the points");
  }
  gicp_status s = set_device(c);
  if (s) return s;
  {
    // its points are the local target's, each once (point ids = local indices)
    std::vector<float4> lp((size_t)nl);
    HIP_TRY(hipMemcpyAsync(lp.data(), c->tgt.cloud->pts.p, sizeof(float4) * nl, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    std::vector<float4> by_orig((size_t)nl);
    for (const float4& p : lp) {
      int o;
      std::memcpy(&o, &p.w, sizeof(int));
      by_orig[(size_t)o] = p;
    }
    std::vector<unsigned char> seen((size_t)nl, 0);
    for (const float4& p : pts) {
      int w;
      std::memcpy(&w, &p.w, sizeof(int));
      if (w < 0 || w >= nl || seen[(size_t)w]++) return fail(GICP_EINVAL, "tie tree points are not the local target's");
      const float4& l = by_orig[(size_t)w];
      if (l.x != p.x || l.y != p.y || l.z != p.z)
        return fail(GICP_EINVAL, "tie tree points are not the local target's (local_index does not map the local "
                                 "target's points onto the whole cloud's)");
    }
  }
  auto t = std::make_shared<NfTreeData>();
  t->n = nl;
  t->cap = h.nnodes;
  HIP_TRY(t->vpts.ensure(sizeof(float4) * (size_t)nl));
  HIP_TRY(t->nodes.ensure(sizeof(NfNode) * (size_t)h.nnodes));
  HIP_TRY(t->box.ensure(2 * sizeof(float4)));
  HIP_TRY(t->status.ensure(2 * sizeof(int)));
  HIP_TRY(hipEventCreateWithFlags(&t->ready, hipEventDisableTiming));
  const int status[2] = {0, h.nnodes};
  HIP_TRY(hipMemcpyAsync(t->vpts.p, pts.data(), sizeof(float4) * (size_t)nl, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(t->nodes.p, nodes.data(), sizeof(NfNode) * nodes.size(), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(t->box.p, h.box, sizeof(h.box), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(t->status.p, status, sizeof(status), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipEventRecord(t->ready, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));   // the host vectors go out of scope
  c->tie_tree = t;
  invalidate_align(c);
  return GICP_OK;
}

gicp_status gicp_set_tie_target(gicp_ctx* c, const float* xyz, size_t n, size_t stride, const int32_t* local_index,
                                size_t n_local) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  if (n == 0) return gicp_set_tie_tree(c, nullptr, 0);
  if (!xyz || !local_index) return fail(GICP_EINVAL, "null argument");
  if (!c->tgt.cloud || (int)n_local != c->tgt.cloud->n) return fail(GICP_ESTATE, "set the local target first (n_local = its size)");
  gicp_status s = check_local_index(local_index, n_local, n);
  if (s) return s;
  s = gicp_tie_builder_set(c, xyz, n, stride);
  const void* blob = nullptr;
  size_t nb = 0;
  if (!s) s = gicp_tie_builder_export(c, local_index, n_local, &blob, &nb);
  if (!s) s = gicp_set_tie_tree(c, blob, nb);
  const gicp_status s2 = gicp_tie_builder_set(c, nullptr, 0, 0);   // the whole cloud does not stay
  return s ? s : s2;
}

gicp_status gicp_set_tie_trees_from_root(gicp_ctx* c, int root, const void* const* blobs, const size_t* sizes) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  if (!c->comm) return fail(GICP_ESTATE, "no communicator (gicp_set_comm)");
  if (root < 0 || root >= c->nranks) return fail(GICP_EINVAL, "root out of range");
  const int R = c->nranks, me = c->rank;
  // A root without blobs (its builder failed) still enters the collective and
  // broadcasts a failure word, so no rank waits forever on the broadcast.
  const bool root_failed = me == root && (!blobs || !sizes);
  if (R == 1) {
    if (root_failed) return fail(GICP_EINVAL, "the root passes every rank's blob");
    return gicp_set_tie_tree(c, blobs[0], sizes[0]);   // nothing to send
  }
  const Rccl& r = rccl();
  if (!r.ok || !r.broadcast || !r.send || !r.recv || !r.group_start || !r.group_end)
    return fail(GICP_ECOMM, "RCCL point-to-point entry points missing");
  gicp_status s = set_device(c);
  if (s) return s;
  s = drain_tail(c);
  if (s) return s;
  // every rank's blob size and the root's status word (one broadcast), then
  // root -> rank point-to-point
  DevBuf dsz;
  HIP_TRY(dsz.ensure(sizeof(unsigned long long) * ((size_t)R + 1)));
  std::vector<unsigned long long> sz((size_t)R + 1, 0);
  if (me == root) {
    if (root_failed) sz[(size_t)R] = 1;
    else
      for (int k = 0; k < R; ++k) sz[(size_t)k] = sizes[k];
  }
  HIP_TRY(hipMemcpyAsync(dsz.p, sz.data(), sizeof(unsigned long long) * (R + 1), hipMemcpyHostToDevice, c->stream));
  NCCL_TRY(r.broadcast(dsz.p, dsz.p, (size_t)R + 1, ncclUint64, root, c->comm, c->stream));
  HIP_TRY(hipMemcpyAsync(sz.data(), dsz.p, sizeof(unsigned long long) * (R + 1), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (root_failed) return fail(GICP_EINVAL, "the root passes every rank's blob");
  if (sz[(size_t)R]) return fail(GICP_ECOMM, "the root's tie-tree builder failed (no blobs sent)");
  DevBuf sendb, recvb;
  std::vector<size_t> off((size_t)R + 1, 0);
  for (int k = 0; k < R; ++k) off[(size_t)k + 1] = off[(size_t)k] + (k == root ? 0 : (size_t)sz[(size_t)k]);
  if (me == root && off[(size_t)R] > 0) {
    HIP_TRY(sendb.ensure(off[(size_t)R]));
    for (int k = 0; k < R; ++k)
      if (k != root && sz[(size_t)k])
        HIP_TRY(hipMemcpyAsync(sendb.as<char>() + off[(size_t)k], blobs[k], sz[(size_t)k], hipMemcpyHostToDevice, c->stream));
  }
  if (me != root && sz[(size_t)me]) HIP_TRY(recvb.ensure(sz[(size_t)me]));
  NCCL_TRY(r.group_start());
  if (me == root) {
    for (int k = 0; k < R; ++k)
      if (k != root && sz[(size_t)k]) NCCL_TRY(r.send(sendb.as<char>() + off[(size_t)k], sz[(size_t)k], ncclUint8, k, c->comm, c->stream));
  } else if (sz[(size_t)me]) {
    NCCL_TRY(r.recv(recvb.p, sz[(size_t)me], ncclUint8, root, c->comm, c->stream));
  }
  NCCL_TRY(r.group_end());
  std::vector<unsigned char> mine;
  if (me != root && sz[(size_t)me]) {
    mine.resize(sz[(size_t)me]);
    HIP_TRY(hipMemcpyAsync(mine.data(), recvb.p, mine.size(), hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (me == root) return gicp_set_tie_tree(c, blobs[root], sizes[root]);
  return gicp_set_tie_tree(c, mine.data(), mine.size());
}

gicp_status gicp_set_shard_groups(gicp_ctx* c, int nparts, int part) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  if (nparts < 0 || (nparts > 0 && (part < 0 || part >= nparts))) return fail(GICP_EINVAL, "invalid shard part");
  c->own_mod = nparts <= 1 ? 0 : nparts;
  c->own_rem = nparts <= 1 ? 0 : part;
  invalidate_align(c);
  return GICP_OK;
}

gicp_status gicp_comm_unique_id(uint8_t* out, size_t nbytes) {
  if (!out || nbytes < sizeof(ncclUniqueId)) return fail(GICP_EINVAL, "unique id buffer must hold 128 bytes");
  const Rccl& r = rccl();
  if (!r.ok) return fail(GICP_ECOMM, r.why);
  ncclUniqueId id;
  NCCL_TRY(r.get_unique_id(&id));
  std::memcpy(out, &id, sizeof(id));
  return GICP_OK;
}

gicp_status gicp_set_comm(gicp_ctx* c, const uint8_t* id, size_t nbytes, int nranks, int rank) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  gicp_status s = set_device(c);
  if (s) return s;
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->comm) {
    (void)rccl().comm_destroy(c->comm);
    c->comm = nullptr;
  }
  drop_graphs(c);
  c->nranks = 1;
  c->rank = 0;
  c->comm_graphs = true;
  c->tail_pending = false;  // the stream was synchronized above
  c->speculate = true;      // identical launch history on every rank
  c->predicted_iters = kDefaultPredictedIters;
  if (nranks == 0) return GICP_OK;  // detach
  if (!id || nbytes < sizeof(ncclUniqueId) || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(GICP_EINVAL, "invalid communicator arguments");
  const Rccl& r = rccl();
  if (!r.ok) return fail(GICP_ECOMM, r.why);
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  NCCL_TRY(r.comm_init_rank(&c->comm, nranks, uid, rank));
  HIP_TRY(c->mom.ensure(sizeof(double) * kSlabStride));
  c->nranks = nranks;
  c->rank = rank;
  invalidate_align(c);
  return GICP_OK;
}

gicp_status gicp_get_comm_info(const gicp_ctx* c, int* nranks, int* rank, int* graphs) {
  if (!c) return fail(GICP_EINVAL, "null ctx");
  if (nranks) *nranks = c->comm ? c->nranks : 0;
  if (rank) *rank = c->rank;
  if (graphs) *graphs = (!c->comm || c->comm_graphs) ? 1 : 0;
  return GICP_OK;
}

gicp_status gicp_get_stream(const gicp_ctx* c, void** stream) {
  if (!c || !stream) return fail(GICP_EINVAL, "null argument");
  *stream = (void*)c->stream;
  return GICP_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Frame-parallel S2S batch (ddlo_gicp.h): nstreams chained chunks, one ctx,
// HIP stream and host thread each.
gicp_status gicp_s2s_batch(int device, const gicp_params* p, const float* const* clouds, const size_t* sizes,
                           size_t stride_bytes, int nframes, int nstreams, float* out16, gicp_result* res) {
  if (!p || !clouds || !sizes || !out16 || nframes < 1 || nstreams < 1)
    return fail(GICP_EINVAL, "invalid batch arguments");
  for (int t = 0; t < nframes; ++t)
    if (!clouds[t] || sizes[t] == 0) return fail(GICP_EINVAL, "null or empty frame");
  for (int e = 0; e < 16; ++e) out16[e] = (e % 5 == 0) ? 1.f : 0.f;
  if (res) std::memset(&res[0], 0, sizeof(gicp_result));
  const int npairs = nframes - 1;
  if (npairs == 0) return GICP_OK;
  const int nthreads = std::min(nstreams, npairs);
  std::vector<gicp_status> status(nthreads, GICP_OK);
  std::vector<std::string> errors(nthreads);
  // contexts are made (and destroyed) on this thread, outside any worker's
  // graph capture
  std::vector<gicp_ctx*> ctxs(nthreads, nullptr);
  for (int w = 0; w < nthreads; ++w) {
    gicp_status s = gicp_ctx_create(device, &ctxs[w]);
    if (!s) s = gicp_set_params(ctxs[w], p);
    if (!s) {
      const char* os = dev_getenv("DDLO_NF_OWN_STREAM");   // 0: the second stream (A/B)
      ctxs[w]->nf_same_stream = !(os && *os == '0');
    }
    if (s) {
      const std::string why = g_last_error;
      for (auto* c : ctxs)
        if (c) (void)gicp_ctx_destroy(c);
      return fail(s, why);
    }
  }
  auto worker = [&](int w) {
    // pairs (t-1, t) for t in [t0, t1)
    const int t0 = 1 + (int)((long)npairs * w / nthreads);
    const int t1 = 1 + (int)((long)npairs * (w + 1) / nthreads);
    gicp_ctx* c = ctxs[w];
    gicp_status s = gicp_set_target(c, clouds[t0 - 1], sizes[t0 - 1], stride_bytes);
    for (int t = t0; t < t1 && !s; ++t) {
      s = set_source_impl(c, clouds[t], sizes[t], stride_bytes, 1, true);
      if (!s) s = gicp_align(c, nullptr, out16 + 16 * (size_t)t, res ? &res[t] : nullptr);
      if (!s) s = gicp_swap_source_target(c);  // scan t becomes the next target (odom.cc:768)
    }
    if (s) {
      status[w] = s;
      errors[w] = g_last_error;
    }
  };
  std::vector<std::thread> pool;
  for (int w = 1; w < nthreads; ++w) pool.emplace_back(worker, w);
  worker(0);
  for (auto& th : pool) th.join();
  for (auto* c : ctxs) (void)gicp_ctx_destroy(c);
  for (int w = 0; w < nthreads; ++w)
    if (status[w]) return fail(status[w], "s2s batch chunk " + std::to_string(w) + ": " + errors[w]);
  return GICP_OK;
}
