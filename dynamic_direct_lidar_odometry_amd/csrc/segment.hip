// segment.hip — range-image segmentation of one organized scan
// (include/ddlo_segment.h).
//
// Device: k_seg_pixels, one thread per pixel, fuses
//   projectScan    (detection.cpp:292-329): range from the sensor position,
//                  minimum range, the "full cloud" (NaN where no range);
//   groundRemoval  (:458-491): the reference walks each column from the
//                  bottom, and a pixel's mark is written by the test of its
//                  own row pair (lower = r: no info -> -1, ground -> 1) after
//                  the test of the pair below it (lower = r + 1: ground -> 1
//                  on the upper pixel).  The last write decides, so
//                    ground(r) = -1 if test(r) has no info, 1 if test(r) is
//                    ground, else 1 if test(r + 1) is ground, else 0
//                  for r in the tested rows; the row just above them only
//                  receives the test(r + 1) write.  Each thread evaluates the
//                  (at most two) tests that write its pixel: no column walk;
//   label init     (:493-504): -1 for ground or no-range pixels, else 0.
// Host: the labelling (cloudSegmentation / labelComponents, :510-724) is a
// breadth-first search whose result depends on the visiting order (segment
// numbers follow the row-major scan, min_z / max_z is an if / else-if over
// the push order, the residual sum is a float sum in push order), so it runs
// on the host as the north star places it, over the label image read back.
//
// Float behaviour follows the reference, where ddlo.h:35 includes <stdlib.h>
// (libstdc++'s wrapper brings std::abs into the global namespace, <cmath>
// the float atan2 / sqrt) so the unqualified abs / atan2 / sqrt calls on
// floats are the float overloads; -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/ddlo_segment.h"
#include "gicp_types.hpp"
#include "launch.hpp"
#include "runtime.hpp"

namespace ddlo {
namespace {

using rt::DevBuf;
using rt::fail;

constexpr int kRejected = DDLO_SEG_REJECTED;

struct SegPixelArgs {
  const unsigned char* raw;
  size_t stride;
  int H, W;
  float x0, y0, z0;      // -T(0:3, 3)
  float min_range;
  int ground_rows;
  float mount, thr;
  float* range;
  signed char* ground;
  int* label;
};

// full_cloud_ point of pixel i (:309-327): the cloud point when finite with
// range >= minimum_range_, else nan_point_.
__device__ __forceinline__ float3 full_point(const SegPixelArgs& a, int i, float* range_out) {
  const float* p = reinterpret_cast<const float*>(a.raw + (size_t)i * a.stride);
  const float px = p[0], py = p[1], pz = p[2];
  float r = 0.f;
  float3 f = make_float3(NAN, NAN, NAN);
  if (isfinite(px) && isfinite(py) && isfinite(pz)) {   // pcl::isFinite
    const float x = px + a.x0, y = py + a.y0, z = pz + a.z0;
    const float d = (float)sqrt((double)((x * x + y * y) + z * z));   // correctly rounded sqrtf
    if (!(d < a.min_range)) {
      r = d;
      f = make_float3(px, py, pz);
    }
  }
  if (range_out) *range_out = r;
  return f;
}

// One ground test, lower = (row, col), upper = (row - 1, col): -1 no info,
// 1 ground, 0 neither (:470-489).
__device__ __forceinline__ int ground_test(const float3& lo, const float3& up, float mount, float thr) {
  if (lo.x == 0.f || up.x == 0.f) return -1;   // a NaN point is not == 0: it falls through to a NaN angle
  const float dx = up.x - lo.x, dy = up.y - lo.y, dz = up.z - lo.z;
  // atan2(float, float) * 180 -> float, / M_PI -> double, stored as float.
  // atan2f is taken as the rounded double result (glibc's atan2f agrees but
  // for rare last-ulp cases; the device atan2f is less accurate)
  const float s = (float)sqrt((double)(dx * dx + dy * dy));
  const float at = (float)atan2((double)dz, (double)s);
  const float angle = (float)((double)(at * 180.f) / M_PI);
  return fabsf(angle - mount) <= thr ? 1 : 0;
}

__global__ __launch_bounds__(256) void k_seg_pixels(SegPixelArgs a) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  const int row = blockIdx.y;
  if (col >= a.W) return;
  const int i = row * a.W + col;
  float r;
  const float3 me = full_point(a, i, &r);
  const int first = a.H - a.ground_rows;   // tested lower rows: first .. H - 1
  signed char g = 0;
  if (row >= first) {   // own test (lower = row, upper = row - 1; row >= 1 since ground_rows < H)
    const float3 up = full_point(a, i - a.W, nullptr);
    const int t = ground_test(me, up, a.mount, a.thr);
    if (t != 0) g = (signed char)t;
  }
  if (g == 0 && row + 1 < a.H && row + 1 >= first) {   // the test below, which marks this pixel as its upper
    const float3 lo = full_point(a, i + a.W, nullptr);
    if (ground_test(lo, me, a.mount, a.thr) == 1) g = 1;
  }
  a.range[i] = r;
  a.ground[i] = g;
  a.label[i] = (g == 1 || r == 0.f) ? DDLO_SEG_EXCLUDED : DDLO_SEG_UNLABELLED;
}

inline int cdiv_s(long a, long b) { return (int)((a + b - 1) / b); }

// The labelling's queues, kept across scans (a ddlo_seg keeps one): a fresh
// set per scan cost four zero-filled allocations of the image size.
struct LabelWork {
  std::vector<int> qy, qx, py, px, rows_hit;
  std::vector<char> line_flag;   // all zero between components
};

// cloudSegmentation + labelComponents (detection.cpp:510-724) over host images.
struct Labeller {
  const ddlo_seg_params& p;
  const float* range;     // H x W
  const float* z;         // H x W: cloud_in_t z
  const float* resid;     // H x W or nullptr (icp_residuals_set_ false)
  int* label;             // H x W, in: -1 / 0
  float sin_x, cos_x, sin_y, cos_y, sensor_z;
  // the angle test without atan2 away from the threshold: atan is monotonic,
  // so for x > 0 the float atan2f(y, x) (within 1 ulp of atan(y / x)) is
  // above theta when y / x > tan(theta (1 + 1e-6)) and not above it when
  // y / x < tan(theta (1 - 1e-6)); in between (and for x <= 0) the
  // reference's atan2 decides.  Same decisions, one division per edge.
  double tan_lo = 0.0, tan_hi = 0.0;
  bool tan_ok = false;
  int label_count = 1;
  std::vector<double>& avg_residual;   // by label
  std::vector<int>& qy;
  std::vector<int>& qx;
  std::vector<int>& py;
  std::vector<int>& px;
  std::vector<int>& rows_hit;
  std::vector<char>& line_flag;

  Labeller(const ddlo_seg_params& p_, const float* range_, const float* z_, const float* resid_, int* label_,
           float sensor_z_, std::vector<double>& avg, LabelWork& w)
      : p(p_), range(range_), z(z_), resid(resid_), label(label_), sensor_z(sensor_z_), avg_residual(avg), qy(w.qy),
        qx(w.qx), py(w.py), px(w.px), rows_hit(w.rows_hit), line_flag(w.line_flag) {
    const int H = p.rows, W = p.cols;
    // loadParams :82-83,108-111: ang_res_x_ = 360.0 / float(W_) (double, stored
    // as float), ang_res_y_ = 2 * ang_bottom_ / float(H_ - 1) (float); double sin/cos
    const float ang_res_x = (float)(360.0 / (double)(float)W);
    const float ang_res_y = 2.f * p.ang_bottom / (float)(H - 1);
    sin_x = (float)std::sin(ang_res_x / 180.0 * M_PI);
    cos_x = (float)std::cos(ang_res_x / 180.0 * M_PI);
    sin_y = (float)std::sin(ang_res_y / 180.0 * M_PI);
    cos_y = (float)std::cos(ang_res_y / 180.0 * M_PI);
    const double th = (double)p.theta;
    tan_ok = th > 1e-3 && th < 1.5;   // a threshold well inside (0, pi / 2): both bounds finite and ordered
    if (tan_ok) {
      tan_lo = std::tan(th * (1.0 - 1e-6));
      tan_hi = std::tan(th * (1.0 + 1e-6));
    }
    const size_t n = (size_t)H * W;
    if (qy.size() < n) {   // (grown once; every slot is written before it is read)
      qy.resize(n);
      qx.resize(n);
      py.resize(n);
      px.resize(n);
    }
    if (line_flag.size() != (size_t)H) line_flag.assign(H, 0);
    rows_hit.clear();
    rows_hit.reserve(H);
    avg_residual.assign(1, 0.0);
  }

  bool in_window(int r, int c) const { return r >= p.win_row0 && r <= p.win_row1 && c >= p.win_col0 && c <= p.win_col1; }

  void run() {
    // seeds in row-major order inside the window (:519-522)
    const int r0 = std::max(0, p.win_row0), r1 = std::min(p.rows - 1, p.win_row1);
    const int c0 = std::max(0, p.win_col0), c1 = std::min(p.cols - 1, p.win_col1);
    for (int i = r0; i <= r1; ++i)
      for (int j = c0; j <= c1; ++j)
        if (label[(size_t)i * p.cols + j] == 0) component(i, j);
  }

  void component(int row, int col) {
    const int H = p.rows, W = p.cols;
    int head = 0, tail = 1;
    qy[0] = row;
    qx[0] = col;
    float min_z = 1e6f, max_z = -1e6f, min_dist = 1e6f, max_dist = -1e6f, total_res = 0.f;
    int res_count = 0;
    py[0] = row;
    px[0] = col;
    int pushed = 1;
    static const int dr[4] = {-1, 0, 0, 1}, dc[4] = {0, 1, -1, 0};   // neighbor_iterator_ (:133-145)
    while (head < tail) {
      const int fy = qy[head], fx = qx[head];
      ++head;
      label[(size_t)fy * W + fx] = label_count;
      for (int k = 0; k < 4; ++k) {
        const int ty = fy + dr[k];
        int tx = fx + dc[k];
        if (ty < 0 || ty >= H) continue;
        if (!in_window(ty, tx)) continue;   // (size_t) compare in the reference: negative never passes
        if (tx < 0) tx = W - 1;             // wrap after the window test, as :598-601
        if (tx >= W) tx = 0;
        const size_t t = (size_t)ty * W + tx, f = (size_t)fy * W + fx;
        if (label[t] != 0) continue;
        const float d1 = std::max(range[f], range[t]);
        const float d2 = std::min(range[f], range[t]);
        const float sa = dr[k] == 0 ? sin_x : sin_y, ca = dr[k] == 0 ? cos_x : cos_y;
        const float y = d2 * sa, x = d1 - d2 * ca;
        bool pass;
        const double ratio = x > 0.f ? (double)y / (double)x : 0.0;
        if (tan_ok && x > 0.f && ratio > tan_hi) pass = true;
        else if (tan_ok && x > 0.f && ratio < tan_lo) pass = false;
        else pass = std::atan2(y, x) > p.theta;
        if (pass) {
          const double zz = z[t];
          if (zz < min_z && zz != 0) min_z = (float)zz;
          else if (zz > max_z) max_z = (float)zz;
          min_dist = std::min(min_dist, std::min(d1, d2));
          max_dist = std::max(max_dist, std::max(d1, d2));
          qy[tail] = ty;
          qx[tail] = tx;
          ++tail;
          label[t] = label_count;
          if (!line_flag[ty]) {
            line_flag[ty] = 1;
            rows_hit.push_back(ty);
          }
          py[pushed] = ty;
          px[pushed] = tx;
          ++pushed;
          if (resid && resid[t] > 0) {
            total_res += resid[t];
            ++res_count;
          }
        }
      }
    }
    const int lines = (int)rows_hit.size();
    for (int r : rows_hit) line_flag[r] = 0;
    rows_hit.clear();
    (void)min_dist;
    bool feasible = false;
    if (pushed >= 50 && lines >= p.min_line_num) feasible = true;
    else if (pushed >= p.valid_point_num && lines >= p.valid_line_num) feasible = true;
    if (feasible) feasible = max_dist <= p.max_distance;
    if (feasible) {
      const float dz = max_z - min_z;
      feasible = p.min_delta_z <= dz && dz <= p.max_delta_z;
    }
    // avg_residuum = res_count > 0 ? total_residuum / res_count : 0 — a float
    // quotient (float / int, float / int conditional), stored as double
    double avg = 0.0;
    if (feasible && resid) avg = (double)(res_count > 0 ? total_res / (float)res_count : 0.f);
    if (feasible) feasible = min_z - sensor_z <= p.max_elevation;
    if (feasible) {
      avg_residual.push_back(avg);   // avg_residuals_[label_count_]
      ++label_count;
    } else {
      for (int i = 0; i < pushed; ++i) label[(size_t)py[i] * W + px[i]] = kRejected;
    }
  }
};

gicp_status check_params(const ddlo_seg_params* p) {
  if (!p) return fail(GICP_EINVAL, "null params");
  if (p->rows < 2 || p->cols < 1 || (long)p->rows * p->cols > INT32_MAX / 4) return fail(GICP_EINVAL, "invalid image size");
  if (p->ground_rows < 0 || p->ground_rows >= p->rows) return fail(GICP_EINVAL, "ground_rows must be in [0, rows)");
  return GICP_OK;
}

}  // namespace
}  // namespace ddlo

using namespace ddlo;

struct ddlo_seg {
  int device = 0;
  ddlo_seg_params p{};
  hipStream_t s = nullptr;
  rt::DevBuf raw, range, ground, label;
  float* pin = nullptr;               // range | label | ground, pinned
  size_t pin_bytes = 0;
  std::vector<float> z;
  // the last scan's images: the pinned read-back buffers themselves (the
  // labelling rewrites h_label in place)
  const float* h_range = nullptr;
  const signed char* h_ground = nullptr;
  int* h_label = nullptr;
  size_t hn = 0;
  std::vector<double> avg;
  LabelWork work;
  bool have = false;
  ddlo_seg_result last{};
};

extern "C" {

gicp_status ddlo_seg_default_params(ddlo_seg_params* p) {
  if (!p) return fail(GICP_EINVAL, "null params");
  std::memset(p, 0, sizeof(*p));
  p->rows = 128;
  p->cols = 1024;
  p->ang_bottom = 45.f;
  p->ground_rows = 30;
  p->ground_angle_threshold = 10.f;
  p->minimum_range = 10.f;
  p->sensor_mount_angle = 10.f;
  p->theta = (float)(60.0 / 180.0 * M_PI);
  p->valid_point_num = 15;
  p->min_line_num = 5;
  p->valid_line_num = 5;
  p->min_delta_z = 0.1f;
  p->max_delta_z = 3.0f;
  p->max_distance = 20.f;
  p->max_elevation = 2.0f;
  p->win_row0 = p->win_col0 = 156;
  p->win_row1 = p->win_col1 = 356;
  return GICP_OK;
}

gicp_status ddlo_seg_create(int device, const ddlo_seg_params* p, ddlo_seg** out) {
  if (!out) return fail(GICP_EINVAL, "null out");
  *out = nullptr;
  auto o = std::make_unique<ddlo_seg>();
  if (p) o->p = *p;
  else ddlo_seg_default_params(&o->p);
  if (gicp_status st = check_params(&o->p)) return st;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return fail(GICP_EHIP, "no HIP device " + std::to_string(device) + " (HIP library present, device not visible)");
  o->device = device;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipStreamCreateWithFlags(&o->s, hipStreamNonBlocking));
  const size_t n = (size_t)o->p.rows * o->p.cols;
  o->pin_bytes = n * (sizeof(float) + sizeof(int)) + n;
  if (hipHostMalloc((void**)&o->pin, o->pin_bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipStreamDestroy(o->s);
    return fail(GICP_EHIP, "pinned allocation failed");
  }
  *out = o.release();
  return GICP_OK;
}

gicp_status ddlo_seg_destroy(ddlo_seg* s) {
  if (!s) return GICP_OK;
  (void)hipSetDevice(s->device);
  (void)hipStreamSynchronize(s->s);
  s->raw.reset();
  s->range.reset();
  s->ground.reset();
  s->label.reset();
  if (s->pin) (void)hipHostFree(s->pin);
  (void)hipStreamDestroy(s->s);
  delete s;
  return GICP_OK;
}

gicp_status ddlo_seg_process(ddlo_seg* o, const float* xyz_t, size_t stride, const float T[16], const float* residual,
                             ddlo_seg_result* res) {
  if (!o || !xyz_t || !T || stride < 12 || stride % 4) return fail(GICP_EINVAL, "invalid argument");
  const ddlo_seg_params& p = o->p;
  const int H = p.rows, W = p.cols;
  const size_t n = (size_t)H * W;
  HIP_TRY(hipSetDevice(o->device));
  o->have = false;
  const size_t raw_sz = (n - 1) * stride + 12;
  HIP_TRY(o->raw.ensure(raw_sz));
  HIP_TRY(o->range.ensure(sizeof(float) * n));
  HIP_TRY(o->ground.ensure(n));
  HIP_TRY(o->label.ensure(sizeof(int) * n));
  HIP_TRY(hipMemcpyAsync(o->raw.p, xyz_t, raw_sz, hipMemcpyHostToDevice, o->s));
  SegPixelArgs a{};
  a.raw = o->raw.as<unsigned char>();
  a.stride = stride;
  a.H = H;
  a.W = W;
  a.x0 = -T[3];   // projectScan: sensor position = T(0:3, 3) (:296-298)
  a.y0 = -T[7];
  a.z0 = -T[11];
  a.min_range = p.minimum_range;
  a.ground_rows = p.ground_rows;
  a.mount = p.sensor_mount_angle;
  a.thr = p.ground_angle_threshold;
  a.range = o->range.as<float>();
  a.ground = o->ground.as<signed char>();
  a.label = o->label.as<int>();
  k_seg_pixels<<<dim3(cdiv_s(W, 256), H), 256, 0, o->s>>>(a);
  HIP_TRY(hipGetLastError());
  float* pin_range = o->pin;
  int* pin_label = reinterpret_cast<int*>(o->pin + n);
  signed char* pin_ground = reinterpret_cast<signed char*>(pin_label + n);
  HIP_TRY(hipMemcpyAsync(pin_range, o->range.p, sizeof(float) * n, hipMemcpyDeviceToHost, o->s));
  HIP_TRY(hipMemcpyAsync(pin_label, o->label.p, sizeof(int) * n, hipMemcpyDeviceToHost, o->s));
  HIP_TRY(hipMemcpyAsync(pin_ground, o->ground.p, n, hipMemcpyDeviceToHost, o->s));
  // the labelling reads cloud_in_t z (:629); gathered while the device works
  o->z.resize(n);
  const unsigned char* b = reinterpret_cast<const unsigned char*>(xyz_t);
  for (size_t i = 0; i < n; ++i) std::memcpy(&o->z[i], b + i * stride + 8, sizeof(float));
  HIP_TRY(hipStreamSynchronize(o->s));
  o->h_range = pin_range;
  o->h_ground = pin_ground;
  o->h_label = pin_label;
  o->hn = n;
  Labeller lb(p, o->h_range, o->z.data(), residual, o->h_label, T[11], o->avg, o->work);
  lb.run();
  ddlo_seg_result r{};
  r.segments = lb.label_count - 1;
  for (size_t i = 0; i < n; ++i) {
    r.ground_pixels += o->h_ground[i] == 1;
    r.range_pixels += o->h_range[i] > 0.f;
    r.rejected_pixels += o->h_label[i] == kRejected;
  }
  o->last = r;
  o->have = true;
  if (res) *res = r;
  return GICP_OK;
}

gicp_status ddlo_seg_images(ddlo_seg* o, float* range, int8_t* ground, int32_t* label) {
  if (!o) return fail(GICP_EINVAL, "null handle");
  if (!o->have) return fail(GICP_EINVAL, "no processed scan");
  const size_t n = o->hn;
  if (range) std::memcpy(range, o->h_range, sizeof(float) * n);
  if (ground) std::memcpy(ground, o->h_ground, n);
  if (label) std::memcpy(label, o->h_label, sizeof(int) * n);
  return GICP_OK;
}

gicp_status ddlo_seg_avg_residuals(ddlo_seg* o, double* out, size_t cap, size_t* n) {
  if (!o || (!out && cap)) return fail(GICP_EINVAL, "invalid argument");
  if (!o->have) return fail(GICP_EINVAL, "no processed scan");
  for (size_t l = 0; l < cap && l < o->avg.size(); ++l) out[l] = o->avg[l];
  if (n) *n = o->avg.size();
  return GICP_OK;
}

gicp_status ddlo_seg_ground_indices(ddlo_seg* o, int32_t* out, size_t cap, size_t* n) {
  if (!o || !n || (!out && cap)) return fail(GICP_EINVAL, "invalid argument");
  if (!o->have) return fail(GICP_EINVAL, "no processed scan");
  const int H = o->p.rows, W = o->p.cols;
  size_t k = 0;
  for (int col = 0; col < W; ++col)
    for (int ri = 0; ri < o->p.ground_rows; ++ri) {
      const int row = H - 1 - ri;
      if (o->h_ground[(size_t)row * W + col] == 1) {
        if (k < cap) out[k] = row * W + col;
        ++k;
      }
    }
  *n = k;
  return GICP_OK;
}

gicp_status ddlo_seg_label_indices(ddlo_seg* o, int32_t* offsets, size_t offsets_cap, int32_t* indices,
                                   size_t indices_cap, size_t* n_indices) {
  if (!o) return fail(GICP_EINVAL, "null handle");
  if (!o->have) return fail(GICP_EINVAL, "no processed scan");
  const int L = o->last.segments;
  if (offsets && offsets_cap < (size_t)L + 2) return fail(GICP_EINVAL, "offsets needs segments + 2 entries");
  std::vector<int32_t> cnt(L + 2, 0);
  const size_t n = o->hn;
  for (size_t i = 0; i < n; ++i) {
    const int l = o->h_label[i];
    if (l > 0 && l != kRejected) ++cnt[l + 1];
  }
  for (int l = 1; l <= L + 1; ++l) cnt[l] += cnt[l - 1];
  const size_t total = (size_t)cnt[L + 1];
  if (n_indices) *n_indices = total;
  if (offsets) std::memcpy(offsets, cnt.data(), sizeof(int32_t) * (L + 2));
  if (indices) {
    if (indices_cap < total) return fail(GICP_EINVAL, "indices buffer too small");
    std::vector<int32_t> pos(cnt.begin(), cnt.end() - 1);
    for (size_t i = 0; i < n; ++i) {   // row-major within a label, as :527-537
      const int l = o->h_label[i];
      if (l > 0 && l != kRejected) indices[pos[l]++] = (int32_t)i;
    }
  }
  return GICP_OK;
}

gicp_status ddlo_seg_label(const ddlo_seg_params* p, const float* range, const float* z, const float* residual,
                           float sensor_z, int32_t* label, double* avg_residual, size_t avg_cap, int32_t* segments) {
  if (gicp_status st = check_params(p)) return st;
  if (!range || !z || !label || (!avg_residual && avg_cap)) return fail(GICP_EINVAL, "invalid argument");
  std::vector<double> avg;
  LabelWork work;
  Labeller lb(*p, range, z, residual, label, sensor_z, avg, work);
  lb.run();
  for (size_t l = 0; l < avg_cap; ++l) avg_residual[l] = l < avg.size() ? avg[l] : 0.0;
  if (segments) *segments = lb.label_count - 1;
  return GICP_OK;
}

}  // extern "C"
