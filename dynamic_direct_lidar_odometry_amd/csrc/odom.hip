// odom.hip — odometry driver around the GICP core (include/ddlo_odom.h;
// SURVEY.md §8(f) rank 1, device voxel filter = rank 3).
//
// Restates the registration half of OdomNode (reference
// dynamic_direct_lidar_odometry/src/odometry/odom.cc) with every point set
// on the device:
//   icpCB                 :614-729   process()
//   preprocessPoints      :442-478   crop box + voxel filter (preprocess.hip)
//   computeSpaciousness   :981-1001  device ranges + sort, host low-pass
//   setAdaptiveParams     :1156-1178
//   initializeInputTarget :480-516
//   setInputSources       :518-532   one device cloud shared by S2S and S2M
//   scanMatching          :745-851   S2S, propagateS2S, cov reuse, swap,
//                                    getSubmapKeyframes, S2M, propagateS2M
//   transformScans        :941-947   device transform to the world frame
//   updateKeyframes       :1067-1154 keyframe decision; the keyframe cloud
//                                    (submap voxel filter) and its k-NN
//                                    covariances stay on the device
//   getSubmapKeyframes    :1215-1315 k nearest + convex-hull + concave-hull
//                                    keyframes; the submap cloud is the
//                                    device concatenation of the keyframes'
//                                    points and covariances (no host copies)
// Deliberate differences, all where the reference reads unsynchronised or
// out-of-range data: the spaciousness metric is computed before the
// adaptive threshold reads it (the reference starts it on a detached thread
// right before, :656-660) and over the scan's n points (its loop reads one
// past the end, :986).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <queue>
#include <vector>

#include "../../include/ddlo_gicp.h"
#include "../../include/ddlo_odom.h"
#include "gicp_types.hpp"
#include "launch.hpp"
#include "runtime.hpp"
#include "devknobs.hpp"

namespace {

using namespace ddlo;
using namespace ddlo::rt;

// ---- small host math (float like the reference's Matrix4f / Quaternionf) ----
void mat4_identity(float* T) {
  for (int i = 0; i < 16; ++i) T[i] = (i % 5 == 0) ? 1.f : 0.f;
}
void mat4_mul(const float* A, const float* B, float* C) {  // C = A * B, row-major
  float R[16];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c)
      R[4 * r + c] = ((A[4 * r] * B[c] + A[4 * r + 1] * B[4 + c]) + A[4 * r + 2] * B[8 + c]) + A[4 * r + 3] * B[12 + c];
  std::memcpy(C, R, sizeof(R));
}

struct Quatf {
  float x = 0.f, y = 0.f, z = 0.f, w = 1.f;
};

// Eigen::Quaternionf(const Matrix3f&) (quaternionbase_assign_impl), then the
// normalisation of propagateS2M (odom.cc:928-937: double norm, float /=)
Quatf quat_from_R(const float* T) {
  auto m = [&](int r, int c) { return T[4 * r + c]; };
  Quatf q;
  float t = m(0, 0) + m(1, 1) + m(2, 2);
  if (t > 0.f) {
    t = std::sqrt(t + 1.0f);
    q.w = 0.5f * t;
    t = 0.5f / t;
    q.x = (m(2, 1) - m(1, 2)) * t;
    q.y = (m(0, 2) - m(2, 0)) * t;
    q.z = (m(1, 0) - m(0, 1)) * t;
  } else {
    int i = 0;
    if (m(1, 1) > m(0, 0)) i = 1;
    if (m(2, 2) > m(i, i)) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(m(i, i) - m(j, j) - m(k, k) + 1.0f);
    float c[3];
    c[i] = 0.5f * t;
    t = 0.5f / t;
    q.w = (m(k, j) - m(j, k)) * t;
    c[j] = (m(j, i) + m(i, j)) * t;
    c[k] = (m(k, i) + m(i, k)) * t;
    q.x = c[0];
    q.y = c[1];
    q.z = c[2];
  }
  const double norm = std::sqrt(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
  q.w = (float)(q.w / norm);
  q.x = (float)(q.x / norm);
  q.y = (float)(q.y / norm);
  q.z = (float)(q.z / norm);
  return q;
}

Quatf quat_mul(const Quatf& a, const Quatf& b) {
  Quatf r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}
Quatf quat_inverse(const Quatf& q) {  // Eigen: conjugate / squaredNorm
  const float n2 = q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z;
  Quatf r;
  r.w = q.w / n2;
  r.x = -q.x / n2;
  r.y = -q.y / n2;
  r.z = -q.z / n2;
  return r;
}

// ---- hulls over the keyframe positions (computeConvexHull / computeConcaveHull) ----
// OdomNode sets both hulls to dimension 3 (odom.cc:87-88), so PCL never
// projects to a plane: pcl::ConvexHull runs qhull in 3-D ("qhull ", no
// joggle; a flat keyframe set is a qhull precision error and an EMPTY hull),
// pcl::ConcaveHull runs qhull's 3-D Delaunay ("qhull d QJ") and keeps the
// alpha shape's boundary triangles.  Both are restated here on the host (a
// few hundred keyframes at most), as the reference runs qhull on its host.
using P3 = std::array<double, 3>;

// vertex set of the 3-D convex hull; empty when the points are coplanar or
// fewer than 4 (qhull: "initial simplex is flat")
std::vector<int> convex_hull(const float* xyz, int n) {
  std::vector<int> out;
  if (n < 4) return out;
  struct F {
    int a, b, c;
    double n[3], d;
    bool alive;
  };
  auto P = [&](int i) { return P3{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]}; };
  auto make = [&](int a, int b, int cc) {
    const P3 A = P(a), B = P(b), Cc = P(cc);
    const double e1[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]}, e2[3] = {Cc[0] - A[0], Cc[1] - A[1], Cc[2] - A[2]};
    F f{a, b, cc, {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]}, 0, true};
    const double nn = std::sqrt(f.n[0] * f.n[0] + f.n[1] * f.n[1] + f.n[2] * f.n[2]);
    if (nn > 0)
      for (int k = 0; k < 3; ++k) f.n[k] /= nn;   // unit normal: the visibility test below is a distance
    f.d = f.n[0] * A[0] + f.n[1] * A[1] + f.n[2] * A[2];
    return f;
  };
  double scale = 0;
  for (int i = 0; i < 3 * n; ++i) scale = std::max(scale, (double)std::fabs(xyz[i]));
  scale = std::max(scale, 1e-30);
  const double eps = 1e-12 * scale;   // a point this close to a facet's plane does not see it (qhull: round-off)
  // initial tetrahedron: farthest-apart picks
  int i0 = 0, i1 = -1, i2 = -1, i3 = -1;
  double best = -1;
  for (int i = 1; i < n; ++i) {
    const P3 a = P(i0), b = P(i);
    const double d = (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
    if (d > best) { best = d; i1 = i; }
  }
  best = -1;
  for (int i = 0; i < n; ++i) {
    if (i == i0 || i == i1) continue;
    const P3 A = P(i0), B = P(i1), Cc = P(i);
    const double e1[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]}, e2[3] = {Cc[0] - A[0], Cc[1] - A[1], Cc[2] - A[2]};
    const double cx = e1[1] * e2[2] - e1[2] * e2[1], cy = e1[2] * e2[0] - e1[0] * e2[2], cz = e1[0] * e2[1] - e1[1] * e2[0];
    const double a2 = cx * cx + cy * cy + cz * cz;
    if (a2 > best) { best = a2; i2 = i; }
  }
  if (i2 < 0 || !(best > 0)) return out;   // collinear
  best = -1;
  const F base = make(i0, i1, i2);
  const double bn = 1.0;
  for (int i = 0; i < n; ++i) {
    if (i == i0 || i == i1 || i == i2) continue;
    const P3 p = P(i);
    const double sd = std::fabs(base.n[0] * p[0] + base.n[1] * p[1] + base.n[2] * p[2] - base.d);
    if (sd > best) { best = sd; i3 = i; }
  }
  // qhull's flat-simplex test is at round-off level: coplanar within ~1e-13 of the extent
  if (!(bn > 0) || i3 < 0 || best / bn <= 1e-13 * scale) return out;
  std::vector<F> fs;
  auto add_oriented = [&](int a, int b, int cc, int inside) {
    F f = make(a, b, cc);
    const P3 q = P(inside);
    if (f.n[0] * q[0] + f.n[1] * q[1] + f.n[2] * q[2] - f.d > 0) f = make(a, cc, b);
    fs.push_back(f);
  };
  add_oriented(i0, i1, i2, i3);
  add_oriented(i0, i1, i3, i2);
  add_oriented(i0, i2, i3, i1);
  add_oriented(i1, i2, i3, i0);
  for (int i = 0; i < n; ++i) {
    if (i == i0 || i == i1 || i == i2 || i == i3) continue;
    const P3 p = P(i);
    std::vector<std::pair<int, int>> edges;
    bool any = false;
    for (auto& f : fs) {
      if (!f.alive) continue;
      if (f.n[0] * p[0] + f.n[1] * p[1] + f.n[2] * p[2] - f.d > eps) {
        f.alive = false;
        any = true;
        edges.push_back({f.a, f.b});
        edges.push_back({f.b, f.c});
        edges.push_back({f.c, f.a});
      }
    }
    if (!any) continue;
    // horizon: directed edges whose reverse was not removed
    for (const auto& e : edges) {
      bool twin = false;
      for (const auto& g : edges)
        if (g.first == e.second && g.second == e.first) { twin = true; break; }
      if (!twin) fs.push_back(make(e.first, e.second, i));
    }
  }
  std::vector<char> on(n, 0);
  for (const auto& f : fs)
    if (f.alive) on[f.a] = on[f.b] = on[f.c] = 1;
  for (int i = 0; i < n; ++i)
    if (on[i]) out.push_back(i);
  return out;
}

// ---- 3-D Delaunay (Bowyer-Watson, long double predicates) ----
using LD = long double;
struct Tet {
  int v[4];
  bool alive;
};

LD det3(LD a, LD b, LD c, LD d, LD e, LD f, LD g, LD h, LD i) { return a * (e * i - f * h) - b * (d * i - f * g) + c * (d * h - e * g); }

// det[b - a; c - a; d - a]
LD orient(const std::vector<std::array<LD, 3>>& p, int a, int b, int c, int d) {
  const auto& A = p[a];
  const auto& B = p[b];
  const auto& C = p[c];
  const auto& D = p[d];
  return det3(B[0] - A[0], B[1] - A[1], B[2] - A[2], C[0] - A[0], C[1] - A[1], C[2] - A[2], D[0] - A[0], D[1] - A[1],
              D[2] - A[2]);
}

// 4x4 lifted determinant; for a positively oriented tetrahedron its sign
// tells whether e lies inside the circumsphere (kInside below)
LD insphere(const std::vector<std::array<LD, 3>>& p, const int* t, int e) {
  LD m[4][4];
  for (int r = 0; r < 4; ++r) {
    const auto& A = p[t[r]];
    const LD x = A[0] - p[e][0], y = A[1] - p[e][1], z = A[2] - p[e][2];
    m[r][0] = x;
    m[r][1] = y;
    m[r][2] = z;
    m[r][3] = x * x + y * y + z * z;
  }
  LD d = 0;
  for (int c = 0; c < 4; ++c) {
    LD sub[9];
    int k = 0;
    for (int r = 1; r < 4; ++r)
      for (int cc = 0; cc < 4; ++cc)
        if (cc != c) sub[k++] = m[r][cc];
    const LD cof = det3(sub[0], sub[1], sub[2], sub[3], sub[4], sub[5], sub[6], sub[7], sub[8]);
    d += ((c & 1) ? -1 : 1) * m[0][c] * cof;
  }
  return d;
}

int inside_sign() {   // the sign insphere() has at the centre of a positive unit tetrahedron
  static const int s = [] {
    std::vector<std::array<LD, 3>> p = {{0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0.25L, 0.25L, 0.25L}};
    const int t[4] = {0, 1, 2, 3};
    return insphere(p, t, 4) > 0 ? 1 : -1;
  }();
  return s;
}

// Delaunay tetrahedra of the points (indices into xyz), the enclosing
// tetrahedron's removed.  Input coordinates are demeaned (PCL demeans before
// qhull) and joggled by a deterministic relative 1e-11 (qhull's QJ joggles
// randomly) so that cospherical / coplanar input has a well-defined answer.
std::vector<Tet> delaunay3(const float* xyz, int n, std::vector<std::array<LD, 3>>& p) {
  std::array<LD, 3> c{0, 0, 0};
  for (int i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a) c[a] += xyz[3 * i + a];
  for (int a = 0; a < 3; ++a) c[a] /= n;
  LD ext = 0;
  p.assign(n + 4, {0, 0, 0});
  uint64_t rng = 0x9E3779B97F4A7C15ull;
  auto next = [&]() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (LD)((rng >> 11) * (1.0 / 9007199254740992.0)) - 0.5L;
  };
  for (int i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a) {
      p[i][a] = (LD)xyz[3 * i + a] - c[a];
      ext = std::max(ext, std::fabs(p[i][a]));
    }
  ext = std::max(ext, (LD)1e-12);
  for (int i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a) p[i][a] += next() * 1e-11L * ext;
  const LD M = 1e4L * ext;
  p[n] = {-M, -M, -M};
  p[n + 1] = {3 * M, -M, -M};
  p[n + 2] = {-M, 3 * M, -M};
  p[n + 3] = {-M, -M, 3 * M};
  std::vector<Tet> T;
  T.push_back({{n, n + 1, n + 2, n + 3}, true});
  if (orient(p, n, n + 1, n + 2, n + 3) < 0) std::swap(T[0].v[2], T[0].v[3]);
  const int ins = inside_sign();
  for (int i = 0; i < n; ++i) {
    std::vector<int> bad;
    for (int t = 0; t < (int)T.size(); ++t)
      if (T[t].alive && insphere(p, T[t].v, i) * ins > 0) bad.push_back(t);
    // cavity boundary: faces of exactly one bad tetrahedron
    std::map<std::array<int, 3>, std::pair<int, std::array<int, 3>>> faces;
    for (int t : bad) {
      T[t].alive = false;
      const int* v = T[t].v;
      const int fidx[4][3] = {{1, 2, 3}, {0, 3, 2}, {0, 1, 3}, {0, 2, 1}};
      for (const auto& f : fidx) {
        std::array<int, 3> o{v[f[0]], v[f[1]], v[f[2]]};
        std::array<int, 3> k = o;
        std::sort(k.begin(), k.end());
        auto it = faces.find(k);
        if (it == faces.end()) faces[k] = {1, o};
        else it->second.first += 1;
      }
    }
    for (const auto& kv : faces) {
      if (kv.second.first != 1) continue;
      const auto& o = kv.second.second;
      Tet nt{{o[0], o[1], o[2], i}, true};
      const LD ov = orient(p, nt.v[0], nt.v[1], nt.v[2], nt.v[3]);
      if (ov == 0) continue;   // degenerate after joggle: drop (never seen)
      if (ov < 0) std::swap(nt.v[0], nt.v[1]);
      T.push_back(nt);
    }
  }
  std::vector<Tet> out;
  for (const auto& t : T)
    if (t.alive && t.v[0] < n && t.v[1] < n && t.v[2] < n && t.v[3] < n) out.push_back(t);
  return out;
}

// circumradius of a tetrahedron (qh_pointdist(vertex, facet->center))
LD tet_radius(const std::vector<std::array<LD, 3>>& p, const Tet& t) {
  const auto& A = p[t.v[0]];
  LD r[3][3], rhs[3];
  for (int k = 0; k < 3; ++k) {
    const auto& B = p[t.v[k + 1]];
    for (int a = 0; a < 3; ++a) r[k][a] = B[a] - A[a];
    rhs[k] = 0.5L * (r[k][0] * r[k][0] + r[k][1] * r[k][1] + r[k][2] * r[k][2]);
  }
  const LD D = det3(r[0][0], r[0][1], r[0][2], r[1][0], r[1][1], r[1][2], r[2][0], r[2][1], r[2][2]);
  if (D == 0) return INFINITY;
  const LD x = det3(rhs[0], r[0][1], r[0][2], rhs[1], r[1][1], r[1][2], rhs[2], r[2][1], r[2][2]) / D;
  const LD y = det3(r[0][0], rhs[0], r[0][2], r[1][0], rhs[1], r[1][2], r[2][0], rhs[2], r[2][2]) / D;
  const LD z = det3(r[0][0], r[0][1], rhs[0], r[1][0], r[1][1], rhs[1], r[2][0], r[2][1], rhs[2]) / D;
  return std::sqrt(x * x + y * y + z * z);
}

// pcl::getCircumcircleRadius (common/impl/common.hpp) of a ridge, whose
// vertices PCL reads as floats of qhull's (demeaned) coordinates: float
// Vector4f norms (Eigen's SSE redux: (x^2 + z^2) + y^2), Heron's formula in double
double tri_radius(const std::vector<std::array<LD, 3>>& p, int a, int b, int c) {
  auto nrm = [&](int i, int j) {
    const float dx = (float)p[j][0] - (float)p[i][0], dy = (float)p[j][1] - (float)p[i][1],
                dz = (float)p[j][2] - (float)p[i][2];
    return (double)std::sqrt((dx * dx + dz * dz) + dy * dy);
  };
  const double p2p1 = nrm(a, b), p3p2 = nrm(b, c), p1p3 = nrm(c, a);
  const double s = (p2p1 + p3p2 + p1p3) / 2.0;
  const double area = std::sqrt(s * (s - p2p1) * (s - p3p2) * (s - p1p3));
  return (p2p1 * p3p2 * p1p3) / (4.0 * area);
}

// Vertex set of pcl::ConcaveHull's 3-D alpha shape (PCL 1.10
// concave_hull.hpp performReconstruction, dim 3): a tetrahedron is "good"
// iff its circumradius <= alpha; a Delaunay triangle is output iff it has a
// side that is not a good tetrahedron (the outside, or a bad one) and its
// circumradius <= alpha (a good tetrahedron's triangles always are);
// setKeepInformation maps the vertices back to input indices.
std::vector<int> concave_hull(const float* xyz, int n, double alpha) {
  std::vector<int> out;
  if (n < 4) return out;
  std::vector<std::array<LD, 3>> p;
  const std::vector<Tet> T = delaunay3(xyz, n, p);
  std::vector<char> good(T.size());
  std::map<std::array<int, 3>, std::array<int, 2>> adj;   // triangle -> its tetrahedra (-1 = outside)
  for (size_t t = 0; t < T.size(); ++t) {
    good[t] = tet_radius(p, T[t]) <= (LD)alpha;
    const int* v = T[t].v;
    const int fidx[4][3] = {{1, 2, 3}, {0, 3, 2}, {0, 1, 3}, {0, 2, 1}};
    for (const auto& f : fidx) {
      std::array<int, 3> k{v[f[0]], v[f[1]], v[f[2]]};
      std::sort(k.begin(), k.end());
      auto it = adj.find(k);
      if (it == adj.end()) adj[k] = {(int)t, -1};
      else it->second[1] = (int)t;
    }
  }
  std::vector<char> on(n, 0);
  for (const auto& kv : adj) {
    const int a = kv.second[0], b = kv.second[1];
    const bool ga = good[a], gb = b >= 0 && good[b];
    if (ga && gb) continue;   // inside the good union
    const auto& f = kv.first;
    if (ga || gb || tri_radius(p, f[0], f[1], f[2]) <= alpha) on[f[0]] = on[f[1]] = on[f[2]] = 1;
  }
  for (int i = 0; i < n; ++i)
    if (on[i]) out.push_back(i);
  return out;
}

// OdomNode::pushSubmapIndices (odom.cc:1180-1213): the k smallest distances
// (max-heap of at most k), then every frame at or below the k-th
void push_submap_indices(const std::vector<float>& dists, int k, const std::vector<int>& frames, std::vector<int>& out) {
  if (dists.empty()) return;
  std::priority_queue<float> pq;
  for (float d : dists) {
    if ((int)pq.size() >= k && pq.top() > d) {
      pq.push(d);
      pq.pop();
    } else if ((int)pq.size() < k) {
      pq.push(d);
    }
  }
  const float kth = pq.top();
  for (size_t i = 0; i < dists.size(); ++i)
    if (dists[i] <= kth) out.push_back(frames[i]);
}

}  // namespace

// ---------------------------------------------------------------------------
struct Keyframe {
  float pose[3];
  Quatf q;
  int n = 0;
  DevBuf pts;   // float4, world frame, original order (after the submap voxel filter)
  DevBuf cov;   // sym6 doubles, original order
};

struct ddlo_odom {
  int device = 0;
  ddlo_odom_params p{};
  gicp_ctx* s2s = nullptr;
  gicp_ctx* s2m = nullptr;
  hipStream_t s = nullptr;
  // scratch (device)
  DevBuf up, a, b, keep, pos, vscratch, cubtmp, medtmp, rng, rng_sorted, cat_pts, cat_cov;
  // pinned host memory: [0] the median range of the current scan, [4..19] the
  // voxel / crop count read-back (int)
  float* median_pin = nullptr;
  int* count_pin = nullptr;
  // the median range runs on the S2M stream (it is read after the S2S align),
  // beside the scan's index build: med_in = the voxel output is ready, med_done
  hipEvent_t med_in = nullptr, med_done = nullptr;
  // DDLO_ODOM_TIMING=1: host wall time per phase, printed at destroy (development)
  bool timing = false;
  double t_phase[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};   // [8] device drain before a frame, [9] H2D call
  long frames = 0;
  // state
  bool initialized = false;   // ddlo_initialized_
  bool have_target = false;
  float T[16], T_s2s[16], T_s2s_prev[16];
  float pose[3] = {0.f, 0.f, 0.f};
  Quatf rotq;
  std::vector<std::unique_ptr<Keyframe>> keyframes;
  std::vector<int> submap_prev, keyframe_convex, keyframe_concave;
  // the hulls are functions of the keyframe positions (append-only, never
  // moved) and, for the concave one, alpha: recomputed only when a keyframe
  // was added or alpha changed (the reference reruns qhull every scan; the
  // 3-D Delaunay of the concave hull costs ~0.1-0.6 ms of host time)
  int convex_nk = -1, concave_nk = -1;
  double concave_alpha = -1.0;
  bool have_median = false;
  float median_prev = 0.f;
  double thresh_dist = 1.0;
  int64_t submap_points = 0;
};

namespace {

gicp_status ensure_tmp(ddlo_odom* o, int n) {
  const size_t t = std::max(crop_box_tmp_bytes(n), voxel_tmp_bytes(n));
  HIP_TRY(o->cubtmp.ensure(t));
  HIP_TRY(o->medtmp.ensure(median_tmp_bytes(n)));
  return GICP_OK;
}

// crop box + voxel filter of the float4 points in o->a (n) -> o->a; returns count
gicp_status preprocess(ddlo_odom* o, int n, bool crop, double crop_size, bool vox, double leaf, int* nout) {
  HIP_TRY(o->b.ensure(sizeof(float4) * (size_t)std::max(n, 1)));
  HIP_TRY(o->keep.ensure(sizeof(int) * (size_t)std::max(n, 1)));
  HIP_TRY(o->pos.ensure(sizeof(int) * (size_t)std::max(n, 1)));
  HIP_TRY(o->vscratch.ensure(sizeof(int) * voxel_scratch_ints(std::max(n, 1))));
  gicp_status st = ensure_tmp(o, std::max(n, 1));
  if (st) return st;
  int m = n;
  if (crop && vox && m > 0) {
    // one pass: the voxel filter over the points the crop box keeps (their
    // bbox, their input order), one count read-back instead of two
    int c = 0;
    if (voxel_grid(o->s, o->a.as<float4>(), m, (float)leaf, o->b.as<float4>(), o->vscratch.as<int>(), o->cubtmp.p,
                   o->cubtmp.bytes, &c, (float)crop_size, o->count_pin))
      return fail(GICP_EHIP, "voxel filter scratch too small");
    if (c >= 0) {
      *nout = c;
      std::swap(o->a.p, o->b.p);
      std::swap(o->a.bytes, o->b.bytes);
      HIP_TRY(hipGetLastError());
      return GICP_OK;
    }
    // grid overflow: the reference keeps the cropped cloud unchanged -> crop alone below
    vox = false;
  }
  if (crop && m > 0) {
    if (crop_box(o->s, o->a.as<float4>(), m, (float)crop_size, o->b.as<float4>(), o->keep.as<int>(), o->pos.as<int>(),
                 o->cubtmp.p, o->cubtmp.bytes, &m, o->count_pin))
      return fail(GICP_EHIP, "crop box scratch too small");
    std::swap(o->a.p, o->b.p);
    std::swap(o->a.bytes, o->b.bytes);
  }
  if (vox && m > 0) {
    int c = 0;
    if (voxel_grid(o->s, o->a.as<float4>(), m, (float)leaf, o->b.as<float4>(), o->vscratch.as<int>(), o->cubtmp.p,
                   o->cubtmp.bytes, &c, 0.f, o->count_pin))
      return fail(GICP_EHIP, "voxel filter scratch too small");
    if (c >= 0) {  // -1: grid overflow, the reference keeps the cloud unchanged
      m = c;
      std::swap(o->a.p, o->b.p);
      std::swap(o->a.bytes, o->b.bytes);
    }
  }
  HIP_TRY(hipGetLastError());
  *nout = m;
  return GICP_OK;
}

// device cloud from float4 points; `finite`: the points are known finite (a
// voxel filter's output, keyframes, the submap), no read-back of the check
// with_cov: covariances follow (the scan, a keyframe), so nanoflann's tree
// for their tie order starts with the index build (not for the submap,
// whose covariances are the keyframes')
gicp_status cloud_from(ddlo_odom* o, gicp_ctx* c, const float4* pts, int n, std::shared_ptr<CloudData>* out,
                       bool finite, bool with_cov) {
  (void)o;
  return build_cloud(c, reinterpret_cast<const float*>(pts), (size_t)n, sizeof(float4), out, true, !finite, with_cov);
}

// keyframe = world-frame copy of the (preprocessed) scan cloud, submap voxel
// filter, k-NN covariances with the S2S parameters (odom.cc:1129-1149)
gicp_status make_keyframe(ddlo_odom* o, const std::shared_ptr<CloudData>& scan) {
  auto kf = std::make_unique<Keyframe>();
  kf->pose[0] = o->pose[0];
  kf->pose[1] = o->pose[1];
  kf->pose[2] = o->pose[2];
  kf->q = o->rotq;
  const int n = scan->n;
  HIP_TRY(o->a.ensure(sizeof(float4) * (size_t)n));
  launch_transform4(o->s, scan->pts.as<float4>(), scan->perm.as<int>(), n, o->T, o->a.as<float4>());
  int m = n;
  gicp_status st = preprocess(o, n, false, 0.0, o->p.vf_submap_use != 0, o->p.vf_submap_res, &m);
  if (st) return st;
  if (m < 1) return fail(GICP_ETOOFEW, "keyframe without points");
  kf->n = m;
  HIP_TRY(kf->pts.ensure(sizeof(float4) * (size_t)m));
  HIP_TRY(hipMemcpyAsync(kf->pts.p, o->a.p, sizeof(float4) * (size_t)m, hipMemcpyDeviceToDevice, o->s));
  Side side;
  st = cloud_from(o, o->s2s, kf->pts.as<float4>(), m, &side.cloud, true, true);
  if (st) return st;
  // s2s->params: the S2S k (gicp_s2s_.calculateSourceCovariances); a
  // keyframe smaller than k uses all of its points (the reference reads
  // uninitialised neighbour slots there)
  st = compute_cov(o->s2s, side, std::min(o->p.s2s.k_correspondences, m));
  if (st) return st;
  HIP_TRY(kf->cov.ensure(sizeof(double) * 6 * (size_t)m));
  launch_gather_cov6(o->s, side.cov->cov6.as<double>(), side.cloud->perm.as<int>(), m, kf->cov.as<double>());
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(o->s));
  st = check_ties(o->s2s);   // the keyframe's (and the first scan's) covariance tie resolution
  if (st) return st;
  o->keyframes.push_back(std::move(kf));
  return GICP_OK;
}

// OdomNode::getSubmapKeyframes (odom.cc:1215-1315); returns whether it changed
gicp_status submap_keyframes(ddlo_odom* o, bool* changed) {
  const int nk = (int)o->keyframes.size();
  std::vector<int> cur;
  std::vector<float> ds;
  std::vector<int> nn;
  const float cx = o->T_s2s[3], cy = o->T_s2s[7], cz = o->T_s2s[11];
  for (int i = 0; i < nk; ++i) {
    const float* k = o->keyframes[i]->pose;
    ds.push_back((float)std::sqrt(std::pow(cx - k[0], 2) + std::pow(cy - k[1], 2) + std::pow(cz - k[2], 2)));
    nn.push_back(i);
  }
  push_submap_indices(ds, o->p.submap_knn, nn, cur);
  std::vector<float> kpos(3 * (size_t)nk);
  for (int i = 0; i < nk; ++i)
    for (int a = 0; a < 3; ++a) kpos[3 * i + a] = o->keyframes[i]->pose[a];
  if (nk >= 4 && nk != o->convex_nk) {   // computeConvexHull: >= 4 keyframes
    o->keyframe_convex = convex_hull(kpos.data(), nk);
    o->convex_nk = nk;
  }
  std::vector<float> cds;
  for (int c : o->keyframe_convex) cds.push_back(ds[c]);
  push_submap_indices(cds, o->p.submap_kcv, o->keyframe_convex, cur);
  if (nk >= 5 && (nk != o->concave_nk || o->thresh_dist != o->concave_alpha)) {   // >= 5 keyframes
    o->keyframe_concave = concave_hull(kpos.data(), nk, o->thresh_dist);
    o->concave_nk = nk;
    o->concave_alpha = o->thresh_dist;
  }
  std::vector<float> kds;
  for (int c : o->keyframe_concave) kds.push_back(ds[c]);
  push_submap_indices(kds, o->p.submap_kcc, o->keyframe_concave, cur);
  std::sort(cur.begin(), cur.end());
  cur.erase(std::unique(cur.begin(), cur.end()), cur.end());
  *changed = cur != o->submap_prev;
  if (!*changed) return GICP_OK;
  // submap cloud + normals: the selected keyframes concatenated in index
  // order, all on the device
  int64_t total = 0;
  for (int k : cur) total += o->keyframes[k]->n;
  if (total > INT32_MAX / 2) return fail(GICP_EINVAL, "submap too large");
  HIP_TRY(o->cat_pts.ensure(sizeof(float4) * (size_t)total));
  HIP_TRY(o->cat_cov.ensure(sizeof(double) * 6 * (size_t)total));
  // everything of the submap build runs on the S2M context's stream: the
  // concatenation, its index (build_cloud) and the covariance import
  hipStream_t sm = o->s2m->stream;
  int64_t off = 0;
  for (int k : cur) {
    const Keyframe& kf = *o->keyframes[k];
    HIP_TRY(hipMemcpyAsync(o->cat_pts.as<float4>() + off, kf.pts.p, sizeof(float4) * kf.n, hipMemcpyDeviceToDevice, sm));
    HIP_TRY(hipMemcpyAsync(o->cat_cov.as<double>() + 6 * off, kf.cov.p, sizeof(double) * 6 * kf.n,
                           hipMemcpyDeviceToDevice, sm));
    off += kf.n;
  }
  Side tgt;
  gicp_status st = cloud_from(o, o->s2m, o->cat_pts.as<float4>(), (int)total, &tgt.cloud, true, false);
  if (st) return st;
  auto cv = std::make_shared<CovData>();
  cv->n = (int)total;
  HIP_TRY(cv->cov6.ensure(sizeof(double) * 6 * (size_t)total));
  launch_cov_import(sm, o->cat_cov.as<double>(), GICP_COV_SYM6, (int)total, tgt.cloud->inv_perm.as<int>(),
                    cv->cov6.as<double>());
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(sm));
  tgt.cov = cv;
  o->s2m->tgt = tgt;        // setInputTarget + setTargetCovariances (odom.cc:780-783)
  invalidate_align(o->s2m);
  o->submap_prev = cur;
  o->submap_points = total;
  return GICP_OK;
}

void copy_pose(const float* T, float* out) { std::memcpy(out, T, sizeof(float) * 16); }

}  // namespace

extern "C" {

gicp_status ddlo_odom_default_params(ddlo_odom_params* p) {
  if (!p) return fail(GICP_EINVAL, "null params");
  std::memset(p, 0, sizeof(*p));
  gicp_default_params(&p->s2s);
  gicp_default_params(&p->s2m);
  // cfg/ddlo.yaml:185-204
  p->s2s.k_correspondences = 10;
  p->s2s.max_correspondence_distance = 1.0;
  p->s2s.max_iterations = 32;
  p->s2s.transformation_epsilon = 0.01;
  p->s2m.k_correspondences = 20;
  p->s2m.max_correspondence_distance = 2.0;
  p->s2m.max_iterations = 32;
  p->s2m.transformation_epsilon = 0.01;
  p->min_num_points = 10;
  p->keyframe_thresh_dist = 1.0;
  p->keyframe_thresh_rot = 0.1;
  p->submap_knn = p->submap_kcv = p->submap_kcc = 10;
  p->adaptive = 1;
  p->crop_use = 1;
  p->crop_size = 1.0;
  p->vf_scan_use = 1;
  p->vf_scan_res = 0.1;
  p->vf_submap_use = 1;
  p->vf_submap_res = 0.1;
  p->skip_first_scan = 1;
  p->s2m_target_grid = GICP_GRID_OFF;
  return GICP_OK;
}

gicp_status ddlo_odom_create(int device, const ddlo_odom_params* p, ddlo_odom** out) {
  if (!out) return fail(GICP_EINVAL, "null out");
  *out = nullptr;
  auto o = std::make_unique<ddlo_odom>();
  if (p) {
    o->p = *p;
  } else {
    ddlo_odom_default_params(&o->p);
  }
  if (o->p.submap_knn < 1 || o->p.submap_kcv < 1 || o->p.submap_kcc < 1) return fail(GICP_EINVAL, "submap k must be >= 1");
  if ((o->p.vf_scan_use && !(o->p.vf_scan_res > 0)) || (o->p.vf_submap_use && !(o->p.vf_submap_res > 0)))
    return fail(GICP_EINVAL, "voxel resolution must be positive");
  o->device = device;
  gicp_status st = gicp_ctx_create(device, &o->s2s);
  if (!st) st = gicp_ctx_create(device, &o->s2m);
  if (!st) st = gicp_set_params(o->s2s, &o->p.s2s);
  if (!st) st = gicp_set_params(o->s2m, &o->p.s2m);
  if (!st) st = gicp_set_target_grid(o->s2m, o->p.s2m_target_grid);
  if (!st) st = gicp_set_target_grid(o->s2s, GICP_GRID_OFF);   // S2S targets live one scan
  if (st) {
    if (o->s2s) gicp_ctx_destroy(o->s2s);
    if (o->s2m) gicp_ctx_destroy(o->s2m);
    return st;
  }
  o->s = o->s2s->stream;  // one stream: the driver's work is one dependent chain
  o->timing = dev_getenv("DDLO_ODOM_TIMING") != nullptr;
  if (hipHostMalloc((void**)&o->median_pin, sizeof(float) * 20, hipHostMallocDefault) != hipSuccess ||
      hipEventCreateWithFlags(&o->med_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&o->med_done, hipEventDisableTiming) != hipSuccess) {
    if (o->median_pin) (void)hipHostFree(o->median_pin);
    if (o->med_in) (void)hipEventDestroy(o->med_in);
    gicp_ctx_destroy(o->s2s);
    gicp_ctx_destroy(o->s2m);
    return fail(GICP_EHIP, "pinned allocation failed");
  }
  *o->median_pin = 0.f;
  o->count_pin = reinterpret_cast<int*>(o->median_pin + 4);
  mat4_identity(o->T);
  mat4_identity(o->T_s2s);
  mat4_identity(o->T_s2s_prev);
  o->thresh_dist = o->p.keyframe_thresh_dist;
  *out = o.release();
  return GICP_OK;
}

gicp_status ddlo_odom_destroy(ddlo_odom* o) {
  if (!o) return GICP_OK;
  (void)hipSetDevice(o->device);
  (void)hipStreamSynchronize(o->s2m->stream);
  (void)hipStreamSynchronize(o->s);
  if (o->timing && o->frames > 0) {
    static const char* names[10] = {"upload", "preprocess", "cloud", "s2s_align", "submap", "s2m_align", "keyframe",
                                    "total", "drain_before", "h2d_call"};
    std::fprintf(stderr, "[odom timing] %ld frames, us/frame:", o->frames);
    for (int k = 0; k < 10; ++k) std::fprintf(stderr, " %s %.1f", names[k], 1e6 * o->t_phase[k] / o->frames);
    std::fprintf(stderr, "\n");
  }
  o->keyframes.clear();
  if (o->median_pin) (void)hipHostFree(o->median_pin);
  if (o->med_in) (void)hipEventDestroy(o->med_in);
  if (o->med_done) (void)hipEventDestroy(o->med_done);
  gicp_ctx_destroy(o->s2m);
  gicp_ctx_destroy(o->s2s);
  delete o;
  return GICP_OK;
}

gicp_status ddlo_odom_process(ddlo_odom* o, const float* xyz, size_t n, size_t stride, ddlo_odom_result* res) {
  if (!o || !res || (!xyz && n) || stride < 12 || stride % 4) return fail(GICP_EINVAL, "invalid argument");
  if (n > (size_t)INT32_MAX / 2) return fail(GICP_EINVAL, "scan too large");
  gicp_status st = set_device(o->s2s);
  if (st) return st;
  begin_ties(o->s2s);
  begin_ties(o->s2m);
  std::memset(res, 0, sizeof(*res));
  copy_pose(o->T, res->T);
  copy_pose(o->T_s2s, res->T_s2s);
  mat4_identity(res->T_s2s_local);
  res->num_keyframes = (int)o->keyframes.size();
  // icpCB: too few points -> return (odom.cc:635-639)
  if ((int64_t)n < o->p.min_num_points) {
    res->status = DDLO_ODOM_SKIPPED;
    return GICP_OK;
  }
  // DLO initialisation consumes the first valid scan (odom.cc:641-646;
  // gravity alignment is out of scope, so it only sets ddlo_initialized_)
  if (!o->initialized) {
    o->initialized = true;
    if (o->p.skip_first_scan) {
      res->status = DDLO_ODOM_INIT;
      return GICP_OK;
    }
  }
  using clk = std::chrono::steady_clock;
  if (o->timing) {   // work of the previous frame still queued on any stream (aux included)
    const auto td = clk::now();
    (void)hipDeviceSynchronize();
    o->t_phase[8] += std::chrono::duration<double>(clk::now() - td).count();
  }
  auto t0 = clk::now(), tl = t0;
  auto mark = [&](int k) {
    if (!o->timing) return;
    (void)hipStreamSynchronize(o->s);
    (void)hipStreamSynchronize(o->s2m->stream);
    const auto t = clk::now();
    o->t_phase[k] += std::chrono::duration<double>(t - tl).count();
    tl = t;
  };
  // upload + preprocessPoints (odom.cc:442-478)
  const int N = (int)n;
  HIP_TRY(o->up.ensure((n - 1) * stride + 12));
  HIP_TRY(hipMemcpyAsync(o->up.p, xyz, (n - 1) * stride + 12, hipMemcpyHostToDevice, o->s));
  if (o->timing) o->t_phase[9] += std::chrono::duration<double>(clk::now() - t0).count();
  HIP_TRY(o->a.ensure(sizeof(float4) * n));
  launch_pack4(o->s, o->up.as<unsigned char>(), stride, N, o->a.as<float4>());
  mark(0);
  int m = N;
  st = preprocess(o, N, o->p.crop_use != 0, o->p.crop_size, o->p.vf_scan_use != 0, o->p.vf_scan_res, &m);
  if (st) return st;
  res->scan_points = m;
  mark(1);
  // computeSpaciousness (odom.cc:981-1001): the median range is selected on
  // the device and copied to pinned memory, on the S2M context's stream (idle
  // until the submap build) beside the scan's index build and the S2S align;
  // metrics() waits for it (nothing before scan matching uses it).  The scan
  // (o->a) is not written again before that wait.
  HIP_TRY(o->rng.ensure(sizeof(float) * (size_t)std::max(m, 1)));
  HIP_TRY(o->rng_sorted.ensure(sizeof(float) * (size_t)std::max(m, 1)));
  {
    hipStream_t sm = o->s2m->stream;
    HIP_TRY(hipEventRecord(o->med_in, o->s));
    HIP_TRY(hipStreamWaitEvent(sm, o->med_in, 0));
    if (m > 0)
      median_range_async(sm, o->a.as<float4>(), m, o->rng.as<float>(), o->rng_sorted.as<float>(), o->medtmp.p,
                         o->medtmp.bytes, o->median_pin);
    else
      *o->median_pin = 0.f;
    HIP_TRY(hipEventRecord(o->med_done, sm));
  }
  // computeMetrics + setAdaptiveParams (odom.cc:981-1001, 1156-1178), once
  // the median has arrived
  auto metrics = [&]() {
    (void)hipEventSynchronize(o->med_done);
    const float median_curr = *o->median_pin;
    if (!o->have_median) {  // static float median_prev = median_curr (first call)
      o->median_prev = median_curr;
      o->have_median = true;
    }
    const float median_lpf = (float)(0.95 * o->median_prev + 0.05 * median_curr);
    o->median_prev = median_lpf;
    res->spaciousness = median_lpf;
    if (o->p.adaptive) {
      if (median_lpf > 20.0) o->thresh_dist = 10.0;
      else if (median_lpf > 10.0 && median_lpf <= 20.0) o->thresh_dist = 5.0;
      else if (median_lpf > 5.0 && median_lpf <= 10.0) o->thresh_dist = 1.0;
      else if (median_lpf <= 5.0) o->thresh_dist = 0.5;
    }
    res->keyframe_thresh_dist = o->thresh_dist;
  };
  if (m < std::max(o->p.s2s.k_correspondences, o->p.s2m.k_correspondences)) {
    HIP_TRY(hipStreamSynchronize(o->s));
    metrics();
    return fail(GICP_ETOOFEW, "preprocessed scan has fewer points than k_correspondences");
  }
  // the preprocessed scan as a device cloud (finite after the voxel filter)
  std::shared_ptr<CloudData> scan;
  st = cloud_from(o, o->s2s, o->a.as<float4>(), m, &scan, o->p.vf_scan_use != 0, true);
  if (st) return st;
  mark(2);

  if (!o->have_target) {
    // initializeInputTarget (odom.cc:480-516)
    o->s2s->tgt = Side();
    o->s2s->tgt.cloud = scan;
    invalidate_align(o->s2s);
    st = compute_cov(o->s2s, o->s2s->tgt);   // calculateTargetCovariances
    if (st) return st;
    st = make_keyframe(o, scan);              // T_ = identity: the scan itself (waits for the stream)
    if (st) return st;
    metrics();
    o->have_target = true;
    res->status = DDLO_ODOM_FIRST;
    res->keyframe_added = 1;
    res->num_keyframes = (int)o->keyframes.size();
    return GICP_OK;
  }
  // setInputSources (odom.cc:518-532): one device cloud for both
  o->s2s->src = Side();
  o->s2s->src.cloud = scan;
  invalidate_align(o->s2s);
  o->s2m->src = Side();
  o->s2m->src.cloud = scan;
  invalidate_align(o->s2m);

  // scanMatching (odom.cc:745-851)
  float T_S2S[16];
  st = gicp_align(o->s2s, nullptr, T_S2S, &res->s2s);   // waits for the stream: the median has arrived
  if (st) return st;
  mark(3);
  metrics();
  copy_pose(T_S2S, res->T_s2s_local);
  mat4_mul(o->T_s2s_prev, T_S2S, o->T_s2s);   // propagateS2S
  copy_pose(o->T_s2s, o->T_s2s_prev);
  o->s2m->src.cov = o->s2s->src.cov;          // gicp_s2m_.source_covs_ = gicp_s2s_.source_covs_
  gicp_swap_source_target(o->s2s);            // the scan becomes the next S2S target
  bool changed = false;
  st = submap_keyframes(o, &changed);
  if (st) return st;
  mark(4);
  st = gicp_align(o->s2m, o->T_s2s, o->T, &res->s2m);
  if (st) return st;
  mark(5);
  copy_pose(o->T, o->T_s2s_prev);             // T_s2s_prev_ = T_
  o->pose[0] = o->T[3];                       // propagateS2M
  o->pose[1] = o->T[7];
  o->pose[2] = o->T[11];
  o->rotq = quat_from_R(o->T);

  // updateKeyframes (odom.cc:1067-1154)
  {
    float closest_d = INFINITY;
    int closest = 0, idx = 0, num_nearby = 0;
    for (const auto& k : o->keyframes) {
      const float dd = (float)std::sqrt(std::pow(o->pose[0] - k->pose[0], 2) + std::pow(o->pose[1] - k->pose[1], 2) +
                                        std::pow(o->pose[2] - k->pose[2], 2));
      if (dd <= o->thresh_dist * 1.5) ++num_nearby;
      if (dd < closest_d) {
        closest_d = dd;
        closest = idx;
      }
      ++idx;
    }
    const Keyframe& ck = *o->keyframes[closest];
    const float dd = (float)std::sqrt(std::pow(o->pose[0] - ck.pose[0], 2) + std::pow(o->pose[1] - ck.pose[1], 2) +
                                      std::pow(o->pose[2] - ck.pose[2], 2));
    const Quatf dq = quat_mul(o->rotq, quat_inverse(ck.q));
    const float theta_rad = (float)(2. * std::atan2(std::sqrt(std::pow(dq.x, 2) + std::pow(dq.y, 2) + std::pow(dq.z, 2)), dq.w));
    const float theta_deg = (float)(theta_rad * (180.0 / M_PI));
    bool add = false;
    if (std::fabs(dd) > o->thresh_dist || std::fabs(theta_deg) > o->p.keyframe_thresh_rot) add = true;
    if (std::fabs(dd) <= o->thresh_dist) add = false;
    if (std::fabs(dd) <= o->thresh_dist && std::fabs(theta_deg) > o->p.keyframe_thresh_rot && num_nearby <= 1) add = true;
    if (add) {
      st = make_keyframe(o, scan);   // registration_scan_t_ = T_ * scan (transformScans)
      if (st) return st;
      res->keyframe_added = 1;
    }
  }
  mark(6);
  if (o->timing) {
    o->t_phase[7] += std::chrono::duration<double>(clk::now() - t0).count();
    ++o->frames;
  }
  res->status = DDLO_ODOM_TRACKED;
  copy_pose(o->T, res->T);
  copy_pose(o->T_s2s, res->T_s2s);
  res->submap_changed = changed ? 1 : 0;
  res->num_keyframes = (int)o->keyframes.size();
  res->submap_keyframes = (int)o->submap_prev.size();
  res->submap_points = o->submap_points;
  return GICP_OK;
}

gicp_status ddlo_odom_keyframe(const ddlo_odom* o, int k, float pose7[7], size_t* npoints) {
  if (!o || k < 0 || k >= (int)o->keyframes.size()) return fail(GICP_EINVAL, "invalid keyframe index");
  const Keyframe& kf = *o->keyframes[k];
  if (pose7) {
    pose7[0] = kf.pose[0];
    pose7[1] = kf.pose[1];
    pose7[2] = kf.pose[2];
    pose7[3] = kf.q.x;
    pose7[4] = kf.q.y;
    pose7[5] = kf.q.z;
    pose7[6] = kf.q.w;
  }
  if (npoints) *npoints = (size_t)kf.n;
  return GICP_OK;
}

gicp_status ddlo_odom_submap(const ddlo_odom* o, int32_t* idx, size_t cap, size_t* n) {
  if (!o || !n) return fail(GICP_EINVAL, "null argument");
  *n = o->submap_prev.size();
  if (idx)
    for (size_t i = 0; i < std::min(cap, o->submap_prev.size()); ++i) idx[i] = o->submap_prev[i];
  return GICP_OK;
}

gicp_status ddlo_odom_ctx(ddlo_odom* o, int which, gicp_ctx** ctx) {
  if (!o || !ctx || (which != 0 && which != 1)) return fail(GICP_EINVAL, "invalid argument");
  *ctx = which == 0 ? o->s2s : o->s2m;
  return GICP_OK;
}

gicp_status ddlo_preprocess(int device, const float* xyz, size_t n, size_t stride, double crop_size, double leaf,
                            float* out, size_t cap, size_t* nout) {
  if ((!xyz && n) || !nout || stride < 12 || stride % 4 || n > (size_t)INT32_MAX / 2) return fail(GICP_EINVAL, "invalid argument");
  ddlo_odom_params p;
  ddlo_odom_default_params(&p);
  ddlo_odom* o = nullptr;
  gicp_status st = ddlo_odom_create(device, &p, &o);
  if (st) return st;
  std::unique_ptr<ddlo_odom, gicp_status (*)(ddlo_odom*)> guard(o, ddlo_odom_destroy);
  *nout = 0;
  if (n == 0) return GICP_OK;
  HIP_TRY(o->up.ensure((n - 1) * stride + 12));
  HIP_TRY(hipMemcpyAsync(o->up.p, xyz, (n - 1) * stride + 12, hipMemcpyHostToDevice, o->s));
  HIP_TRY(o->a.ensure(sizeof(float4) * n));
  launch_pack4(o->s, o->up.as<unsigned char>(), stride, (int)n, o->a.as<float4>());
  int m = 0;
  st = preprocess(o, (int)n, crop_size > 0, crop_size, leaf > 0, leaf, &m);
  if (st) return st;
  *nout = (size_t)m;
  if (out && m > 0) {
    if ((size_t)m > cap) return fail(GICP_EINVAL, "output capacity too small");
    std::vector<float4> h(m);
    HIP_TRY(hipMemcpyAsync(h.data(), o->a.p, sizeof(float4) * m, hipMemcpyDeviceToHost, o->s));
    HIP_TRY(hipStreamSynchronize(o->s));
    for (int i = 0; i < m; ++i) {
      out[3 * i] = h[i].x;
      out[3 * i + 1] = h[i].y;
      out[3 * i + 2] = h[i].z;
    }
  }
  return GICP_OK;
}

gicp_status ddlo_convex_hull(const float* xyz, int n, int32_t* idx, int cap, int* nidx) {
  if ((!xyz && n) || (!idx && cap > 0) || !nidx || n < 0 || cap < 0) return fail(GICP_EINVAL, "invalid argument");
  const std::vector<int> h = convex_hull(xyz, n);
  for (size_t i = 0; i < h.size() && (int)i < cap; ++i) idx[i] = h[i];
  *nidx = (int)h.size();
  return GICP_OK;
}

gicp_status ddlo_concave_hull(const float* xyz, int n, double alpha, int32_t* idx, int cap, int* nidx) {
  if ((!xyz && n) || (!idx && cap > 0) || !nidx || n < 0 || cap < 0) return fail(GICP_EINVAL, "invalid argument");
  const std::vector<int> h = concave_hull(xyz, n, alpha);
  for (size_t i = 0; i < h.size() && (int)i < cap; ++i) idx[i] = h[i];
  *nidx = (int)h.size();
  return GICP_OK;
}

}  // extern "C"
