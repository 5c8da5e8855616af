/*
 * oracle/cpu_ref.cpp — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference NanoGICP hot path, used (1) as the parity
 * checker of the HIP path in tests/, __graft_entry__.smoke() and (2) as the
 * timed CPU baseline ("kind": "port") in bench.py.  The product never links,
 * loads or calls this file.
 *
 * What it restates (reference = /root/reference/dynamic_direct_lidar_odometry):
 *   KdTree              nanoflann KDTreeSingleIndexAdaptor, L2 float, DIM 3,
 *                       leaf_max_size 100 (include/nano_gicp/nanoflann.hpp:119,
 *                       impl/nanoflann_impl.hpp:987-1143 build,
 *                       :1365-1384,1495-1566 search, :161-242 KNNResultSet,
 *                       :496-524 L2_Simple_Adaptor distance order)
 *   calculate_covariances  impl/nano_gicp_impl.hpp:373-441
 *   update_correspondences impl/nano_gicp_impl.hpp:234-275
 *   linearize              impl/nano_gicp_impl.hpp:277-342
 *   compute_error          impl/nano_gicp_impl.hpp:344-371
 *   computeTransformation  impl/lsq_registration_impl.hpp:95-126
 *   is_converged / step_gn / step_lm  :128-139 / :155-173 / :175-232
 *   so3_exp, skewd         gicp/so3.hpp:63-74, :101-124
 * Eigen::LDLT (pivoted), Eigen::JacobiSVD, Matrix4d::inverse and
 * Quaternion::toRotationMatrix are restated from their published algorithms
 * (Eigen 3.3.7, implied by the reference's ros:noetic image, docker/Dockerfile:1).
 *
 * Parity pinning: the kd-tree half is pinned bit-exactly against the
 * reference's own nanoflann compiled from /root/reference (oracle/_ref, see
 * oracle/Makefile and tests/test_oracle_pin.py).  The GICP half needs Eigen /
 * PCL, which are absent, so it is NOT pinned against the reference binary:
 * it is cross-checked against an independent numpy/scipy implementation
 * (tests/test_oracle_numpy.py) — "parity unpinned" for that half.
 *
 * fp32 query transform order: q_i = (R_i0*x + R_i1*y) + (R_i2*z + t_i), no
 * FMA — Eigen 3.3's coefficient-based lazy product of the 3x4 affine block
 * with a Vector4f unrolls its 4-term redux pairwise.  The HIP path uses the
 * same order, so correspondences match bit-for-bit.
 */
#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/ddlo_gicp.h"

namespace oref {

/* ========================= nanoflann restatement ========================= */
struct Interval { float low, high; };
using BBox = Interval[3];

struct Node {
  // leaf: left/right point range in vind; non-leaf: divfeat/divlow/divhigh
  int left = 0, right = 0;
  int divfeat = 0;
  float divlow = 0.f, divhigh = 0.f;
  int child1 = -1, child2 = -1;
};

class KdTree {
 public:
  void build(const float* xyz, int n, int leaf_max = 100) {
    pts_ = xyz;
    n_ = n;
    leaf_max_ = leaf_max;
    vind_.resize(n);
    for (int i = 0; i < n; ++i) vind_[i] = i;
    nodes_.clear();
    nodes_.reserve(2 * (n / std::max(1, leaf_max / 2)) + 16);
    root_ = -1;
    if (n == 0) return;
    computeBoundingBox(root_bbox_);
    BBox bb;
    std::memcpy(bb, root_bbox_, sizeof(BBox));
    root_ = divideTree(0, n, bb);
  }

  int size() const { return n_; }

  // tests: vind and the nodes in preorder (= this restatement's allocation
  // order): (child1, child2, divfeat, -1) or (left, right, -1, -1) for a
  // leaf, and (divlow, divhigh); returns the node count (-1: cap too small)
  int export_tree(int* vind, int* nodes4, float* div2, int cap) const {
    for (int i = 0; i < n_; ++i) vind[i] = vind_[i];
    if ((int)nodes_.size() > cap) return -1;
    for (size_t i = 0; i < nodes_.size(); ++i) {
      const Node& nd = nodes_[i];
      const bool leaf = nd.child1 < 0 && nd.child2 < 0;
      nodes4[4 * i] = leaf ? nd.left : nd.child1;
      nodes4[4 * i + 1] = leaf ? nd.right : nd.child2;
      nodes4[4 * i + 2] = leaf ? -1 : nd.divfeat;
      nodes4[4 * i + 3] = -1;
      div2[2 * i] = leaf ? 0.f : nd.divlow;
      div2[2 * i + 1] = leaf ? 0.f : nd.divhigh;
    }
    return (int)nodes_.size();
  }

  // nearestKSearch: returns count found (== k when n >= k)
  int knn(const float* q, int k, int* idx, float* dist) const {
    // KNNResultSet::init (nanoflann_impl.hpp:180-187)
    int count = 0;
    if (k) dist[k - 1] = std::numeric_limits<float>::max();
    if (n_ == 0) return 0;
    float dists[3] = {0.f, 0.f, 0.f};
    float distsq = computeInitialDistances(q, dists);
    Result rs{idx, dist, k, &count};
    searchLevel(rs, q, root_, distsq, dists, 1.0f);
    return count;
  }

 private:
  struct Result {
    int* indices;
    float* dists;
    int capacity;
    int* count;
    float worst() const { return dists[capacity - 1]; }
    // KNNResultSet::addPoint (nanoflann_impl.hpp:205-237), default (non
    // NANOFLANN_FIRST_MATCH) tie rule: strict '>' shift.
    void add(float d, int index) {
      int i;
      for (i = *count; i > 0; --i) {
        if (dists[i - 1] > d) {
          if (i < capacity) {
            dists[i] = dists[i - 1];
            indices[i] = indices[i - 1];
          }
        } else {
          break;
        }
      }
      if (i < capacity) {
        dists[i] = d;
        indices[i] = index;
      }
      if (*count < capacity) (*count)++;
    }
  };

  float pt(int idx, int dim) const { return pts_[3 * idx + dim]; }

  // L2_Simple_Adaptor::evalMetric (nanoflann_impl.hpp:511-520)
  float evalMetric(const float* a, int b) const {
    float result = 0.f;
    for (int i = 0; i < 3; ++i) {
      const float diff = a[i] - pt(b, i);
      result += diff * diff;
    }
    return result;
  }
  static float accum(float a, float b) { return (a - b) * (a - b); }

  void computeBoundingBox(BBox& bbox) const {  // :1459-1487 (adaptor has no bbox)
    for (int i = 0; i < 3; ++i) bbox[i].low = bbox[i].high = pt(0, i);
    for (int k = 1; k < n_; ++k)
      for (int i = 0; i < 3; ++i) {
        if (pt(k, i) < bbox[i].low) bbox[i].low = pt(k, i);
        if (pt(k, i) > bbox[i].high) bbox[i].high = pt(k, i);
      }
  }

  void computeMinMax(const int* ind, int count, int element, float& mn, float& mx) const {  // :967-980
    mn = pt(ind[0], element);
    mx = pt(ind[0], element);
    for (int i = 1; i < count; ++i) {
      float v = pt(ind[i], element);
      if (v < mn) mn = v;
      if (v > mx) mx = v;
    }
  }

  int divideTree(int left, int right, BBox& bbox) {  // :987-1043
    int node = (int)nodes_.size();
    nodes_.emplace_back();
    if ((right - left) <= leaf_max_) {
      nodes_[node].left = left;
      nodes_[node].right = right;
      for (int i = 0; i < 3; ++i) {
        bbox[i].low = pt(vind_[left], i);
        bbox[i].high = pt(vind_[left], i);
      }
      for (int k = left + 1; k < right; ++k)
        for (int i = 0; i < 3; ++i) {
          if (bbox[i].low > pt(vind_[k], i)) bbox[i].low = pt(vind_[k], i);
          if (bbox[i].high < pt(vind_[k], i)) bbox[i].high = pt(vind_[k], i);
        }
    } else {
      int idx, cutfeat;
      float cutval;
      middleSplit(&vind_[0] + left, right - left, idx, cutfeat, cutval, bbox);
      nodes_[node].divfeat = cutfeat;
      BBox left_bbox, right_bbox;
      std::memcpy(left_bbox, bbox, sizeof(BBox));
      left_bbox[cutfeat].high = cutval;
      int c1 = divideTree(left, left + idx, left_bbox);
      std::memcpy(right_bbox, bbox, sizeof(BBox));
      right_bbox[cutfeat].low = cutval;
      int c2 = divideTree(left + idx, right, right_bbox);
      nodes_[node].child1 = c1;
      nodes_[node].child2 = c2;
      nodes_[node].divlow = left_bbox[cutfeat].high;
      nodes_[node].divhigh = right_bbox[cutfeat].low;
      for (int i = 0; i < 3; ++i) {
        bbox[i].low = std::min(left_bbox[i].low, right_bbox[i].low);
        bbox[i].high = std::max(left_bbox[i].high, right_bbox[i].high);
      }
    }
    return node;
  }

  void middleSplit(int* ind, int count, int& index, int& cutfeat, float& cutval, const BBox& bbox) {  // :1045-1096
    const float EPS = 0.00001f;
    float max_span = bbox[0].high - bbox[0].low;
    for (int i = 1; i < 3; ++i) {
      float span = bbox[i].high - bbox[i].low;
      if (span > max_span) max_span = span;
    }
    float max_spread = -1;
    cutfeat = 0;
    for (int i = 0; i < 3; ++i) {
      float span = bbox[i].high - bbox[i].low;
      if (span > (1 - EPS) * max_span) {
        float mn, mx;
        computeMinMax(ind, count, i, mn, mx);
        float spread = mx - mn;
        if (spread > max_spread) {
          cutfeat = i;
          max_spread = spread;
        }
      }
    }
    float split_val = (bbox[cutfeat].low + bbox[cutfeat].high) / 2;
    float mn, mx;
    computeMinMax(ind, count, cutfeat, mn, mx);
    if (split_val < mn)
      cutval = mn;
    else if (split_val > mx)
      cutval = mx;
    else
      cutval = split_val;
    int lim1, lim2;
    planeSplit(ind, count, cutfeat, cutval, lim1, lim2);
    if (lim1 > count / 2)
      index = lim1;
    else if (lim2 < count / 2)
      index = lim2;
    else
      index = count / 2;
  }

  void planeSplit(int* ind, int count, int cutfeat, float cutval, int& lim1, int& lim2) {  // :1107-1143
    int left = 0, right = count - 1;
    for (;;) {
      while (left <= right && pt(ind[left], cutfeat) < cutval) ++left;
      while (right && left <= right && pt(ind[right], cutfeat) >= cutval) --right;
      if (left > right || !right) break;
      std::swap(ind[left], ind[right]);
      ++left;
      --right;
    }
    lim1 = left;
    right = count - 1;
    for (;;) {
      while (left <= right && pt(ind[left], cutfeat) <= cutval) ++left;
      while (right && left <= right && pt(ind[right], cutfeat) > cutval) --right;
      if (left > right || !right) break;
      std::swap(ind[left], ind[right]);
      ++left;
      --right;
    }
    lim2 = left;
  }

  float computeInitialDistances(const float* vec, float* dists) const {  // :1145-1164
    float distsq = 0.f;
    for (int i = 0; i < 3; ++i) {
      if (vec[i] < root_bbox_[i].low) {
        dists[i] = accum(vec[i], root_bbox_[i].low);
        distsq += dists[i];
      }
      if (vec[i] > root_bbox_[i].high) {
        dists[i] = accum(vec[i], root_bbox_[i].high);
        distsq += dists[i];
      }
    }
    return distsq;
  }

  void searchLevel(Result& rs, const float* vec, int node_i, float mindistsq, float* dists, float epsError) const {
    const Node& node = nodes_[node_i];  // :1495-1566
    if (node.child1 < 0 && node.child2 < 0) {
      float worst_dist = rs.worst();
      for (int i = node.left; i < node.right; ++i) {
        const int index = vind_[i];
        float d = evalMetric(vec, index);
        if (d < worst_dist) rs.add(d, vind_[i]);
      }
      return;
    }
    int idx = node.divfeat;
    float val = vec[idx];
    float diff1 = val - node.divlow;
    float diff2 = val - node.divhigh;
    int bestChild, otherChild;
    float cut_dist;
    if ((diff1 + diff2) < 0) {
      bestChild = node.child1;
      otherChild = node.child2;
      cut_dist = accum(val, node.divhigh);
    } else {
      bestChild = node.child2;
      otherChild = node.child1;
      cut_dist = accum(val, node.divlow);
    }
    searchLevel(rs, vec, bestChild, mindistsq, dists, epsError);
    float dst = dists[idx];
    mindistsq = mindistsq + cut_dist - dst;
    dists[idx] = cut_dist;
    if (mindistsq * epsError <= rs.worst()) searchLevel(rs, vec, otherChild, mindistsq, dists, epsError);
    dists[idx] = dst;
  }

  const float* pts_ = nullptr;
  int n_ = 0;
  int leaf_max_ = 100;
  std::vector<int> vind_;
  std::vector<Node> nodes_;
  int root_ = -1;
  BBox root_bbox_;
};

/* ============================ small linear algebra ======================= */
struct Mat4 { double m[16]; };  // row-major, the reference's Eigen::Matrix4d
struct Mat6 { double m[36]; };
struct Iso { double R[9]; double t[3]; };  // Eigen::Isometry3d

static inline Iso iso_identity() {
  Iso x;
  for (int i = 0; i < 9; ++i) x.R[i] = (i % 4 == 0) ? 1.0 : 0.0;
  x.t[0] = x.t[1] = x.t[2] = 0.0;
  return x;
}

// x = a * b (Isometry product: R = Ra Rb, t = Ra tb + ta)
static inline Iso iso_mul(const Iso& a, const Iso& b) {
  Iso r;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      r.R[3 * i + j] = a.R[3 * i + 0] * b.R[0 + j] + a.R[3 * i + 1] * b.R[3 + j] + a.R[3 * i + 2] * b.R[6 + j];
    r.t[i] = (a.R[3 * i + 0] * b.t[0] + a.R[3 * i + 1] * b.t[1] + a.R[3 * i + 2] * b.t[2]) + a.t[i];
  }
  return r;
}

// so3_exp (gicp/so3.hpp:101-124) -> Quaternion::toRotationMatrix (Eigen)
static inline void so3_exp(const double* w, double* R) {
  double theta_sq = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  double imag, real;
  if (theta_sq < 1e-10) {
    double theta_quad = theta_sq * theta_sq;
    imag = 0.5 - 1.0 / 48.0 * theta_sq + 1.0 / 3840.0 * theta_quad;
    real = 1.0 - 1.0 / 8.0 * theta_sq + 1.0 / 384.0 * theta_quad;
  } else {
    double theta = std::sqrt(theta_sq);
    double half = 0.5 * theta;
    imag = std::sin(half) / theta;
    real = std::cos(half);
  }
  const double qw = real, qx = imag * w[0], qy = imag * w[1], qz = imag * w[2];
  const double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
  const double twx = tx * qw, twy = ty * qw, twz = tz * qw;
  const double txx = tx * qx, txy = ty * qx, txz = tz * qx;
  const double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

// Eigen::LDLT<Matrix<double,6,6>> compute + solve (pivoted, lower storage).
static void ldlt_solve6(const double* A_in, const double* rhs, double* x) {
  const int n = 6;
  double m[36];
  std::memcpy(m, A_in, sizeof(m));
  int tr[6];
  double temp[6];
  for (int k = 0; k < n; ++k) {
    int big = k;
    double bigv = std::fabs(m[k * n + k]);
    for (int i = k + 1; i < n; ++i)
      if (std::fabs(m[i * n + i]) > bigv) { bigv = std::fabs(m[i * n + i]); big = i; }
    tr[k] = big;
    if (k != big) {
      for (int j = 0; j < k; ++j) std::swap(m[k * n + j], m[big * n + j]);
      for (int i = big + 1; i < n; ++i) std::swap(m[i * n + k], m[i * n + big]);
      std::swap(m[k * n + k], m[big * n + big]);
      for (int i = k + 1; i < big; ++i) {
        double t = m[i * n + k];
        m[i * n + k] = m[big * n + i];
        m[big * n + i] = t;
      }
    }
    int rs = n - k - 1;
    if (k > 0) {
      for (int j = 0; j < k; ++j) temp[j] = m[j * n + j] * m[k * n + j];
      double s = 0;
      for (int j = 0; j < k; ++j) s += m[k * n + j] * temp[j];
      m[k * n + k] -= s;
      for (int i = k + 1; i < n; ++i) {
        double a = 0;
        for (int j = 0; j < k; ++j) a += m[i * n + j] * temp[j];
        m[i * n + k] -= a;
      }
    }
    double akk = m[k * n + k];
    if (rs > 0 && std::fabs(akk) > 0.0)
      for (int i = k + 1; i < n; ++i) m[i * n + k] /= akk;
  }
  double y[6];
  for (int i = 0; i < n; ++i) y[i] = rhs[i];
  for (int k = 0; k < n; ++k) std::swap(y[k], y[tr[k]]);
  for (int i = 0; i < n; ++i)  // L unit lower
    for (int j = 0; j < i; ++j) y[i] -= m[i * n + j] * y[j];
  const double tol = std::numeric_limits<double>::min();
  for (int i = 0; i < n; ++i) y[i] = (std::fabs(m[i * n + i]) > tol) ? y[i] / m[i * n + i] : 0.0;
  for (int i = n - 1; i >= 0; --i)  // L^T
    for (int j = i + 1; j < n; ++j) y[i] -= m[j * n + i] * y[j];
  for (int k = n - 1; k >= 0; --k) std::swap(y[k], y[tr[k]]);
  for (int i = 0; i < n; ++i) x[i] = y[i];
}

// General 4x4 inverse (cofactor expansion), as Matrix4d::inverse().
static void inv4(const double* m, double* inv) {
  double a[16];
  a[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
  a[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
  a[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
  a[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
  a[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
  a[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
  a[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
  a[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
  a[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
  a[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
  a[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
  a[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
  a[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
  a[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
  a[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
  a[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
  double det = m[0] * a[0] + m[1] * a[4] + m[2] * a[8] + m[3] * a[12];
  double id = 1.0 / det;
  for (int i = 0; i < 16; ++i) inv[i] = a[i] * id;
}

// Symmetric 3x3 eigen-decomposition by cyclic Jacobi (double).  Used to
// restate Eigen::JacobiSVD on the (symmetric PSD) covariance: for a symmetric
// matrix the SVD is |lambda| with V = eigenvectors, U = sign(lambda) V.
static void sym_eig3(const double* A, double* lam, double* V /*col-major vectors: V[3*j+i] = v_j[i]*/) {
  double a[3][3] = {{A[0], A[1], A[2]}, {A[3], A[4], A[5]}, {A[6], A[7], A[8]}};
  double v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  for (int sweep = 0; sweep < 50; ++sweep) {
    double off = std::fabs(a[0][1]) + std::fabs(a[0][2]) + std::fabs(a[1][2]);
    double scale = std::fabs(a[0][0]) + std::fabs(a[1][1]) + std::fabs(a[2][2]);
    if (off <= 1e-300 || off <= scale * 1e-18) break;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        double apq = a[p][q];
        if (apq == 0.0) continue;
        double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
        double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        double c = 1.0 / std::sqrt(t * t + 1.0);
        double s = t * c;
        for (int k = 0; k < 3; ++k) {  // A <- J^T A J
          double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - s * akq;
          a[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; ++k) {
          double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - s * aqk;
          a[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 3; ++k) {
          double vkp = v[k][p], vkq = v[k][q];
          v[k][p] = c * vkp - s * vkq;
          v[k][q] = s * vkp + c * vkq;
        }
      }
  }
  for (int j = 0; j < 3; ++j) {
    lam[j] = a[j][j];
    for (int i = 0; i < 3; ++i) V[3 * j + i] = v[i][j];
  }
}

static void regularize(const double* C /*3x3 row-major*/, int method, double* out /*3x3*/) {
  if (method == GICP_REG_NONE) {
    std::memcpy(out, C, 9 * sizeof(double));
    return;
  }
  if (method == GICP_REG_FROBENIUS) {  // nano_gicp_impl.hpp:405-412
    double Cl[16] = {0};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Cl[4 * i + j] = C[3 * i + j] + (i == j ? 1e-3 : 0.0);
    Cl[15] = 1.0;
    double Ci[16];
    inv4(Cl, Ci);
    double nrm = 0;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) nrm += Ci[4 * i + j] * Ci[4 * i + j];
    nrm = std::sqrt(nrm);
    double N[16] = {0};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) N[4 * i + j] = Ci[4 * i + j] / nrm;
    N[15] = 1.0;
    double R[16];
    inv4(N, R);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) out[3 * i + j] = R[4 * i + j];
    return;
  }
  // JacobiSVD route (:415-436): singular values sorted descending.
  double lam[3], V[9];
  sym_eig3(C, lam, V);
  int ord[3] = {0, 1, 2};
  std::sort(ord, ord + 3, [&](int a, int b) { return std::fabs(lam[a]) > std::fabs(lam[b]); });
  double sv[3], vals[3];
  for (int i = 0; i < 3; ++i) sv[i] = std::fabs(lam[ord[i]]);
  if (method == GICP_REG_PLANE) {
    vals[0] = 1; vals[1] = 1; vals[2] = 1e-3;
  } else if (method == GICP_REG_MIN_EIG) {
    for (int i = 0; i < 3; ++i) vals[i] = std::max(sv[i], 1e-3);
  } else {  // NORMALIZED_MIN_EIG
    for (int i = 0; i < 3; ++i) vals[i] = std::max(sv[i] / sv[0], 1e-3);
  }
  for (int i = 0; i < 9; ++i) out[i] = 0.0;
  for (int j = 0; j < 3; ++j) {
    const double* v = &V[3 * ord[j]];
    const double sgn = lam[ord[j]] < 0 ? -1.0 : 1.0;  // U col = sign * V col
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) out[3 * r + c] += sgn * v[r] * vals[j] * v[c];
  }
}

/* ============================== NanoGICP ================================= */
static int omp_threads(int want) {
#ifdef _OPENMP
  return want > 0 ? want : omp_get_max_threads();
#else
  (void)want;
  return 1;
#endif
}
static int omp_tid() {
#ifdef _OPENMP
  return omp_get_thread_num();
#else
  return 0;
#endif
}

// calculate_covariances (nano_gicp_impl.hpp:373-441) -> Matrix4d per point
static void calculate_covariances(const float* xyz, int n, const KdTree& tree, int k, int reg, Mat4* covs, int nthreads) {
  const int nt = omp_threads(nthreads);
#pragma omp parallel for num_threads(nt) schedule(guided, 8)
  for (int i = 0; i < n; i++) {
    std::vector<int> k_indices(k);
    std::vector<float> k_sq(k);
    tree.knn(&xyz[3 * i], k, k_indices.data(), k_sq.data());
    // neighbors 4 x k (w = 1), centred by the row mean, cov = X X^T / k
    double mean[3] = {0, 0, 0};
    for (int j = 0; j < k; ++j)
      for (int d = 0; d < 3; ++d) mean[d] += (double)xyz[3 * k_indices[j] + d];
    for (int d = 0; d < 3; ++d) mean[d] /= k;
    double C[9] = {0};
    for (int j = 0; j < k; ++j) {
      double c[3];
      for (int d = 0; d < 3; ++d) c[d] = (double)xyz[3 * k_indices[j] + d] - mean[d];
      for (int r = 0; r < 3; ++r)
        for (int s = 0; s < 3; ++s) C[3 * r + s] += c[r] * c[s];
    }
    for (int e = 0; e < 9; ++e) C[e] /= k;
    double Rg[9];
    regularize(C, reg, Rg);
    Mat4& out = covs[i];
    std::memset(out.m, 0, sizeof(out.m));
    for (int r = 0; r < 3; ++r)
      for (int s = 0; s < 3; ++s) out.m[4 * r + s] = Rg[3 * r + s];
  }
}

struct Gicp {
  gicp_params p;
  int nthreads = 0;
  const float* src = nullptr;
  int ns = 0;
  const float* tgt = nullptr;
  int nt = 0;
  KdTree src_tree, tgt_tree;
  std::vector<Mat4> src_covs, tgt_covs, mahalanobis;
  std::vector<int> corr;
  std::vector<float> sqd;
  double lm_lambda = -1.0;
  Mat6 final_hessian;
  int lm_trials = 0;
  int lin_calls = 0;
  // optional per-iteration trace: [cost, pose(12)] per linearize call
  std::vector<double> trace;

  static void iso_to4(const Iso& x, double* T) {
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) T[4 * i + j] = x.R[3 * i + j];
      T[4 * i + 3] = x.t[i];
    }
    T[12] = T[13] = T[14] = 0;
    T[15] = 1;
  }

  // update_correspondences (nano_gicp_impl.hpp:234-275)
  void update_correspondences(const Iso& trans) {
    float Rf[9], tf[3];
    for (int i = 0; i < 9; ++i) Rf[i] = (float)trans.R[i];
    for (int i = 0; i < 3; ++i) tf[i] = (float)trans.t[i];
    double T[16];
    iso_to4(trans, T);
    corr.resize(ns);
    sqd.resize(ns);
    mahalanobis.resize(ns);
    const double thr2 = p.max_correspondence_distance * p.max_correspondence_distance;
    const int nth = omp_threads(nthreads);
#pragma omp parallel for num_threads(nth) schedule(guided, 8)
    for (int i = 0; i < ns; i++) {
      const float x = src[3 * i], y = src[3 * i + 1], z = src[3 * i + 2];
      float q[3];
      for (int r = 0; r < 3; ++r) q[r] = (Rf[3 * r] * x + Rf[3 * r + 1] * y) + (Rf[3 * r + 2] * z + tf[r]);
      int idx;
      float d;
      tgt_tree.knn(q, 1, &idx, &d);
      sqd[i] = d;
      corr[i] = (double)d < thr2 ? idx : -1;
      if (corr[i] < 0) continue;
      const Mat4& cA = src_covs[i];
      const Mat4& cB = tgt_covs[idx];
      // RCR = cov_B + T cov_A T^T ; RCR(3,3) = 1 ; M = RCR^-1 ; M(3,3) = 0
      double TC[16], RCR[16];
      for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
          double s = 0;
          for (int k = 0; k < 4; ++k) s += T[4 * r + k] * cA.m[4 * k + c];
          TC[4 * r + c] = s;
        }
      for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
          double s = 0;
          for (int k = 0; k < 4; ++k) s += TC[4 * r + k] * T[4 * c + k];
          RCR[4 * r + c] = cB.m[4 * r + c] + s;
        }
      RCR[15] = 1.0;
      inv4(RCR, mahalanobis[i].m);
      mahalanobis[i].m[15] = 0.0;
    }
  }

  // linearize (nano_gicp_impl.hpp:277-342)
  double linearize(const Iso& trans, double* H, double* b) {
    update_correspondences(trans);
    ++lin_calls;
    double T[16];
    iso_to4(trans, T);
    const int nth = omp_threads(nthreads);
    std::vector<Mat6> Hs(nth);
    std::vector<std::array<double, 6>> bs(nth);
    for (int t = 0; t < nth; ++t) {
      std::memset(Hs[t].m, 0, sizeof(Hs[t].m));
      bs[t].fill(0.0);
    }
    double sum_errors = 0.0;
#pragma omp parallel for num_threads(nth) reduction(+ : sum_errors) schedule(guided, 8)
    for (int i = 0; i < ns; i++) {
      int j = corr[i];
      if (j < 0) continue;
      double a[4] = {(double)src[3 * i], (double)src[3 * i + 1], (double)src[3 * i + 2], 1.0};
      double bpt[4] = {(double)tgt[3 * j], (double)tgt[3 * j + 1], (double)tgt[3 * j + 2], 1.0};
      double ta[4];
      for (int r = 0; r < 3; ++r) ta[r] = (T[4 * r] * a[0] + T[4 * r + 1] * a[1]) + (T[4 * r + 2] * a[2] + T[4 * r + 3] * a[3]);
      ta[3] = 1.0;
      double e[4];
      for (int r = 0; r < 4; ++r) e[r] = bpt[r] - ta[r];
      const double* M = mahalanobis[i].m;
      double Me[4];
      for (int r = 0; r < 4; ++r) Me[r] = M[4 * r] * e[0] + M[4 * r + 1] * e[1] + M[4 * r + 2] * e[2] + M[4 * r + 3] * e[3];
      sum_errors += e[0] * Me[0] + e[1] * Me[1] + e[2] * Me[2] + e[3] * Me[3];
      if (!H || !b) continue;
      // dtdx0 4x6 = [skewd(ta) | -I ; 0]
      double J[4][6] = {{0}};
      J[0][1] = -ta[2]; J[0][2] = ta[1];
      J[1][0] = ta[2];  J[1][2] = -ta[0];
      J[2][0] = -ta[1]; J[2][1] = ta[0];
      J[0][3] = -1; J[1][4] = -1; J[2][5] = -1;
      double MJ[4][6];
      for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 6; ++c) MJ[r][c] = M[4 * r] * J[0][c] + M[4 * r + 1] * J[1][c] + M[4 * r + 2] * J[2][c] + M[4 * r + 3] * J[3][c];
      Mat6& Ht = Hs[omp_tid()];
      auto& bt = bs[omp_tid()];
      for (int r = 0; r < 6; ++r) {
        for (int c = 0; c < 6; ++c) Ht.m[6 * r + c] += J[0][r] * MJ[0][c] + J[1][r] * MJ[1][c] + J[2][r] * MJ[2][c] + J[3][r] * MJ[3][c];
        bt[r] += J[0][r] * Me[0] + J[1][r] * Me[1] + J[2][r] * Me[2] + J[3][r] * Me[3];
      }
    }
    if (H && b) {
      std::memset(H, 0, 36 * sizeof(double));
      std::memset(b, 0, 6 * sizeof(double));
      for (int t = 0; t < nth; ++t) {
        for (int e = 0; e < 36; ++e) H[e] += Hs[t].m[e];
        for (int e = 0; e < 6; ++e) b[e] += bs[t][e];
      }
    }
    trace.push_back(sum_errors);
    for (int i = 0; i < 9; ++i) trace.push_back(trans.R[i]);
    for (int i = 0; i < 3; ++i) trace.push_back(trans.t[i]);
    return sum_errors;
  }

  // compute_error (nano_gicp_impl.hpp:344-371)
  double compute_error(const Iso& trans) {
    ++lm_trials;
    double T[16];
    iso_to4(trans, T);
    double sum_errors = 0.0;
    const int nth = omp_threads(nthreads);
#pragma omp parallel for num_threads(nth) reduction(+ : sum_errors) schedule(guided, 8)
    for (int i = 0; i < ns; i++) {
      int j = corr[i];
      if (j < 0) continue;
      double a[4] = {(double)src[3 * i], (double)src[3 * i + 1], (double)src[3 * i + 2], 1.0};
      double ta[4];
      for (int r = 0; r < 3; ++r) ta[r] = (T[4 * r] * a[0] + T[4 * r + 1] * a[1]) + (T[4 * r + 2] * a[2] + T[4 * r + 3] * a[3]);
      ta[3] = 1.0;
      double e[4] = {(double)tgt[3 * j] - ta[0], (double)tgt[3 * j + 1] - ta[1], (double)tgt[3 * j + 2] - ta[2], 0.0};
      const double* M = mahalanobis[i].m;
      double s = 0;
      for (int r = 0; r < 4; ++r) s += e[r] * (M[4 * r] * e[0] + M[4 * r + 1] * e[1] + M[4 * r + 2] * e[2] + M[4 * r + 3] * e[3]);
      sum_errors += s;
    }
    return sum_errors;
  }

  bool is_converged(const Iso& delta) const {  // lsq_registration_impl.hpp:128-139
    if (p.fixed_iterations > 0) return false;
    // (1 / eps) * |x| per entry, then the max (:135-138); the product rounds
    // monotonically, so scaling the largest |x| gives the same maximum
    double mr = 0.0, mt = 0.0;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) mr = std::max(mr, std::fabs(delta.R[3 * i + j] - (i == j ? 1.0 : 0.0)));
    for (int i = 0; i < 3; ++i) mt = std::max(mt, std::fabs(delta.t[i]));
    return std::max(1.0 / p.rotation_epsilon * mr, 1.0 / p.transformation_epsilon * mt) < 1;
  }

  static Iso make_delta(const double* d) {
    Iso x;
    so3_exp(d, x.R);
    x.t[0] = d[3]; x.t[1] = d[4]; x.t[2] = d[5];
    return x;
  }

  bool step_gn(Iso& x0, Iso& delta) {  // :155-173
    double H[36], b[6];
    linearize(x0, H, b);
    double nb[6], d[6];
    for (int i = 0; i < 6; ++i) nb[i] = -b[i];
    ldlt_solve6(H, nb, d);
    delta = make_delta(d);
    x0 = iso_mul(delta, x0);
    std::memcpy(final_hessian.m, H, sizeof(H));
    return true;
  }

  bool step_lm(Iso& x0, Iso& delta) {  // :175-232
    double H[36], b[6];
    double y0 = linearize(x0, H, b);
    if (lm_lambda < 0.0) {
      double mx = 0;
      for (int i = 0; i < 6; ++i) mx = std::max(mx, std::fabs(H[7 * i]));
      lm_lambda = p.lm_init_lambda_factor * mx;
    }
    double nu = 2.0;
    for (int i = 0; i < p.lm_max_iterations; i++) {
      double A[36];
      std::memcpy(A, H, sizeof(A));
      for (int k = 0; k < 6; ++k) A[7 * k] += lm_lambda;
      double nb[6], d[6];
      for (int k = 0; k < 6; ++k) nb[k] = -b[k];
      ldlt_solve6(A, nb, d);
      delta = make_delta(d);
      Iso xi = iso_mul(delta, x0);
      double yi = compute_error(xi);
      double den = 0;
      for (int k = 0; k < 6; ++k) den += d[k] * (lm_lambda * d[k] - b[k]);
      double rho = (y0 - yi) / den;
      if (rho < 0) {
        if (is_converged(delta)) return true;
        lm_lambda = nu * lm_lambda;
        nu = 2 * nu;
        continue;
      }
      x0 = xi;
      lm_lambda = lm_lambda * std::max(1.0 / 3.0, 1 - std::pow(2 * rho - 1, 3));
      std::memcpy(final_hessian.m, H, sizeof(H));
      return true;
    }
    return false;
  }

  // computeTransformation (nano_gicp_impl.hpp:183-196 + lsq_registration_impl.hpp:95-126)
  void align(const float* guess, float* out, gicp_result* res) {
    if ((int)src_covs.size() != ns) {
      src_covs.resize(ns);
      calculate_covariances(src, ns, src_tree, p.k_correspondences, p.regularization, src_covs.data(), nthreads);
    }
    if ((int)tgt_covs.size() != nt) {
      tgt_covs.resize(nt);
      calculate_covariances(tgt, nt, tgt_tree, p.k_correspondences, p.regularization, tgt_covs.data(), nthreads);
    }
    Iso x0;
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) x0.R[3 * i + j] = (double)guess[4 * i + j];
      x0.t[i] = (double)guess[4 * i + 3];
    }
    lm_lambda = -1.0;
    bool converged = false;
    int nr_iter = 0;
    bool lm_failed = false;
    lm_trials = 0;
    lin_calls = 0;
    trace.clear();
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < 6; ++j) final_hessian.m[6 * i + j] = (i == j) ? 1.0 : 0.0;
    const int max_it = p.fixed_iterations > 0 ? p.fixed_iterations : p.max_iterations;
    for (int i = 0; i < max_it && !converged; i++) {
      nr_iter = i;
      Iso delta;
      bool ok = (p.optimizer == GICP_OPT_GAUSS_NEWTON) ? step_gn(x0, delta) : step_lm(x0, delta);
      if (!ok) {
        lm_failed = true;  // "lm not converged!!"
        break;
      }
      converged = is_converged(delta);
    }
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) out[4 * i + j] = (float)x0.R[3 * i + j];
      out[4 * i + 3] = (float)x0.t[i];
    }
    out[12] = out[13] = out[14] = 0.f;
    out[15] = 1.f;
    if (res) {
      std::memset(res, 0, sizeof(*res));
      res->converged = converged;
      res->nr_iterations = nr_iter;
      res->iterations_run = lin_calls;
      res->lm_failed = lm_failed;
      res->lm_trials = lm_trials;
      int nc = 0;
      for (int i = 0; i < ns; ++i) nc += corr[i] >= 0;
      res->num_correspondences = nc;
      res->final_cost = trace.empty() ? 0.0 : trace[trace.size() - 13];
      std::memcpy(res->final_hessian, final_hessian.m, sizeof(res->final_hessian));
      res->lm_lambda = lm_lambda;
    }
  }
};

static void unpack_cov(const double* cov, int layout, Mat4& out) {
  std::memset(out.m, 0, sizeof(out.m));
  if (layout == GICP_COV_MAT4D) {
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) out.m[4 * r + c] = cov[4 * r + c];
  } else {
    const double xx = cov[0], xy = cov[1], xz = cov[2], yy = cov[3], yz = cov[4], zz = cov[5];
    double m[9] = {xx, xy, xz, xy, yy, yz, xz, yz, zz};
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) out.m[4 * r + c] = m[3 * r + c];
  }
}

}  // namespace oref

/* ================================ C API ================================== */
extern "C" {

void* oref_tree_build(const float* xyz, int n) {
  auto* t = new oref::KdTree();
  t->build(xyz, n, 100);
  return t;
}
void oref_tree_free(void* t) { delete static_cast<oref::KdTree*>(t); }
int oref_tree_export(void* t, int* vind, int* nodes4, float* div2, int cap) {
  return static_cast<oref::KdTree*>(t)->export_tree(vind, nodes4, div2, cap);
}

// k-NN of nq queries; outputs idx[nq*k], d[nq*k]; returns 0
int oref_tree_knn(void* th, const float* q, int nq, int k, int* idx, float* d, int nthreads) {
  auto* t = static_cast<oref::KdTree*>(th);
  const int nt = oref::omp_threads(nthreads);
#pragma omp parallel for num_threads(nt) schedule(guided, 8)
  for (int i = 0; i < nq; ++i) t->knn(&q[3 * i], k, &idx[(size_t)i * k], &d[(size_t)i * k]);
  return 0;
}

// covariances of a cloud (own kd-tree, k neighbours incl. self); out SYM6 per point
int oref_covariances(const float* xyz, int n, int k, int reg, double* out6, int nthreads) {
  if (n < k || k <= 0) return GICP_ETOOFEW;
  oref::KdTree t;
  t.build(xyz, n, 100);
  std::vector<oref::Mat4> covs(n);
  oref::calculate_covariances(xyz, n, t, k, reg, covs.data(), nthreads);
  for (int i = 0; i < n; ++i) {
    const double* m = covs[i].m;
    double* o = &out6[6 * (size_t)i];
    o[0] = m[0]; o[1] = m[1]; o[2] = m[2]; o[3] = m[5]; o[4] = m[6]; o[5] = m[10];
  }
  return 0;
}

struct oref_gicp;
// Create a GICP problem: clouds are referenced (not copied) and must outlive the handle.
oref_gicp* oref_gicp_create(const gicp_params* p, const float* src, int ns, const float* tgt, int nt, int nthreads) {
  auto* g = new oref::Gicp();
  g->p = *p;
  g->nthreads = nthreads;
  g->src = src;
  g->ns = ns;
  g->tgt = tgt;
  g->nt = nt;
  g->src_tree.build(src, ns, 100);
  g->tgt_tree.build(tgt, nt, 100);
  return reinterpret_cast<oref_gicp*>(g);
}
void oref_gicp_free(oref_gicp* h) { delete reinterpret_cast<oref::Gicp*>(h); }
void oref_gicp_set_threads(oref_gicp* h, int nthreads) { reinterpret_cast<oref::Gicp*>(h)->nthreads = nthreads; }
void oref_gicp_set_params(oref_gicp* h, const gicp_params* p) { reinterpret_cast<oref::Gicp*>(h)->p = *p; }

int oref_gicp_set_covariances(oref_gicp* h, int side, const double* cov, int n, int layout) {
  auto* g = reinterpret_cast<oref::Gicp*>(h);
  auto& v = side == GICP_SIDE_SOURCE ? g->src_covs : g->tgt_covs;
  v.resize(n);
  const int w = layout == GICP_COV_MAT4D ? 16 : 6;
  for (int i = 0; i < n; ++i) oref::unpack_cov(&cov[(size_t)w * i], layout, v[i]);
  return 0;
}
int oref_gicp_compute_covariances(oref_gicp* h, int side) {
  auto* g = reinterpret_cast<oref::Gicp*>(h);
  if (side == GICP_SIDE_SOURCE) {
    g->src_covs.resize(g->ns);
    oref::calculate_covariances(g->src, g->ns, g->src_tree, g->p.k_correspondences, g->p.regularization, g->src_covs.data(), g->nthreads);
  } else {
    g->tgt_covs.resize(g->nt);
    oref::calculate_covariances(g->tgt, g->nt, g->tgt_tree, g->p.k_correspondences, g->p.regularization, g->tgt_covs.data(), g->nthreads);
  }
  return 0;
}
int oref_gicp_get_covariances(oref_gicp* h, int side, double* out6) {
  auto* g = reinterpret_cast<oref::Gicp*>(h);
  auto& v = side == GICP_SIDE_SOURCE ? g->src_covs : g->tgt_covs;
  for (size_t i = 0; i < v.size(); ++i) {
    const double* m = v[i].m;
    double* o = &out6[6 * i];
    o[0] = m[0]; o[1] = m[1]; o[2] = m[2]; o[3] = m[5]; o[4] = m[6]; o[5] = m[10];
  }
  return 0;
}

int oref_gicp_align(oref_gicp* h, const float* guess16, float* out16, gicp_result* res) {
  auto* g = reinterpret_cast<oref::Gicp*>(h);
  float I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  g->align(guess16 ? guess16 : I, out16, res);
  return 0;
}

// linearize at pose16 (row-major double); requires covariances set/computed
int oref_gicp_linearize(oref_gicp* h, const double* pose16, double* H36, double* b6, double* cost, int* corr, float* sqd) {
  auto* g = reinterpret_cast<oref::Gicp*>(h);
  if ((int)g->src_covs.size() != g->ns || (int)g->tgt_covs.size() != g->nt) return GICP_ESTATE;
  oref::Iso x;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) x.R[3 * i + j] = pose16[4 * i + j];
    x.t[i] = pose16[4 * i + 3];
  }
  double c = g->linearize(x, H36, b6);
  if (cost) *cost = c;
  if (corr) std::memcpy(corr, g->corr.data(), sizeof(int) * g->ns);
  if (sqd) std::memcpy(sqd, g->sqd.data(), sizeof(float) * g->ns);
  return 0;
}

double oref_gicp_compute_error(oref_gicp* h, const double* pose16) {
  auto* g = reinterpret_cast<oref::Gicp*>(h);
  oref::Iso x;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) x.R[3 * i + j] = pose16[4 * i + j];
    x.t[i] = pose16[4 * i + 3];
  }
  return g->compute_error(x);
}

// correspondences/sq distances of the last linearize (reference getResiduals source data)
int oref_gicp_last_correspondences(oref_gicp* h, int* corr, float* sqd) {
  auto* g = reinterpret_cast<oref::Gicp*>(h);
  if (corr) std::memcpy(corr, g->corr.data(), sizeof(int) * g->corr.size());
  if (sqd) std::memcpy(sqd, g->sqd.data(), sizeof(float) * g->sqd.size());
  return (int)g->corr.size();
}

// per-linearize trace of the last align: n entries of [cost, R(9), t(3)]
int oref_gicp_trace(oref_gicp* h, double* out, int max_entries) {
  auto* g = reinterpret_cast<oref::Gicp*>(h);
  int n = (int)(g->trace.size() / 13);
  int m = std::min(n, max_entries);
  if (out) std::memcpy(out, g->trace.data(), sizeof(double) * 13 * m);
  return n;
}

// pcl::VoxelGrid<PointXYZI>::applyFilter (PCL 1.10, filters/impl/voxel_grid.hpp;
// used at odom.cc:469-475 and :1133-1137), xyz part: finite points only,
// min/max box, int voxel index (ijk - min_b) . divb_mul, std::sort of the
// (idx, point) pairs by idx (the SAME libstdc++ introsort, so equal-index
// points keep the reference's summation order), one centroid per run:
// float sum / count (CentroidPoint's AccumulatorXYZ).  Returns the output
// count, or -1 when the grid overflows an int (the reference then copies
// the input unchanged).
int oref_voxel_grid(const float* xyz, int n, float leaf, float* out) {
  const float inv = 1.0f / leaf;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  bool any = false;
  for (int i = 0; i < n; ++i) {
    const float* p = xyz + 3 * i;
    if (!(std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2]))) continue;
    any = true;
    for (int a = 0; a < 3; ++a) {
      mn[a] = std::min(mn[a], p[a]);
      mx[a] = std::max(mx[a], p[a]);
    }
  }
  if (!any) return 0;
  long long d[3];
  for (int a = 0; a < 3; ++a) d[a] = static_cast<long long>((mx[a] - mn[a]) * inv) + 1;
  if ((d[0] * d[1] * d[2]) > static_cast<long long>(std::numeric_limits<int>::max())) return -1;
  int minb[3], divb[3];
  for (int a = 0; a < 3; ++a) {
    minb[a] = static_cast<int>(std::floor(mn[a] * inv));
    const int maxb = static_cast<int>(std::floor(mx[a] * inv));
    divb[a] = maxb - minb[a] + 1;
  }
  const int mul[3] = {1, divb[0], divb[0] * divb[1]};
  struct Idx {
    unsigned idx, pt;
    bool operator<(const Idx& o) const { return idx < o.idx; }
  };
  std::vector<Idx> v;
  v.reserve(n);
  for (int i = 0; i < n; ++i) {
    const float* p = xyz + 3 * i;
    if (!(std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2]))) continue;
    int ijk[3];
    for (int a = 0; a < 3; ++a) ijk[a] = static_cast<int>(std::floor(p[a] * inv) - static_cast<float>(minb[a]));
    v.push_back({static_cast<unsigned>(ijk[0] * mul[0] + ijk[1] * mul[1] + ijk[2] * mul[2]), (unsigned)i});
  }
  std::sort(v.begin(), v.end(), std::less<Idx>());
  int m = 0;
  size_t k = 0;
  while (k < v.size()) {
    size_t e = k + 1;
    while (e < v.size() && v[e].idx == v[k].idx) ++e;
    float sx = 0.f, sy = 0.f, sz = 0.f;
    for (size_t q = k; q < e; ++q) {
      const float* p = xyz + 3 * v[q].pt;
      sx += p[0];
      sy += p[1];
      sz += p[2];
    }
    const float c = static_cast<float>(e - k);
    out[3 * m] = sx / c;
    out[3 * m + 1] = sy / c;
    out[3 * m + 2] = sz / c;
    ++m;
    k = e;
  }
  return m;
}

// Known-answer helpers
void oref_so3_exp(const double* w, double* R9) { oref::so3_exp(w, R9); }
void oref_ldlt_solve6(const double* A, const double* b, double* x) { oref::ldlt_solve6(A, b, x); }
void oref_regularize(const double* C9, int method, double* out9) { oref::regularize(C9, method, out9); }
int oref_max_threads(void) { return oref::omp_threads(0); }

}  // extern "C"
