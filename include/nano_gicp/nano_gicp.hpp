// nano_gicp/nano_gicp.hpp — drop-in C++ facade of the MI355X GICP core.
//
// Mirrors the surface OdomNode uses of the reference's
// nano_gicp::NanoGICP<PointXYZI, PointXYZI> (reference
// include/nano_gicp/nano_gicp.hpp:58-148, lsq_registration.hpp:60-128, and
// the pcl::Registration calls at src/odometry/odom.cc:92-112,518-532,745-851)
// on top of the C-ABI in ddlo_gicp.h.  PCL-free: clouds are ddlo::PointCloud
// of 32-byte points laid out like pcl::PointXYZI (x, y, z, pad, intensity,
// pad[3]), so a pcl::PointCloud<pcl::PointXYZI> can be handed over by
// pointer+stride without copying.
//
// Semantics kept from the reference:
//   * setInputSource / setInputTarget early-out on pointer identity
//     (nano_gicp_impl.hpp:125,135,148) and clear that side's covariances;
//   * computeTransformation computes missing covariances (:186-193);
//   * swapSourceAndTarget swaps clouds, indices and covariances (:97-106);
//   * LM failure prints "lm not converged!!" and keeps the last pose
//     (lsq_registration_impl.hpp:115-119);
//   * getResiduals returns sqrt of the 1-NN squared distances of the last
//     linearization (:225-232).
// The reference's public members source_kdtree_ / source_covs_ that OdomNode
// assigns across instances (odom.cc:530,765) are replaced by
// shareSourceFrom(other): the device cloud, index and covariances are shared
// (copy-on-write) instead of copied.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <iostream>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "../ddlo_gicp.h"

namespace ddlo {

struct alignas(16) PointXYZI {  // byte layout of pcl::PointXYZI
  float x = 0.f, y = 0.f, z = 0.f, pad0 = 1.f;
  float intensity = 0.f, pad1 = 0.f, pad2 = 0.f, pad3 = 0.f;
};
static_assert(sizeof(PointXYZI) == 32, "PointXYZI must be 32 bytes like pcl::PointXYZI");

template <class PointT>
struct PointCloud {
  using Ptr = std::shared_ptr<PointCloud>;
  using ConstPtr = std::shared_ptr<const PointCloud>;
  std::vector<PointT> points;
  std::size_t size() const { return points.size(); }
  bool empty() const { return points.empty(); }
  const PointT& at(std::size_t i) const { return points.at(i); }
  PointT& at(std::size_t i) { return points.at(i); }
};

// Row-major 4x4 matrices standing in for Eigen::Matrix4f / Matrix4d.
struct Matrix4f {
  std::array<float, 16> m{1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  float& operator()(int r, int c) { return m[4 * r + c]; }
  float operator()(int r, int c) const { return m[4 * r + c]; }
  static Matrix4f Identity() { return Matrix4f(); }
  const float* data() const { return m.data(); }
  float* data() { return m.data(); }
};
struct Matrix4d {
  std::array<double, 16> m{};
  double& operator()(int r, int c) { return m[4 * r + c]; }
  double operator()(int r, int c) const { return m[4 * r + c]; }
};
struct Matrix6d {
  std::array<double, 36> m{};
  double operator()(int r, int c) const { return m[6 * r + c]; }
};
using CovarianceList = std::vector<Matrix4d>;

// Same enumerators as nano_gicp::RegularizationMethod (gicp/gicp_settings.hpp:47-54).
enum class RegularizationMethod { NONE, MIN_EIG, NORMALIZED_MIN_EIG, PLANE, FROBENIUS };

class GicpError : public std::runtime_error {
 public:
  GicpError(gicp_status s, const std::string& what) : std::runtime_error(what), status(s) {}
  gicp_status status;
};

namespace detail {
inline void check(gicp_status s, const char* where) {
  if (s != GICP_OK) throw GicpError(s, std::string(where) + ": " + gicp_last_error());
}
struct CtxDeleter {
  void operator()(gicp_ctx* c) const { gicp_ctx_destroy(c); }
};
}  // namespace detail

template <typename PointSource, typename PointTarget>
class NanoGICP {
 public:
  using PointCloudSource = PointCloud<PointSource>;
  using PointCloudSourceConstPtr = typename PointCloudSource::ConstPtr;
  using PointCloudTarget = PointCloud<PointTarget>;
  using PointCloudTargetConstPtr = typename PointCloudTarget::ConstPtr;

  explicit NanoGICP(int device = 0) {
    gicp_ctx* c = nullptr;
    detail::check(gicp_ctx_create(device, &c), "gicp_ctx_create");
    ctx_.reset(c);
    detail::check(gicp_default_params(&params_), "gicp_default_params");
  }

  // --- setters used by OdomNode (odom.cc:92-112) ---------------------------
  void setCorrespondenceRandomness(int k) { params_.k_correspondences = k; push(); }
  void setMaxCorrespondenceDistance(double d) { params_.max_correspondence_distance = d; push(); }
  void setMaximumIterations(int n) { params_.max_iterations = n; push(); }
  void setTransformationEpsilon(double e) { params_.transformation_epsilon = e; push(); }
  void setRotationEpsilon(double e) { params_.rotation_epsilon = e; push(); }
  void setInitialLambdaFactor(double f) { params_.lm_init_lambda_factor = f; push(); }
  void setRegularizationMethod(RegularizationMethod m) { params_.regularization = (int32_t)m; push(); }
  // Accepted and ignored, as in NanoGICP:
  void setEuclideanFitnessEpsilon(double) {}
  void setRANSACIterations(int) {}
  void setRANSACOutlierRejectionThreshold(double) {}
  template <class T> void setSearchMethodSource(const T&, bool = false) {}
  template <class T> void setSearchMethodTarget(const T&, bool = false) {}
  void setNumThreads(int) {}
  void setDebugPrint(bool) {}
  // Extensions (benchmarks / cfg 2): Gauss-Newton and fixed iteration counts.
  void setOptimizer(gicp_optimizer o) { params_.optimizer = o; push(); }
  void setFixedIterations(int n) { params_.fixed_iterations = n; push(); }

  // --- clouds ---------------------------------------------------------------
  void setInputSource(const PointCloudSourceConstPtr& cloud) { set_source(cloud, 1); }
  void registerInputSource(const PointCloudSourceConstPtr& cloud) { set_source(cloud, 0); }
  void setInputTarget(const PointCloudTargetConstPtr& cloud) {
    if (target_ == cloud) return;
    detail::check(gicp_set_target(ctx_.get(), first_xyz(*cloud), cloud->size(), sizeof(PointTarget)),
                  "gicp_set_target");
    target_ = cloud;
  }
  void clearSource() { detail::check(gicp_clear_source(ctx_.get()), "gicp_clear_source"); input_.reset(); }
  void clearTarget() { detail::check(gicp_clear_target(ctx_.get()), "gicp_clear_target"); target_.reset(); }

  void swapSourceAndTarget() {
    static_assert(std::is_same<PointSource, PointTarget>::value,
                  "swapSourceAndTarget needs identical point types (as NanoGICP<PointXYZI, PointXYZI>)");
    detail::check(gicp_swap_source_target(ctx_.get()), "gicp_swap_source_target");
    std::swap(input_, target_);
  }
  // replaces `other_gicp.source_kdtree_ = this->source_kdtree_` and the
  // source_covs_ copy OdomNode performs (odom.cc:530,765)
  void shareSourceFrom(const NanoGICP& other) {
    detail::check(gicp_share_source(ctx_.get(), other.ctx_.get()), "gicp_share_source");
    input_ = other.input_;
  }

  // --- covariances ----------------------------------------------------------
  bool calculateSourceCovariances() {
    detail::check(gicp_compute_covariances(ctx_.get(), GICP_SIDE_SOURCE), "gicp_compute_covariances");
    return true;
  }
  bool calculateTargetCovariances() {
    detail::check(gicp_compute_covariances(ctx_.get(), GICP_SIDE_TARGET), "gicp_compute_covariances");
    return true;
  }
  void setSourceCovariances(const CovarianceList& covs) { set_covs(GICP_SIDE_SOURCE, covs); }
  void setTargetCovariances(const CovarianceList& covs) { set_covs(GICP_SIDE_TARGET, covs); }
  CovarianceList getSourceCovariances() const { return get_covs(GICP_SIDE_SOURCE); }
  CovarianceList getTargetCovariances() const { return get_covs(GICP_SIDE_TARGET); }

  // --- registration (pcl::Registration::align) ------------------------------
  void align(PointCloudSource& output) { align(output, Matrix4f::Identity()); }
  void align(PointCloudSource& output, const Matrix4f& guess) {
    gicp_result res;
    detail::check(gicp_align(ctx_.get(), guess.data(), final_.data(), &res), "gicp_align");
    result_ = res;
    if (res.lm_failed) std::cerr << "lm not converged!!" << std::endl;
    // output = transformPointCloud(*input_, final_transformation_)
    output = *input_;
    if (!output.points.empty())
      detail::check(gicp_transform_source(ctx_.get(), &output.points[0].x, output.size(), sizeof(PointSource)),
                    "gicp_transform_source");
  }
  Matrix4f getFinalTransformation() const { return final_; }
  bool hasConverged() const { return result_.converged != 0; }
  int getNumIterations() const { return result_.nr_iterations; }
  Matrix6d getFinalHessian() const {
    Matrix6d h;
    std::memcpy(h.m.data(), result_.final_hessian, sizeof(h.m));
    return h;
  }
  const gicp_result& lastResult() const { return result_; }

  void getResiduals(std::vector<double>& residuals, const Matrix4f& /*trans: ignored, as in the reference*/ = {}) {
    residuals.resize(input_ ? input_->size() : 0);
    if (residuals.empty()) return;
    detail::check(gicp_get_residuals(ctx_.get(), residuals.data(), residuals.size()), "gicp_get_residuals");
  }

  gicp_ctx* ctx() const { return ctx_.get(); }

 private:
  template <class P>
  static const float* first_xyz(const PointCloud<P>& c) { return c.points.empty() ? nullptr : &c.points[0].x; }

  void push() { detail::check(gicp_set_params(ctx_.get(), &params_), "gicp_set_params"); }
  void set_source(const PointCloudSourceConstPtr& cloud, int build) {
    if (input_ == cloud) return;  // pointer identity early-out (:125,135)
    detail::check(gicp_set_source(ctx_.get(), first_xyz(*cloud), cloud->size(), sizeof(PointSource), build),
                  "gicp_set_source");
    input_ = cloud;
  }
  void set_covs(int side, const CovarianceList& covs) {
    detail::check(gicp_set_covariances(ctx_.get(), side, covs.empty() ? nullptr : covs[0].m.data(), covs.size(),
                                       GICP_COV_MAT4D),
                  "gicp_set_covariances");
  }
  CovarianceList get_covs(int side) const {
    std::size_t n = 0;
    detail::check(gicp_get_size(ctx_.get(), side, &n), "gicp_get_size");
    CovarianceList out(n);
    if (n) detail::check(gicp_get_covariances(ctx_.get(), side, out[0].m.data(), n, GICP_COV_MAT4D), "gicp_get_covariances");
    return out;
  }

  std::unique_ptr<gicp_ctx, detail::CtxDeleter> ctx_;
  gicp_params params_{};
  gicp_result result_{};
  Matrix4f final_;
  PointCloudSourceConstPtr input_;
  PointCloudTargetConstPtr target_;
};

}  // namespace ddlo
