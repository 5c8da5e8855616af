// tests/cpp/oracle_san.cpp — TEST INFRASTRUCTURE: drives the CPU oracle
// (oracle/cpu_ref.cpp) through every entry point under AddressSanitizer +
// UndefinedBehaviorSanitizer (SURVEY.md §5 "Race detection / sanitizers";
// built by `make -C oracle san`, run by tests/test_oracle_san.py).  Exit code
// 0 and no sanitizer report = clean.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/ddlo_gicp.h"

extern "C" {
struct oref_gicp;
void* oref_tree_build(const float* xyz, int n);
void oref_tree_free(void* t);
int oref_tree_export(void* t, int* vind, int* nodes4, float* div2, int cap);
int oref_tree_knn(void* th, const float* q, int nq, int k, int* idx, float* d, int nthreads);
int oref_covariances(const float* xyz, int n, int k, int reg, double* out6, int nthreads);
oref_gicp* oref_gicp_create(const gicp_params* p, const float* src, int ns, const float* tgt, int nt, int nthreads);
void oref_gicp_free(oref_gicp* h);
int oref_gicp_compute_covariances(oref_gicp* h, int side);
int oref_gicp_get_covariances(oref_gicp* h, int side, double* out6);
int oref_gicp_align(oref_gicp* h, const float* guess16, float* out16, gicp_result* res);
int oref_gicp_linearize(oref_gicp* h, const double* pose16, double* H36, double* b6, double* cost, int* corr, float* sqd);
double oref_gicp_compute_error(oref_gicp* h, const double* pose16);
int oref_gicp_last_correspondences(oref_gicp* h, int* corr, float* sqd);
int oref_gicp_trace(oref_gicp* h, double* out, int max_entries);
int oref_voxel_grid(const float* xyz, int n, float leaf, float* out);
void oref_so3_exp(const double* w, double* R9);
void oref_ldlt_solve6(const double* A, const double* b, double* x);
void oref_regularize(const double* C9, int method, double* out9);
}

static std::vector<float> cloud(int n, unsigned seed, float sx, float sy, float sz) {
  std::mt19937 g(seed);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> p(3 * (size_t)n);
  for (int i = 0; i < n; ++i) {
    p[3 * i] = sx * nd(g);
    p[3 * i + 1] = sy * nd(g);
    p[3 * i + 2] = sz * nd(g);
  }
  return p;
}

int main() {
  int fails = 0;
  // kd-tree on ragged sizes, duplicates and a lattice
  for (int n : {1, 7, 100, 101, 5000}) {
    std::vector<float> p = cloud(n, 1 + n, 10, 10, 2);
    if (n == 5000)
      for (int i = 0; i < 1000; ++i) std::memcpy(&p[3 * (size_t)(i + 2000)], &p[3 * (size_t)i], 12);   // duplicates
    void* t = oref_tree_build(p.data(), n);
    const int k = n < 10 ? n : 10;
    std::vector<int> idx((size_t)n * k);
    std::vector<float> d((size_t)n * k);
    oref_tree_knn(t, p.data(), n, k, idx.data(), d.data(), 2);
    std::vector<int> vind(n), nodes(4 * (2 * (size_t)n + 2));
    std::vector<float> div(2 * (2 * (size_t)n + 2));
    if (oref_tree_export(t, vind.data(), nodes.data(), div.data(), 2 * n + 2) <= 0) ++fails;
    oref_tree_free(t);
  }
  std::vector<float> lat;
  for (int x = 0; x < 12; ++x)
    for (int y = 0; y < 12; ++y)
      for (int z = 0; z < 4; ++z) {
        lat.push_back((float)x);
        lat.push_back((float)y);
        lat.push_back((float)z);
      }
  const int nl = (int)lat.size() / 3;
  for (int reg = 0; reg < 5; ++reg) {
    std::vector<double> cov(6 * (size_t)nl);
    if (oref_covariances(lat.data(), nl, 10, reg, cov.data(), 2)) ++fails;
  }
  // GICP: LM and GN, linearize, error, residual plumbing
  std::vector<float> tgt = cloud(4000, 11, 15, 15, 3), src(tgt);
  for (size_t i = 0; i < src.size(); i += 3) {
    src[i] += 0.2f;
    src[i + 1] -= 0.1f;
  }
  for (int opt = 0; opt < 2; ++opt) {
    gicp_params p;
    std::memset(&p, 0, sizeof(p));
    p.k_correspondences = 10;
    p.max_iterations = 16;
    p.max_correspondence_distance = 1.0;
    p.transformation_epsilon = 5e-4;
    p.rotation_epsilon = 2e-3;
    p.lm_init_lambda_factor = 1e-9;
    p.regularization = 3;
    p.optimizer = opt;
    p.lm_max_iterations = 10;
    oref_gicp* h = oref_gicp_create(&p, src.data(), 4000, tgt.data(), 4000, 2);
    oref_gicp_compute_covariances(h, 0);
    oref_gicp_compute_covariances(h, 1);
    std::vector<double> c6(6 * 4000);
    oref_gicp_get_covariances(h, 0, c6.data());
    float out[16];
    gicp_result res;
    std::memset(&res, 0, sizeof(res));
    oref_gicp_align(h, nullptr, out, &res);
    if (!(std::fabs(out[3] + 0.2f) < 0.05f)) ++fails;
    double pose[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    double H[36], b[6], cost;
    std::vector<int> corr(4000);
    std::vector<float> sqd(4000);
    oref_gicp_linearize(h, pose, H, b, &cost, corr.data(), sqd.data());
    (void)oref_gicp_compute_error(h, pose);
    oref_gicp_last_correspondences(h, corr.data(), sqd.data());
    std::vector<double> tr(64 * 64);
    oref_gicp_trace(h, tr.data(), 64);
    oref_gicp_free(h);
  }
  std::vector<float> vox(3 * 4000);
  if (oref_voxel_grid(tgt.data(), 4000, 0.5f, vox.data()) <= 0) ++fails;
  const double w[3] = {0.1, -0.2, 0.05};
  double R[9], C9[9] = {2, 0.1, 0, 0.1, 1, 0, 0, 0, 1e-4}, o9[9];
  oref_so3_exp(w, R);
  double A[36] = {0}, bb[6] = {1, 2, 3, 4, 5, 6}, x[6];
  for (int i = 0; i < 6; ++i) A[7 * i] = 2.0 + i;
  oref_ldlt_solve6(A, bb, x);
  for (int m = 0; m < 5; ++m) oref_regularize(C9, m, o9);
  std::printf("oracle sanitizer run: %s\n", fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}
