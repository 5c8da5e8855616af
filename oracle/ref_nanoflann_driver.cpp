/*
 * oracle/ref_nanoflann_driver.cpp — TEST INFRASTRUCTURE ONLY.
 *
 * Thin C driver around the reference's OWN vendored nanoflann
 * (dynamic_direct_lidar_odometry/include/nano_gicp/impl/nanoflann_impl.hpp,
 * STL-only), included from /root/reference where it lies (see
 * oracle/Makefile; nothing of the reference is copied into this repo).  It
 * instantiates exactly the type the reference uses,
 *   KDTreeSingleIndexAdaptor<SO3_Adaptor<float, Adaptor>, Adaptor, 3, int>
 * with KDTreeSingleIndexAdaptorParams(100)  (nanoflann.hpp:119,134,186-196),
 * and queries it the way KdTreeFLANN::nearestKSearch does (nanoflann.hpp:
 * 145-156): KNNResultSet<float,int>, default SearchParams.  The output
 * library lands in oracle/_ref/ (git-ignored) and is used only to pin the
 * oracle's kd-tree restatement and to generate tests/golden fixtures.
 */
#include <cstddef>
#include <vector>

#include "nano_gicp/impl/nanoflann_impl.hpp"

namespace {
struct FlatCloud {
  const float* p;
  size_t n;
  inline size_t kdtree_get_point_count() const { return n; }
  inline float kdtree_get_pt(const size_t idx, int dim) const { return p[3 * idx + dim]; }
  template <class BBOX>
  bool kdtree_get_bbox(BBOX&) const { return false; }  // as PointCloud_Adaptor
};
using Tree = nanoflann::KDTreeSingleIndexAdaptor<nanoflann::SO3_Adaptor<float, FlatCloud>, FlatCloud, 3, int>;
struct Handle {
  FlatCloud cloud;
  Tree tree;
  Handle(const float* p, size_t n) : cloud{p, n}, tree(3, cloud, nanoflann::KDTreeSingleIndexAdaptorParams(100)) {
    tree.buildIndex();
  }
};
}  // namespace

extern "C" {
void* ref_tree_build(const float* xyz, int n) { return new Handle(xyz, (size_t)n); }
void ref_tree_free(void* h) { delete static_cast<Handle*>(h); }
int ref_tree_knn(void* h, const float* q, int nq, int k, int* idx, float* d) {
  auto* t = static_cast<Handle*>(h);
#pragma omp parallel for schedule(guided, 8)
  for (int i = 0; i < nq; ++i) {
    nanoflann::KNNResultSet<float, int> rs(k);
    rs.init(&idx[(size_t)i * k], &d[(size_t)i * k]);
    t->tree.findNeighbors(rs, &q[3 * i], nanoflann::SearchParams());
  }
  return 0;
}
}
