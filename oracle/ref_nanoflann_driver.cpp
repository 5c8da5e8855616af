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
#include <functional>
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
// the built tree (tests): vind, and the nodes in preorder (the order
// divideTree allocates them): (child1, child2, divfeat, -1) with preorder
// child indices, or (left, right, -1, -1) for a leaf; (divlow, divhigh).
// Returns the node count (-1: cap too small).
int ref_tree_export(void* h, int* vind, int* nodes4, float* div2, int cap) {
  auto* t = static_cast<Handle*>(h);
  for (size_t i = 0; i < t->tree.vind.size(); ++i) vind[i] = t->tree.vind[i];
  int next = 0;
  bool ok = true;
  std::function<int(Tree::NodePtr)> walk = [&](Tree::NodePtr nd) -> int {
    const int id = next++;
    if (id >= cap) {
      ok = false;
      return id;
    }
    nodes4[4 * id + 3] = -1;
    if (!nd->child1 && !nd->child2) {
      nodes4[4 * id] = (int)nd->node_type.lr.left;
      nodes4[4 * id + 1] = (int)nd->node_type.lr.right;
      nodes4[4 * id + 2] = -1;
      div2[2 * id] = div2[2 * id + 1] = 0.f;
      return id;
    }
    nodes4[4 * id + 2] = nd->node_type.sub.divfeat;
    div2[2 * id] = nd->node_type.sub.divlow;
    div2[2 * id + 1] = nd->node_type.sub.divhigh;
    const int c1 = walk(nd->child1);
    const int c2 = walk(nd->child2);
    if (ok) {
      nodes4[4 * id] = c1;
      nodes4[4 * id + 1] = c2;
    }
    return id;
  };
  walk(t->tree.root_node);
  return ok ? next : -1;
}
}
