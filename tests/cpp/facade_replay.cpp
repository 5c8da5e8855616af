// tests/cpp/facade_replay.cpp — replays OdomNode's per-scan call sequence
// into the NanoGICP C++ facade (reference src/odometry/odom.cc:480-532,
// 745-793) on frames written by tests/test_facade.py, and prints the S2S and
// S2M poses of every frame.  The Python test compares them with the CPU
// oracle driven through the same sequence.
//
// Input (binary, little endian):
//   int32 nframes; per frame: int32 n; float32 xyz[n][3]
//   int32 nsub; float32 xyz[nsub][3]; float64 cov6[nsub][6]   (S2M target)
// Output (stdout): per frame "frame <i> s2s <16 floats> s2m <16 floats>"
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <vector>

#include "nano_gicp/nano_gicp.hpp"

using ddlo::PointXYZI;
using Cloud = ddlo::PointCloud<PointXYZI>;

static Cloud::Ptr read_cloud(std::ifstream& f) {
  int32_t n = 0;
  f.read(reinterpret_cast<char*>(&n), 4);
  std::vector<float> xyz(3 * (size_t)n);
  f.read(reinterpret_cast<char*>(xyz.data()), 12 * (size_t)n);
  auto c = std::make_shared<Cloud>();
  c->points.resize(n);
  for (int i = 0; i < n; ++i) {
    c->points[i].x = xyz[3 * i];
    c->points[i].y = xyz[3 * i + 1];
    c->points[i].z = xyz[3 * i + 2];
  }
  return c;
}

static void print(const char* tag, const ddlo::Matrix4f& T) {
  std::printf(" %s", tag);
  for (int i = 0; i < 16; ++i) std::printf(" %.9g", T.m[i]);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s frames.bin\n", argv[0]);
    return 2;
  }
  std::ifstream f(argv[1], std::ios::binary);
  int32_t nframes = 0;
  f.read(reinterpret_cast<char*>(&nframes), 4);
  std::vector<Cloud::Ptr> frames;
  for (int i = 0; i < nframes; ++i) frames.push_back(read_cloud(f));
  Cloud::Ptr submap = read_cloud(f);
  std::vector<double> cov6(6 * submap->size());
  f.read(reinterpret_cast<char*>(cov6.data()), 8 * cov6.size());
  ddlo::CovarianceList subcov(submap->size());
  for (size_t i = 0; i < submap->size(); ++i) {
    const double* c = &cov6[6 * i];
    ddlo::Matrix4d& m = subcov[i];
    m(0, 0) = c[0]; m(0, 1) = c[1]; m(0, 2) = c[2];
    m(1, 0) = c[1]; m(1, 1) = c[3]; m(1, 2) = c[4];
    m(2, 0) = c[2]; m(2, 1) = c[4]; m(2, 2) = c[5];
  }

  try {
    // OdomNode constructor (odom.cc:92-112) with ddlo.yaml GICP values
    ddlo::NanoGICP<PointXYZI, PointXYZI> s2s, s2m;
    s2s.setCorrespondenceRandomness(10);
    s2s.setMaxCorrespondenceDistance(1.0);
    s2s.setMaximumIterations(32);
    s2s.setTransformationEpsilon(0.01);
    s2s.setEuclideanFitnessEpsilon(0.01);
    s2s.setRANSACIterations(5);
    s2s.setRANSACOutlierRejectionThreshold(1.0);
    s2m.setCorrespondenceRandomness(20);
    s2m.setMaxCorrespondenceDistance(2.0);
    s2m.setMaximumIterations(32);
    s2m.setTransformationEpsilon(0.01);
    // first scan: initializeInputTarget (odom.cc:487-488)
    s2s.setInputTarget(frames[0]);
    s2s.calculateTargetCovariances();
    // S2M target: the submap and its covariances (odom.cc:780-783)
    s2m.setInputTarget(submap);
    s2m.setTargetCovariances(subcov);
    ddlo::Matrix4f T_prev = ddlo::Matrix4f::Identity();
    for (int i = 1; i < nframes; ++i) {
      // setInputSources (odom.cc:518-532)
      s2s.setInputSource(frames[i]);
      s2m.registerInputSource(frames[i]);
      // scanMatching (odom.cc:754-787)
      Cloud aligned;
      s2s.align(aligned);
      const ddlo::Matrix4f T_s2s = s2s.getFinalTransformation();
      s2m.shareSourceFrom(s2s);  // source_kdtree_ alias + source_covs_ copy (:530, :765)
      s2s.swapSourceAndTarget();
      // guess = T_prev * T_S2S (propagateS2S, odom.cc:921-939)
      ddlo::Matrix4f guess;
      for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
          float s = 0.f;
          for (int k = 0; k < 4; ++k) s += T_prev(r, k) * T_s2s(k, c);
          guess(r, c) = s;
        }
      s2m.align(aligned, guess);
      const ddlo::Matrix4f T = s2m.getFinalTransformation();
      std::vector<double> residuals;
      s2m.getResiduals(residuals, T);
      std::printf("frame %d", i);
      print("s2s", T_s2s);
      print("s2m", T);
      std::printf(" nres %zu\n", residuals.size());
      T_prev = T;
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "facade_replay: %s\n", e.what());
    return 1;
  }
  return 0;
}
