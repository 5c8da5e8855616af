/*
 * ddlo_odom.h — C-ABI of the odometry driver around the GICP core
 * (with the device voxel filter of rank 3).
 *
 * One ddlo_odom == the registration half of OdomNode (reference
 * dynamic_direct_lidar_odometry/src/odometry/odom.cc): per scan the
 * preprocessing (crop box + voxel filter, odom.cc:442-478), the spaciousness
 * metric and adaptive keyframe threshold (:981-1001, :1156-1178), S2S then
 * S2M registration with pose propagation (:745-851, :921-939), keyframe
 * selection (:1067-1154) and submap assembly from the k nearest / convex-hull
 * / concave-hull keyframes (:1180-1315).  Everything that touches points —
 * scans, keyframe clouds, their covariances and the submap — stays in device
 * memory; the host keeps only poses and index lists.
 *
 * Not restated (outside the GICP path): ROS I/O, IMU gravity
 * alignment, the organized-cloud row/col downsampling filter, dynamic-object
 * detection and tracking, publishing and trajectory files.
 */
#ifndef DDLO_ODOM_H
#define DDLO_ODOM_H

#include "ddlo_gicp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* OdomNode parameters (odom.cc:196-252; defaults = cfg/ddlo.yaml:158-204). */
typedef struct ddlo_odom_params {
  gicp_params s2s;                 /* odomNode/gicp/s2s/... (k 10, maxCorr 1.0, maxIter 32, transEps 0.01) */
  gicp_params s2m;                 /* odomNode/gicp/s2m/... (k 20, maxCorr 2.0, maxIter 32, transEps 0.01) */
  int32_t min_num_points;          /* odomNode/gicp/minNumPoints (10): smaller scans are skipped (:635-639) */
  double keyframe_thresh_dist;     /* odomNode/keyframe/threshD (1.0 m); replaced every scan when adaptive */
  double keyframe_thresh_rot;      /* odomNode/keyframe/threshR (0.1 deg) */
  int32_t submap_knn;              /* odomNode/submap/keyframe/knn (10) */
  int32_t submap_kcv;              /* .../kcv (10) */
  int32_t submap_kcc;              /* .../kcc (10) */
  int32_t adaptive;                /* 1 = setAdaptiveParams every scan (the reference always does) */
  int32_t crop_use;                /* preprocessing/cropBoxFilter/use (1) */
  double crop_size;                /* .../size (1.0 m): points inside [-s, s]^3 are removed */
  int32_t vf_scan_use;             /* preprocessing/voxelFilter/scan/use (1) */
  double vf_scan_res;              /* .../res (0.1 m) */
  int32_t vf_submap_use;           /* preprocessing/voxelFilter/submap/use (1): applied to keyframes */
  double vf_submap_res;            /* .../res (0.1 m) */
  int32_t skip_first_scan;         /* 1 (reference): the first scan with >= min_num_points points only
                                      initialises (initializeDDLO, odom.cc:641-646), so keyframe 0 is
                                      the second one; 0: the first scan becomes the target at once */
  int32_t s2m_target_grid;         /* candidate cells of the S2M submap (gicp_set_target_grid): 0 off
                                      (default: a submap lives ~20 scans, fewer than the build pays for),
                                      1 auto, 2 on */
} ddlo_odom_params;

typedef enum ddlo_odom_status {
  DDLO_ODOM_TRACKED = 0,   /* S2S + S2M ran, the pose was updated               */
  DDLO_ODOM_FIRST = 1,     /* first scan: became the S2S target and keyframe 0 */
  DDLO_ODOM_SKIPPED = 2,   /* fewer than min_num_points points (reference: return) */
  DDLO_ODOM_INIT = 3       /* consumed by the initialisation (initializeDDLO, odom.cc:641-646) */
} ddlo_odom_status;

typedef struct ddlo_odom_result {
  int32_t status;                  /* ddlo_odom_status */
  int32_t scan_points;             /* points after preprocessing */
  float T[16];                     /* T_: global pose after S2M (row-major) */
  float T_s2s[16];                 /* T_s2s_: global S2S estimate (the S2M guess) */
  float T_s2s_local[16];           /* T_S2S: scan-to-scan transform */
  gicp_result s2s;
  gicp_result s2m;
  int32_t keyframe_added;          /* updateKeyframes appended a keyframe */
  int32_t submap_changed;          /* submap_hasChanged_ */
  int32_t num_keyframes;
  int32_t submap_keyframes;        /* keyframes in the current submap */
  int64_t submap_points;
  double spaciousness;             /* metrics_.spaciousness.back() */
  double keyframe_thresh_dist;     /* the threshold in effect for this scan */
} ddlo_odom_result;

gicp_status ddlo_odom_default_params(ddlo_odom_params* out);
gicp_status ddlo_odom_create(int device, const ddlo_odom_params* p, struct ddlo_odom** out);
gicp_status ddlo_odom_destroy(struct ddlo_odom* o);
/* OdomNode::icpCB for one scan (odom.cc:614-729, registration part).  xyz:
 * float x, y, z of point 0, consecutive points stride_bytes apart; copied.
 * A keyframe whose submap-voxel-filtered cloud has fewer points than the S2S
 * k gets covariances from all of its points (the reference reads
 * uninitialised neighbour slots there, nanoflann.hpp:149-155).  An error
 * return leaves the driver unusable: destroy it. */
gicp_status ddlo_odom_process(struct ddlo_odom* o, const float* xyz, size_t n, size_t stride_bytes,
                              ddlo_odom_result* res);
/* Keyframe k: world pose (x, y, z, qx, qy, qz, qw as the reference's pose_ /
 * rotq_) and its point count (after the submap voxel filter). */
gicp_status ddlo_odom_keyframe(const struct ddlo_odom* o, int k, float pose7[7], size_t* npoints);
/* Keyframe indices of the current submap (sorted, submap_kf_idx_prev_). */
gicp_status ddlo_odom_submap(const struct ddlo_odom* o, int32_t* idx, size_t cap, size_t* n);
/* The S2S (which = 0) or S2M (which = 1) GICP context, for the gicp_* getters
 * (residuals, residual image, correspondences) of the last scan. */
gicp_status ddlo_odom_ctx(struct ddlo_odom* o, int which, struct gicp_ctx** ctx);
/* Device preprocessing on its own (tests, benchmarks): crop box (crop_size
 * > 0) then voxel filter (leaf > 0) of n points; writes the surviving points
 * (x, y, z float, 12 B each) to out and their count to *nout (cap = capacity
 * of out in points). */
gicp_status ddlo_preprocess(int device, const float* xyz, size_t n, size_t stride_bytes, double crop_size, double leaf,
                            float* out, size_t cap, size_t* nout);

/* Hull keyframe selection (OdomNode::computeConvexHull / computeConcaveHull,
 * odom.cc:1003-1065, pcl::ConvexHull / pcl::ConcaveHull with setDimension(3),
 * odom.cc:87-88, over the keyframe positions): indices of the input points on
 * the hull, ascending.  Convex: qhull's 3-D vertex set, empty for fewer than
 * 4 or coplanar points (qhull's flat-simplex error).  Concave: the vertices
 * of the 3-D alpha shape's boundary triangles (Delaunay triangles of
 * circumradius <= alpha not enclosed by two tetrahedra of circumradius <=
 * alpha).  idx receives at most cap indices; *nidx = the hull's size (it may
 * exceed cap).  Exposed for the tests. */
gicp_status ddlo_convex_hull(const float* xyz, int n, int32_t* idx, int cap, int* nidx);
gicp_status ddlo_concave_hull(const float* xyz, int n, double alpha, int32_t* idx, int cap, int* nidx);

#ifdef __cplusplus
}
#endif

#endif /* DDLO_ODOM_H */
