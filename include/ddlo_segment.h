/*
 * ddlo_segment.h — C-ABI of the range-image segmentation that feeds DDLO's
 * dynamic-object detection (host-side per the north
 * star; the per-pixel passes run on the device, the order-dependent labelling
 * on the host).
 *
 * Replaces DetectionModule (reference
 * dynamic_direct_lidar_odometry/src/detection/detection.cpp,
 * include/detection/detection.h) for the calls OdomNode::applySegmentation
 * makes (odom.cc:853-857):
 *   ddlo_seg_create    DetectionModule ctor: loadParams :72-129 + allocateMemory :131-159
 *   ddlo_seg_process   projectScan :254-382 (range image of the transformed organized
 *                      cloud, measured from the sensor position T(0:3, 3)),
 *                      projectResiduals :203-252 (the residual image is an input:
 *                      gicp_residual_image, ddlo_gicp.h, produces it),
 *                      groundRemoval :448-508, cloudSegmentation :510-542 and
 *                      labelComponents :544-724
 *   ddlo_seg_ground_indices   getGroundIndices :1002-1013
 *   ddlo_seg_label_indices    label_indices_i_ (cloudSegmentation :524-538)
 *   ddlo_seg_label     labelComponents over caller-provided images (host only)
 *
 * Bounding boxes, tracking, visualisation and evaluation (computeAllObjects,
 * trackDetections, visualize, evaluate) are outside the registration path and
 * not restated.
 */
#ifndef DDLO_SEGMENT_H
#define DDLO_SEGMENT_H

#include "ddlo_gicp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* DetectionModule::loadParams (detection.cpp:72-129) with the member types of
   detection.h:60-85.  ddlo_seg_default_params gives the code's defaults;
   note that ROS reads ang_bottom, groundAngleThreshold, minimumRange,
   sensorMountAngle and maxDistance as int (their defaults are int literals),
   so yaml values such as minimumRange: 0.3 arrive rounded (to 0). */
typedef struct ddlo_seg_params {
  int32_t rows;                    /* odomNode/detection/rows (128): H_ */
  int32_t cols;                    /* .../columns (1024): W_ */
  float ang_bottom;                /* .../ang_bottom (45): ang_res_y = 2 ang_bottom / float(H - 1) */
  int32_t ground_rows;             /* .../groundRows (30); must be < rows (the reference reads row -1 otherwise) */
  float ground_angle_threshold;    /* .../groundAngleThreshold (10 deg) */
  float minimum_range;             /* .../minimumRange (10 m) */
  float sensor_mount_angle;        /* .../sensorMountAngle (10 deg) */
  float theta;                     /* .../theta (60 deg in rad): segmentation angle threshold */
  int32_t valid_point_num;         /* .../validPointNum (15) */
  int32_t min_line_num;            /* .../minLineNum (5): lines needed by segments of >= 50 points */
  int32_t valid_line_num;          /* .../validLineNum (5) */
  float min_delta_z;               /* .../minDeltaZ (0.1 m) */
  float max_delta_z;               /* .../maxDeltaZ (3.0 m) */
  float max_distance;              /* .../maxDistance (20 m) */
  float max_elevation;             /* .../maxElevation (2.0 m) above the sensor height T(2, 3) */
  /* labelling window, inclusive (valid_range, detection.cpp:514-516,569-571:
     rows and columns 156..356, hard-coded there for a 512 x 512 image) */
  int32_t win_row0, win_row1, win_col0, win_col1;
} ddlo_seg_params;

typedef struct ddlo_seg_result {
  int32_t segments;                /* feasible segments: labels 1 .. segments (label_count_ - 1) */
  int32_t ground_pixels;           /* ground_mat_ == 1 */
  int32_t range_pixels;            /* range_mat_ > 0 */
  int32_t rejected_pixels;         /* label_mat_ == 999999 */
} ddlo_seg_result;

/* label image values (detection.cpp:493-504,582,642,720) */
#define DDLO_SEG_EXCLUDED (-1)     /* ground or no range */
#define DDLO_SEG_UNLABELLED 0      /* outside the window, never reached */
#define DDLO_SEG_REJECTED 999999   /* part of an infeasible segment */

typedef struct ddlo_seg ddlo_seg;

gicp_status ddlo_seg_default_params(ddlo_seg_params* out);

/* rows >= 2, cols >= 1, 0 <= ground_rows < rows. */
gicp_status ddlo_seg_create(int device, const ddlo_seg_params* p, ddlo_seg** out);
gicp_status ddlo_seg_destroy(ddlo_seg* s);

/* One organized scan.  xyz_t: rows x cols points (row-major, row 0 = top,
   row rows-1 = the lowest beam), x, y, z float first, consecutive points
   stride_bytes apart, already in the world frame (cloud_in_t); non-finite
   points are no-return pixels.  T: the scan's pose (row-major 4x4).
   residual: rows x cols residual image (projectResiduals' residuals_mat_) or
   NULL (icp_residuals_set_ false: every average residual is 0). */
gicp_status ddlo_seg_process(ddlo_seg* s, const float* xyz_t, size_t stride_bytes, const float T[16],
                             const float* residual, ddlo_seg_result* res);

/* Images of the last ddlo_seg_process (rows x cols, row-major); any may be
   NULL: range_mat_ (float), ground_mat_ (int8: -1 no info, 0, 1 ground),
   label_mat_ (int32, DDLO_SEG_* above or 1 .. segments). */
gicp_status ddlo_seg_images(ddlo_seg* s, float* range, int8_t* ground, int32_t* label);

/* avg_residuals_[l] for l in [0, segments]: out[l] for l < cap; *n = segments + 1. */
gicp_status ddlo_seg_avg_residuals(ddlo_seg* s, double* out, size_t cap, size_t* n);

/* getGroundIndices: pixels with ground_mat_ == 1 among the bottom ground_rows
   rows, column by column, bottom row first.  *n = count; out may be NULL. */
gicp_status ddlo_seg_ground_indices(ddlo_seg* s, int32_t* out, size_t cap, size_t* n);

/* label_indices_i_: row-major pixel indices of every segment, as CSR:
   offsets[l] .. offsets[l + 1] (l = 1 .. segments; offsets has segments + 2
   entries, offsets[0] = offsets[1] = 0) index into indices.  Either pointer
   may be NULL to query *n_indices. */
gicp_status ddlo_seg_label_indices(ddlo_seg* s, int32_t* offsets, size_t offsets_cap, int32_t* indices,
                                   size_t indices_cap, size_t* n_indices);

/* The labelling alone (cloudSegmentation + labelComponents), on the host,
   over caller images: range (rows x cols), z (cloud_in_t z, NaN = no point),
   residual (or NULL), label (in: -1 / 0 as groundRemoval leaves it; out: the
   labels).  sensor_z = T(2, 3).  avg_residual[l] for l < avg_cap. */
gicp_status ddlo_seg_label(const ddlo_seg_params* p, const float* range, const float* z, const float* residual,
                           float sensor_z, int32_t* label, double* avg_residual, size_t avg_cap, int32_t* segments);

#ifdef __cplusplus
}
#endif

#endif /* DDLO_SEGMENT_H */
