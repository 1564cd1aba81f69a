/* slio_frontend.h -- C-ABI of the MI355X front-end:
 * LIO-SAM ImageProjection::projectPointCloud + cloudExtraction and
 * FeatureExtraction::calculateSmoothness + markOccludedPoints +
 * extractFeatures (incl. the per-ring pcl::VoxelGrid) as HIP kernels on gfx950.
 *
 * Reference seams (class members operating on class-owned arrays):
 *   ImageProjection::cloudHandler      LIO-SAM/src/imageProjection.cpp:193-212
 *     projectPointCloud :610-650, deskewPoint :565-604, findRotation :492-529,
 *     cloudExtraction :656-678 -> cloud_info.msg (startRingIndex, endRingIndex,
 *     pointColInd, pointRange, cloud_deskewed)
 *   FeatureExtraction::laserCloudInfoHandler  LIO-SAM/src/featureExtraction.cpp:88-100
 *     calculateSmoothness :108-131, markOccludedPoints :137-177,
 *     extractFeatures :183-296 -> cloud_corner, cloud_surface
 * The IMU queue handling (imuDeskewInfo :345-392) stays on the host: it hands
 * the integrated rotation table to slio_lio_set_deskew.
 *
 * Conventions as in slio.h: opaque handle, plain host pointers, int status
 * (SLIO_OK = 0, negative on error, message via slio_last_error()); points are
 * SoA float32; xyzi outputs are interleaved float32 (x, y, z, intensity).
 */
#ifndef SLIO_FRONTEND_H
#define SLIO_FRONTEND_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct slio_lio* slio_lio_handle;

typedef struct slio_lio_params {
  int32_t device;          /* HIP device ordinal                                   */
  int32_t n_scan;          /* N_SCAN (params.yaml:27, default 16)                  */
  int32_t horizon_scan;    /* Horizon_SCAN (params.yaml:28, default 1800)          */
  int32_t downsample_rate; /* downsampleRate (params.yaml:29, default 1)           */
  float lidar_min_range;   /* lidarMinRange (params.yaml:30, default 1.0)          */
  float lidar_max_range;   /* lidarMaxRange (params.yaml:31, default 1000.0)       */
  float edge_threshold;    /* edgeThreshold (params.yaml:57, default 1.0)          */
  float surf_threshold;    /* surfThreshold (params.yaml:58, default 0.1)          */
  float surf_leaf_size;    /* odometrySurfLeafSize (params.yaml:63, default 0.4)   */
  int32_t max_points;      /* input capacity (0 -> n_scan * horizon_scan)          */
  int32_t reserved[4];
} slio_lio_params;

typedef struct slio_lio_counts {
  int64_t n_extracted; /* points in cloud_deskewed / pointColInd / pointRange       */
  int64_t n_corner;    /* cloud_corner                                             */
  int64_t n_surface;   /* cloud_surface (after the per-ring VoxelGrid)            */
} slio_lio_counts;

/* params.yaml defaults (VLP-16: 16 x 1800). */
int slio_lio_params_default(slio_lio_params* p);
int slio_lio_create(slio_lio_handle* out, const slio_lio_params* p);
int slio_lio_destroy(slio_lio_handle h);
/* Enqueue on a caller stream (hipStream_t); NULL -> the handle's own stream. */
int slio_lio_set_stream(slio_lio_handle h, void* stream);

/* Deskew table of imuDeskewInfo (imageProjection.cpp:345-392): n_imu =
 * imuPointerCur + 1 entries of imuTime / imuRotX / imuRotY / imuRotZ (n_imu <=
 * 2000 = queueLength) and timeScanCur.  enabled = (deskewFlag == 1 &&
 * cloudInfo.imuAvailable); 0 leaves points as they are (deskewPoint :566). */
int slio_lio_set_deskew(slio_lio_handle h, const double* imu_time, const double* rot_x,
                        const double* rot_y, const double* rot_z, int32_t n_imu,
                        double time_scan_cur, int32_t enabled);

/* laserCloudIn (VelodynePointXYZIRT, imageProjection.cpp:4-15): x, y, z,
 * intensity, ring, time (s after timeScanCur; Ouster: t * 1e-9f, :244-258). */
int slio_lio_upload(slio_lio_handle h, const float* x, const float* y, const float* z,
                    const float* intensity, const uint16_t* ring, const float* time, int64_t n);

/* The whole front-end for the uploaded scan, enqueued on the stream. */
int slio_lio_run_async(slio_lio_handle h);
/* slio_lio_run_async + wait; counts may be NULL. */
int slio_lio_run(slio_lio_handle h, slio_lio_counts* counts);
int slio_lio_get_counts(slio_lio_handle h, slio_lio_counts* counts);

/* Kernel timing: enable != 0 times every k_lio_features launch (the
 * dominant kernel; start/stop hipEvents carried in the dispatch packet) and
 * accumulates device milliseconds; 0 disables.  SLIO_LIO_PROFILE_KEEP keeps
 * the totals (pause / resume).  Read: accumulated ms and launch count
 * (synchronises the stream). */
#define SLIO_LIO_PROFILE_KEEP 16
int slio_lio_profile(slio_lio_handle h, int enable);
int slio_lio_profile_read(slio_lio_handle h, double* ms, int64_t* launches);

/* rangeMat (n_scan * horizon_scan, FLT_MAX = empty, :146) and, per cell, the
 * index of the input point that filled it (-1 = empty). Either may be NULL. */
int slio_lio_get_range_image(slio_lio_handle h, float* range_mat, int32_t* cell_point);
/* cloud_info: startRingIndex / endRingIndex [n_scan], pointColInd /
 * pointRange [n_extracted], cloud_deskewed xyzi [n_extracted * 4].  Any may be NULL. */
int slio_lio_get_cloud_info(slio_lio_handle h, int32_t* start_ring, int32_t* end_ring,
                            int32_t* col_ind, float* point_range, float* xyzi);
/* Per extracted point: cloudCurvature, cloudNeighborPicked after
 * markOccludedPoints, final cloudLabel (1 corner, -1 flat, 0 other).  Any may be NULL. */
int slio_lio_get_features(slio_lio_handle h, float* curvature, uint8_t* picked, int32_t* label);
/* cloud_corner [n_corner * 4], cloud_surface [n_surface * 4].  Either may be NULL. */
int slio_lio_get_clouds(slio_lio_handle h, float* corner_xyzi, float* surface_xyzi);

#ifdef __cplusplus
}
#endif

#endif /* SLIO_FRONTEND_H */
