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

/* Kernel timing: enable != 0 times every feature stage (k_fe_pick start to
 * k_fe_voxel end, the dominant part; start/stop hipEvents carried in the
 * dispatch packets) and
 * accumulates device milliseconds; 0 disables.  SLIO_LIO_PROFILE_KEEP keeps
 * the totals (pause / resume).  Read: accumulated ms and launch count
 * (synchronises the stream). */
#define SLIO_LIO_PROFILE_KEEP 16
/* enable | SLIO_LIO_PROFILE_SCAN: time every whole scan instead (the first
 * launch's start to the last launch's end: all the front-end's kernels). */
#define SLIO_LIO_PROFILE_SCAN 32
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

/* ======================================================================
 * LeGO-LOAM
 *   ImageProjection::cloudHandler  LeGO-LOAM/src/imageProjection.cpp:151-158
 *     findStartEndAngle :160-175, projectPointCloud :177-213 (the LAST point
 *     wins a cell), groundRemoval :216-262, cloudSegmentation :268-330 +
 *     labelComponents :332-393 -> cloud_info.msg + segmented / outlier clouds
 *   FeatureAssociation::runFeatureAssociation (front half)
 *     featureAssociation.cpp: adjustDistortion :617-805, calculateSmoothness
 *     :807-834, markOccludedPoints :838-876, extractFeatures :883-1007
 * The IMU ring buffer (imuHandler / AccumulateIMUShiftAndRotation :430-588)
 * is host state handed over with slio_lego_set_imu.
 * ====================================================================== */
typedef struct slio_lego* slio_lego_handle;

typedef struct slio_lego_params {
  int32_t device;
  int32_t n_scan;                  /* N_SCAN (utility.h:20, 16)                */
  int32_t horizon_scan;            /* Horizon_SCAN (1800)                      */
  int32_t ground_scan_ind;         /* groundScanInd (7)                        */
  int32_t segment_valid_point_num; /* segmentValidPointNum (5)                 */
  int32_t segment_valid_line_num;  /* segmentValidLineNum (3)                  */
  float ang_res_x;                 /* 0.2 deg                                  */
  float ang_res_y;                 /* 2.0 deg                                  */
  float ang_bottom;                /* 15.0 + 0.1 deg                           */
  float sensor_mount_angle;        /* 0 deg                                    */
  float segment_theta;             /* 1.0472 rad (60 deg)                      */
  float edge_threshold;            /* 0.1                                      */
  float surf_threshold;            /* 0.1                                      */
  float leaf_size;                 /* less-flat VoxelGrid leaf (0.2, :222)     */
  float scan_period;               /* 0.1 s                                    */
  int32_t max_points;              /* input capacity (0 -> 4 * cells)          */
  int32_t reserved[4];
} slio_lego_params;

/* FeatureAssociation IMU state read by adjustDistortion: the que_len-entry
 * ring buffer (imuTime double, the rest float), imuPointerLast (-1: no IMU),
 * imuPointerLastIteration, timeScanCur and imuAngularRotation{X,Y,Z}Last. */
typedef struct slio_lego_imu {
  const double* time;
  const float *roll, *pitch, *yaw;
  const float *velo_x, *velo_y, *velo_z;
  const float *shift_x, *shift_y, *shift_z;
  const float *ang_x, *ang_y, *ang_z; /* imuAngularRotation{X,Y,Z} */
  int32_t pointer_last, pointer_last_iteration, que_len;
  double time_scan_cur;
  float ang_last[3];
} slio_lego_imu;

/* State adjustDistortion leaves for the back half (updateInitialGuess
 * :1999-2029): imu{Roll,Pitch,Yaw}Start, imu{Roll,Pitch,Yaw}Cur of the last
 * point, imuVeloFromStart{X,Y,Z}Cur of the last point, imuAngularFromStart,
 * the new imuAngularRotation*Last and imuPointerLastIteration. */
typedef struct slio_lego_imu_out {
  float rpy_start[3], rpy_cur[3], velo_from_start[3], angular_from_start[3], ang_last[3];
  int32_t pointer_last_iteration;
} slio_lego_imu_out;

typedef struct slio_lego_counts {
  int64_t n_segmented, n_outlier, n_sharp, n_less_sharp, n_flat, n_less_flat;
  float orientation[3]; /* startOrientation, endOrientation, orientationDiff */
} slio_lego_counts;

int slio_lego_params_default(slio_lego_params* p);
int slio_lego_create(slio_lego_handle* out, const slio_lego_params* p);
int slio_lego_destroy(slio_lego_handle h);
int slio_lego_set_stream(slio_lego_handle h, void* stream);
/* IMU state for the next run; NULL or pointer_last < 0 -> no IMU correction. */
int slio_lego_set_imu(slio_lego_handle h, const slio_lego_imu* imu);
/* laserCloudIn x, y, z (PointXYZI order of the driver); findStartEndAngle runs here. */
int slio_lego_upload(slio_lego_handle h, const float* x, const float* y, const float* z, int64_t n);
int slio_lego_run_async(slio_lego_handle h);
int slio_lego_run(slio_lego_handle h, slio_lego_counts* counts);
/* Waits for the sweep.  SLIO_ETIMEOUT: the row stage's wait for an earlier
 * ring gave up (~0.5 s; the sweep's outputs are void, the next sweep is not
 * affected). */
int slio_lego_get_counts(slio_lego_handle h, slio_lego_counts* counts);
/* rangeMat, the input index that filled each cell (-1 empty), groundMat, labelMat. */
int slio_lego_get_image(slio_lego_handle h, float* range_mat, int32_t* cell_point, int8_t* ground,
                        int32_t* label);
/* cloud_info (startRingIndex, endRingIndex, segmentedCloudGroundFlag,
 * segmentedCloudColInd, segmentedCloudRange), segmented cloud xyzi (as
 * imageProjection publishes it) and outlier cloud xyzi.  Any may be NULL. */
int slio_lego_get_seg_info(slio_lego_handle h, int32_t* start_ring, int32_t* end_ring,
                           uint8_t* ground_flag, int32_t* col_ind, float* range, float* seg_xyzi,
                           float* outlier_xyzi);
/* After adjustDistortion: the segmented cloud in the LOAM frame (x, y, z,
 * ring + scanPeriod * relTime), cloudCurvature, cloudNeighborPicked after
 * markOccludedPoints, cloudLabel (2 sharp, 1 less sharp, -1 flat, 0), IMU state. */
int slio_lego_get_features(slio_lego_handle h, float* deskewed, float* curvature, uint8_t* picked,
                           int32_t* label, slio_lego_imu_out* imu_out);
/* cornerPointsSharp, cornerPointsLessSharp, surfPointsFlat, surfPointsLessFlat. */
int slio_lego_get_clouds(slio_lego_handle h, float* sharp, float* less_sharp, float* flat,
                         float* less_flat);
/* Timing of the feature kernels (or, with SLIO_LIO_PROFILE_SCAN, of the
 * whole sweep), as slio_lio_profile. */
int slio_lego_profile(slio_lego_handle h, int enable);
int slio_lego_profile_read(slio_lego_handle h, double* ms, int64_t* launches);

#ifdef __cplusplus
}
#endif

#endif /* SLIO_FRONTEND_H */
