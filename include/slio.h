/*
 * slio.h — C-ABI drop-in boundary of the MI355X IKF scan-matching core.
 *
 * The reference (zhan994/agi_lidar_slam, S-FAST_LIO) has no plugin API for this
 * path; its seam is the C++ call
 *
 *   kf.update_iterated_dyn_share_modified(R, feats_down_body, ikdtree,
 *                                         Nearest_Points, maximum_iter,
 *                                         extrinsic_est)
 *       src/S-FAST_LIO/include/esekfom.hpp:270-275
 *       called from src/S-FAST_LIO/src/laserMapping.cpp:772-774
 *       and        src/S-FAST_LIO/src/laserMapping_re.cpp:663-665
 *
 * and, inside it, one measurement pass
 *
 *   esekf::h_share_model(dyn_share_datastruct&, feats_down_body, ikdtree,
 *                        Nearest_Points, extrinsic_est)
 *       src/S-FAST_LIO/include/esekfom.hpp:106-227
 *
 * whose per-point work (body->world transform, ikd-Tree 5-NN
 * KD_TREE::Nearest_Search ikd_Tree.cpp:370-402, esti_plane common_lib.h:102-134,
 * residual + range gate, Jacobian row) and whose H^T H / H^T h products
 * (esekfom.hpp:306-319) run here as HIP kernels on gfx950.  The 24x24 filter
 * algebra stays on the host (slio_ikf_update below, host C++).
 *
 * Conventions: plain pointers and sizes, int status (0 ok, <0 error, never
 * throws), one opaque handle per filter; a handle is not thread-safe.  All
 * host buffers are caller-owned.  Errors: slio_last_error() returns a
 * thread-local message for the last failing call on this thread.
 */
#ifndef SLIO_H
#define SLIO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SLIO_NUM_MATCH 5   /* NUM_MATCH_POINTS, common_lib.h:22 */
#define SLIO_NPROD 91      /* 78 (H^T H upper triangle) + 12 (H^T h) + 1 (m) */
#define SLIO_NHTH 78
#define SLIO_NSUPER 8      /* fixed summation tree: 8 super-chunks of the scan */
#define SLIO_CHUNK 128     /* scan points per reduction chunk (one workgroup) */

enum {
  SLIO_OK = 0,
  SLIO_EINVAL = -1,    /* bad argument */
  SLIO_ENOMEM = -2,    /* device or host allocation failed */
  SLIO_EDEVICE = -3,   /* HIP runtime error */
  SLIO_ECAPACITY = -4, /* scan larger than params.max_points */
  SLIO_ESTATE = -5,    /* call out of order (e.g. iterate before map upload) */
  SLIO_ETIMEOUT = -6   /* a device-side wait of the update gave up (the persistent
                          update's pass flag or a fused group's gate, > 1 s): the
                          result is not written; the handle's arrival counters
                          are reset, so the next update runs normally */
};

typedef struct slio_ctx* slio_handle;

typedef struct slio_params {
  int32_t device;          /* HIP device ordinal                              */
  int32_t max_points;      /* scan capacity; reference caps at 100000
                              (esekfom.hpp:23-29)                             */
  int32_t rank;            /* this handle's shard of the scan points          */
  int32_t nranks;          /* 1, 2, 4 or 8 (must divide SLIO_NSUPER)          */
  float grid_cell;         /* map grid cell edge in metres; 0 (default): auto,
                              1.0 m, or 1.25 m when the 1.0 m grid would have
                              more than 2^27 cells (speed only)               */
  float plane_threshold;   /* esti_plane threshold, 0.1f (esekfom.hpp:157)    */
  float max_match_sqd;     /* 5th-NN sq.-distance gate, 5 (esekfom.hpp:147)   */
  int32_t lanes_per_query; /* search lanes per scan point: 1, 2, 4, 8 (0 ->
                              tuned default)                                  */
  int64_t max_grid_cells;  /* dense cell-table budget (0 -> 1<<29)            */
  float search_radius;     /* first search sphere radius in metres (default 0:
                              scan the 3x3x3 cell block first); capped at 1.99
                              cells.
                              Any value gives the exact 5-NN; it only tunes
                              speed.                                           */
  float far_query_margin;  /* scan points farther than this (metres) outside
                              the map grid's bounding box get no neighbours
                              (index -1, never selected) instead of the exact
                              coarse-level far search.  They cannot pass the
                              max_match_sqd gate anyway, so only
                              Nearest_Points would differ from ikd-Tree.
                              Default 0: no cut, exact everywhere.            */
} slio_params;

/* Pose slice of state_ikfom used by the measurement model
 * (use-ikfom.hpp:18-27).  Rotations are Sophus::SO3 unit quaternions stored
 * (w, x, y, z); the kernel rotates points with the quaternion exactly as
 * SO3::operator*(Vector3d) does (esekfom.hpp:128-129). */
typedef struct slio_pose {
  double rot[4];  /* x_.rot          */
  double pos[3];  /* x_.pos          */
  double rli[4];  /* x_.offset_R_L_I */
  double tli[3];  /* x_.offset_T_L_I */
} slio_pose;

/* Full 24-D state_ikfom (use-ikfom.hpp:18-27); vector order of boxplus /
 * boxminus (esekfom.hpp:59-73, 236-258): pos, rot, R_LI, T_LI, vel, bg, ba,
 * grav. */
typedef struct slio_state {
  double pos[3];
  double rot[4];
  double rli[4];
  double tli[3];
  double vel[3];
  double bg[3];
  double ba[3];
  double grav[3];
} slio_state;

/* ---- handle lifecycle --------------------------------------------------- */
int slio_params_default(slio_params* p);
int slio_create(slio_handle* out, const slio_params* p);
int slio_destroy(slio_handle h);
/* Use an external hipStream_t (e.g. torch's current stream) instead of the
 * handle's own stream; NULL restores the handle's stream.  torch's DEFAULT
 * stream has the handle NULL: to share a stream with torch collectives, make a
 * torch.cuda.Stream current and pass that one. */
int slio_set_stream(slio_handle h, void* hip_stream);
const char* slio_last_error(void);
/* Fingerprint of the sources this library was compiled from (16 hex digits
 * of a SHA-256 over the csrc sources and these headers; build.py computes the
 * same digest), so a caller can tell a stale prebuilt library. */
const char* slio_build_id(void);

/* ---- map (replaces KD_TREE::Build, ikd_Tree.cpp:355-367, for a static map;
 *      the search side replaces KD_TREE::Nearest_Search ikd_Tree.cpp:370) -- */
/* Upload a map snapshot (host SoA float32, n points) and build the device
 * grid index.  Neighbour indices reported later refer to positions in these
 * arrays.  Device memory: 16 B per point + 4 B per grid cell for the cell-
 * sorted map, and (speed only) ~9x that for the block rows, which are skipped
 * when they do not fit, when n > 477M, or when SLIO_NO_BLOCK_ROWS=1 is set;
 * results are identical either way. */
int slio_map_upload(slio_handle h, const float* x, const float* y,
                    const float* z, int64_t n);
/* Share src's read-only device map with h (same device; batched replay).
 * The share holds the map src had at the time of the call (reference-
 * counted): a later slio_map_upload on src gives src a new map and leaves h
 * on the old one until h shares again (esekf.Esekf re-shares when its
 * KdTreeMap's generation changes). */
int slio_map_share(slio_handle h, slio_handle src);
/* Grid diagnostics: dims[3], cell edge, number of map points. */
int slio_map_info(slio_handle h, int32_t dims[3], float* cell, int64_t* n);

/* ---- map maintenance (the live laserMapping map, replaces the ikd-Tree
 *      calls of laserMapping.cpp:364, 430-431 and map_incremental :382-433) */
/* Map point ids: slio_map_upload gives 0..n-1; each add call gives the new
 * points that survive it the next ids, in list order.  Nearest_Points
 * indices (slio_get_neighbors) are these ids.  Changes are applied to the
 * device map at once (deletions) or queued (additions) and the search index
 * is rebuilt on the device before the next search pass -- no host copy of
 * the map, no re-upload.  A map shared by several handles changes for all of
 * them; do not change it while another handle's update is in flight. */
/* KD_TREE::Add_Points (ikd_Tree.cpp:419-512).  downsample = 1: for every
 * point (in order) the points already in its voxel box [floor(p/ds)*ds,
 * +ds) and the point itself keep only the one nearest the box centre
 * (ties: the stored point with the lower id wins only when strictly
 * nearer); *counter = Add_Points' return value.  downsample = 0: every
 * point is added. */
int slio_map_add_points(slio_handle h, const float* x, const float* y,
                        const float* z, int64_t n, int downsample,
                        float downsample_size, int64_t* counter);
/* KD_TREE::Delete_Point_Boxes (ikd_Tree.cpp:559-579): removes the points in
 * the half-open boxes [min, max) (boxes: nboxes x {min x, y, z, max x, y,
 * z}); *deleted = number of points removed. */
int slio_map_delete_boxes(slio_handle h, const float* boxes, int64_t nboxes,
                          int64_t* deleted);
/* map_incremental (laserMapping.cpp:382-433) on the device: the handle's
 * scan (feats_down_body) to world at state x with pointBodyToWorld's
 * rotation matrices (:276-287), classified against the Nearest_Points of
 * the handle's last search pass (which must have run on the current map),
 * then Add_Points(PointToAdd, downsample, filter_size_map_min) and
 * Add_Points(PointNoNeedDownsample, no downsample).  counts = {|PointToAdd|,
 * |PointNoNeedDownsample|, Add_Points' counter}.  nranks must be 1. */
int slio_map_incremental(slio_handle h, const slio_state* x,
                         double filter_size_map_min, int ekf_inited,
                         int64_t counts[3]);
/* The valid map points in ascending id (KD_TREE::flatten /
 * featsFromMap): cap is the buffers' length; *n = number of points
 * (ECAPACITY if cap is smaller). */
int slio_map_download(slio_handle h, float* x, float* y, float* z,
                      uint32_t* ids, int64_t cap, int64_t* n);
/* lasermap_fov_segment (laserMapping.cpp:309-365), host only: moves the
 * local map box [box_min, box_max] (in/out) with the LiDAR position and
 * returns up to 3 boxes to delete (for slio_map_delete_boxes). */
int slio_fov_segment(const double pos_lid[3], float box_min[3], float box_max[3],
                     int* initialized, double cube_len, float det_range,
                     float boxes_out[18], int* nboxes);

/* ---- scan (feats_down_body, laserMapping.cpp:737-739) -------------------- */
/* Upload the whole scan (host SoA float32, body frame).  With nranks > 1
 * every rank uploads the full scan and processes its own point shard. */
int slio_scan_upload(slio_handle h, const float* x, const float* y,
                     const float* z, int64_t n);
/* downSizeFilterSurf (laserMapping.cpp:683-686, 737-739) on the device: the
 * raw scan (feats_undistort, host SoA float32, n points) through
 * pcl::VoxelGrid with edge `leaf` (PCL 1.10 applyFilter + CentroidPoint:
 * voxel index over the cloud's bounding box, centroids in ascending voxel
 * index, float sums / count; non-finite points skipped; a leaf too small for
 * the cloud copies the input) becomes the handle's scan (feats_down_body),
 * *n_down points, ready for the passes below.  Inside a voxel the points are
 * summed in ascending input order (PCL's std::sort leaves that order
 * implementation-defined; a voxel of >= 3 points can differ from PCL's in
 * the last bits).  ECAPACITY if more than max_points voxels remain. */
int slio_scan_upload_voxel(slio_handle h, const float* x, const float* y,
                           const float* z, int64_t n, float leaf,
                           int64_t* n_down);
/* The handle's current scan (feats_down_body) back to the host. */
int slio_scan_download(slio_handle h, float* x, float* y, float* z);
/* Point range [begin, end) this handle processes for the uploaded scan. */
int slio_shard_range(slio_handle h, int64_t* begin, int64_t* end);

/* ---- one h_share_model pass (esekfom.hpp:106-227) + reduction ----------- */
/* Enqueue one measurement pass on the device.  do_search = ekfom_data.converge
 * (esekfom.hpp:138): 1 re-runs the 5-NN search and the gate, 0 reuses the
 * neighbours / plane / selection of the previous pass exactly like
 * point_selected_surf does.  The pass leaves SLIO_NSUPER x SLIO_NPROD fp64
 * super-chunk sums in the handle's device buffer (rows of super-chunks this
 * rank does not own are zero, so a SUM all-reduce over ranks is an exact
 * gather).  Returns the device pointer through d_super if non-NULL. */
int slio_iterate_async(slio_handle h, const slio_pose* x, int do_search,
                       int extrinsic_est, double** d_super);
/* Make the handle write its super-chunk sums into a caller-owned device
 * buffer of SLIO_NSUPER*SLIO_NPROD doubles (e.g. a torch tensor that an RCCL
 * all-reduce then operates on); NULL restores the handle's own buffer. */
int slio_set_super_buffer(slio_handle h, double* dev_buf);
/* Copy the super-chunk sums to host (synchronises the stream). */
int slio_super_download(slio_handle h, double super_out[SLIO_NSUPER * SLIO_NPROD]);
/* Fixed-order sum of the super-chunk rows: H^T H upper triangle (row-major,
 * i <= j), H^T h with h_i = -pd2 (esekfom.hpp:225), and m = effct_feat_num. */
int slio_reduce_super(const double super_in[SLIO_NSUPER * SLIO_NPROD],
                      double HTH[SLIO_NHTH], double HTh[12], int64_t* m);
/* Convenience: iterate_async + download + reduce (single rank). */
int slio_iterate(slio_handle h, const slio_pose* x, int do_search,
                 int extrinsic_est, double HTH[SLIO_NHTH], double HTh[12],
                 int64_t* m);

/* ---- per-point results (Nearest_Points / point_selected_surf / normvec) -- */
/* For the shard's points (n = end - begin): neighbour map indices (-1 if
 * fewer than 5 map points exist), f32 squared distances ascending (the
 * pointSearchSqDis of esekfom.hpp:135-141), final selection flag.  They are
 * the last SEARCH pass's results: the search pass stores only the neighbours'
 * map positions, and ids and distances are derived from them on this call
 * (or, automatically, before the handle's scan or map is replaced). */
int slio_get_neighbors(slio_handle h, int32_t* idx, float* sqd, uint8_t* sel);
/* Number of scan points of the last pass (of this handle's shard) whose
 * 5-NN search did not finish on the fine grid -- 5th neighbour beyond the
 * 5x5x5 fine-cell cube, or query cell more than 2 cells outside the grid --
 * and went to the coarse-level far search instead (diagnostic; synchronises
 * the stream). */
int slio_far_queries(slio_handle h, int64_t* n);
/* Plane (a, b, c, d) per point; (a,b,c) unit normal, d offset, or NaNs where
 * esti_plane failed or the point was gated out before the fit. */
int slio_get_planes(slio_handle h, float* abcd);
/* Residual pd2 (normvec->points[i].intensity, esekfom.hpp:159-171) of the last
 * pass for selected points, NaN otherwise. */
int slio_get_residuals(slio_handle h, float* pd2);

/* ---- kernel timing (HIP events on the handle's stream) ------------------- */
#define SLIO_KERNEL_SEARCH 0   /* fused search pass (kNN + plane + Jacobian + chunk sums) */
#define SLIO_KERNEL_REUSE 1    /* non-search pass                                          */
#define SLIO_KERNEL_SUPER 2    /* super-chunk sums (+ fused filter step)                   */
#define SLIO_PROFILE_KEEP 16   /* flag: keep the accumulated totals                         */
/* enable == 1 times every launch of every kind (start/stop hipEvents carried
 * in the dispatch packet) and accumulates elapsed device time per kind;
 * otherwise only the kinds whose bit 1 << (kind + 1) is set are timed (e.g.
 * 1 << (SLIO_KERNEL_SEARCH + 1) = 2 times the search pass alone).  Without
 * SLIO_PROFILE_KEEP any call resets the totals; with it, the call only
 * changes what is timed (SLIO_PROFILE_KEEP alone pauses), so timing can be
 * sampled over a subset of launches.  0 disables and resets. */
int slio_profile(slio_handle h, int enable);
/* Accumulated device milliseconds and launch count of a kernel kind
 * (synchronises the stream). */
int slio_profile_read(slio_handle h, int kind, double* ms, int64_t* launches);

/* ---- host IKF driver (update_iterated_dyn_share_modified, host C++) ------ */
/* Optional cross-rank reduction hook: must SUM-all-reduce `count` doubles at
 * device pointer dev_buf in place, ordered on `stream`. */
typedef int (*slio_allreduce_fn)(void* ctx, double* dev_buf, int64_t count,
                                 void* stream);

typedef struct slio_ikf_stats {
  int32_t passes;        /* h_share_model passes run                   */
  int32_t searches;      /* passes with the kNN search                 */
  int32_t valid_passes;  /* passes with effct_feat_num >= 1            */
  int32_t converged;     /* dyn_share.converge at exit                 */
  int64_t last_m;        /* effct_feat_num of the last pass            */
  double device_ms;      /* wall time inside device passes (host clock)*/
} slio_ikf_stats;

#define SLIO_MODE_REFERENCE 0  /* esekfom.hpp:292-345 control flow       */
#define SLIO_MODE_FIXED 1      /* exactly maximum_iter passes, kNN search
                                  every pass, P update at the end        */

/* Run the iterated update on state x (in/out) and covariance P (24x24
 * row-major, in/out) with measurement noise R (LASER_POINT_COV,
 * laserMapping.cpp:29).  reduce may be NULL for a single rank. */
int slio_ikf_update(slio_handle h, slio_state* x, double P[576], double R,
                    int maximum_iter, int extrinsic_est, int mode,
                    slio_allreduce_fn reduce, void* reduce_ctx,
                    slio_ikf_stats* stats);

/* Same update, device-resident: state, covariance and the control flags of
 * esekfom.hpp:292-345 live in HBM and the filter step runs on the device
 * after each pass, so the passes are enqueued back to back with no host round
 * trip; the host synchronises once at the end.  The device filter step is the
 * information form on the D columns H can have non-zero -- D = 6 without
 * extrinsic estimation (H's columns 6..11 are zero, esekfom.hpp:218-220), 12
 * with it -- while slio_ikf_update's host step always works on 12: the same
 * algebra, different operation order, so the two agree to rounding (not
 * bitwise).  In the single-rank configuration each pass after the first is
 * one launch (search or reuse pass, its sums and the filter step).  `reduce` (if any) is called once per pass at
 * enqueue time and must enqueue a stream-ordered SUM all-reduce; with NULL
 * and nranks > 1 the handle's communicator is used (slio_comm_init). */
int slio_ikf_update_device(slio_handle h, slio_state* x, double P[576], double R,
                           int maximum_iter, int extrinsic_est, int mode,
                           slio_allreduce_fn reduce, void* reduce_ctx,
                           slio_ikf_stats* stats);

/* ---- multi-GPU: the per-pass all-reduce inside the library (RCCL) --------
 * The scan's points shard across ranks (slio_params rank / nranks); each
 * pass's 8 x 91 fp64 super rows are SUM-all-reduced (one ncclAllReduce over
 * xGMI) and every rank runs the identical filter step, so all ranks hold the
 * same x and P, bit for bit, as one rank would.  Replaces the per-iteration
 * all-reduce the reference does not have (its laserMapping.cpp:772-774 update
 * runs on one CPU process). */
#define SLIO_COMM_ID_BYTES 128
/* One process, ndev GPUs (the reference's single-process laserMapping node):
 * out[r] = a handle of rank r on devices[r].  p gives the other parameters
 * (rank / nranks / device are set here); ndev divides 8.  Each handle then
 * takes the map (slio_map_upload: a replica per GPU, or slio_map_share between
 * ranks on one device) and the whole scan (slio_scan_upload), and
 * slio_group_ikf_update runs the update on all of them.  The group's reduce
 * backend (slio_group_reduce_kind):
 *   SLIO_GROUP_RCCL   (1) one communicator over all ranks (ncclCommInitAll),
 *                         when every rank has its own GPU;
 *   SLIO_GROUP_DEVICE (2) an in-device fixed-order sum of the ranks' super
 *                         rows by one kernel on rank 0's stream (ordered by
 *                         HIP events), when ranks share a device (RCCL
 *                         refuses that), or across peer-accessible GPUs when
 *                         the environment sets SLIO_GROUP_REDUCE=device.
 * SLIO_GROUP_REDUCE=rccl forces RCCL (an error when ranks share a device).
 * Both give the same bits as one rank. */
#define SLIO_GROUP_RCCL 1
#define SLIO_GROUP_DEVICE 2
int slio_create_group(slio_handle* out, int ndev, const int* devices, const slio_params* p);
/* The reduce backend of a group handle (SLIO_GROUP_*), 0 for a handle made by
 * slio_create, < 0 for a null handle. */
int slio_group_reduce_kind(slio_handle h);
/* slio_ikf_update_device on every rank of a group, enqueued from the calling
 * thread: per pass, each rank's search pass, the all-reduce of the ranks'
 * super rows (RCCL: one ncclGroup; in-device: k_group_reduce), each rank's
 * filter step -- no host round trip until the end.  x and P (in / out) and
 * stats come back from rank 0; the call fails (SLIO_EDEVICE) if any rank's x
 * or P differs from rank 0's.  On any error every rank's stream is drained
 * before the call returns, and the calling thread's current device is
 * restored in every case. */
int slio_group_ikf_update(slio_handle* hs, int n, slio_state* x, double P[576], double R,
                          int maximum_iter, int extrinsic_est, int mode, slio_ikf_stats* stats);
/* One process per GPU (e.g. torchrun): rank 0 makes an id (ncclGetUniqueId),
 * the caller hands it to every rank, each initialises its handle's
 * communicator (ncclCommInitRank with the handle's rank / nranks, a
 * collective call); slio_ikf_update_device with reduce == NULL then
 * all-reduces in the library on the handle's stream. */
int slio_comm_unique_id(uint8_t id[SLIO_COMM_ID_BYTES]);
int slio_comm_init(slio_handle h, const uint8_t id[SLIO_COMM_ID_BYTES]);

/* ---- IMU forward propagation and scan undistortion (ImuProcess::UndistortPcl,
 *      src/S-FAST_LIO/src/IMU_Processing.hpp:253-402) ------------------------ */
/* One IMU sample: stamp (s), linear acceleration, angular velocity. */
typedef struct slio_imu_sample {
  double t;
  double acc[3];
  double gyr[3];
} slio_imu_sample;
/* Pose6D (common_lib.h / set_pose6d): offset from the scan start (s), the
 * world-frame acceleration and bias-free angular velocity at that sample,
 * velocity, position, rotation matrix (row-major). */
typedef struct slio_imu_pose {
  double offset_time;
  double acc[3];
  double gyr[3];
  double vel[3];
  double pos[3];
  double rot[9];
} slio_imu_pose;
/* esekf::predict (esekfom.hpp:82-95) with the process model of
 * use-ikfom.hpp (get_f, df_dx, df_dw): x [+]= f dt, P = F P F^T + G Q G^T. */
int slio_ikf_predict(slio_state* x, double P[576], double dt, const double Q[144],
                     const double acc[3], const double gyr[3]);
/* UndistortPcl steps 1-4 (IMU_Processing.hpp:253-346), host: forward
 * propagation over imu[0..nimu) (imu[0] = the previous scan's last sample,
 * last_imu_, then meas.imu), predicting x / P in place; writes the IMUpose
 * table (*npose <= nimu entries).  acc_s_last / angvel_last /
 * last_lidar_end_time are the ImuProcess members carried between scans. */
int slio_imu_forward(const slio_imu_sample* imu, int nimu, double pcl_beg_time,
                     double pcl_end_time, double* last_lidar_end_time,
                     double mean_acc_norm, const double cov_gyr[3],
                     const double cov_acc[3], const double cov_bias_gyr[3],
                     const double cov_bias_acc[3], double acc_s_last[3],
                     double angvel_last[3], slio_state* x, double P[576],
                     slio_imu_pose* poses, int cap, int* npose);
/* UndistortPcl step 5 (IMU_Processing.hpp:351-401) on the device: the raw
 * scan (x, y, z float32, t = per-point time offset in ms, the `curvature`
 * field of preprocess) sorted by time, every point with t / 1000 > the first
 * pose's offset moved to the scan end state x_end by the IMU pose segment it
 * falls in.  Results (feats_undistort, time order) to the host arrays. */
int slio_undistort(slio_handle h, const float* x, const float* y, const float* z,
                   const float* t_ms, int64_t n, const slio_imu_pose* poses,
                   int npose, const slio_state* x_end, float* ox, float* oy,
                   float* oz, float* ot_ms);
/* The same undistortion, then downSizeFilterSurf (see slio_scan_upload_voxel)
 * without leaving the device: the result is the handle's scan. */
int slio_scan_upload_undistort_voxel(slio_handle h, const float* x, const float* y,
                                     const float* z, const float* t_ms, int64_t n,
                                     const slio_imu_pose* poses, int npose,
                                     const slio_state* x_end, float leaf,
                                     int64_t* n_down);

/* ---- LIO-SAM scan-to-map (src/LIO-SAM/src/mapOptmization.cpp) -------------
 * One handle per feature class: map = laserCloud{Corner,Surf}FromMapDS
 * (slio_map_upload), scan = laserCloud{Corner,Surf}LastDS (slio_scan_upload). */
/* cornerOptimization (kind 0, :1303-1432) / surfOptimization (kind 1,
 * :1438-1515) at transformTobeMapped = {roll, pitch, yaw, x, y, z}:
 * pointAssociateToMap, exact 5-NN in the handle's map, point-to-line (3x3
 * covariance, cv::eigen restated as OpenCV's Jacobi) or point-to-plane
 * (ColPivHouseholderQR) coefficients; kept on the device.  *nsel = number of
 * selected points (laserCloudOri{Corner,Surf}Flag). */
int slio_s2m_coeffs(slio_handle h, int kind, const float transform[6], int64_t* nsel);
/* The handle's coefficients (n x {x, y, z, intensity}) and flags to host. */
int slio_s2m_get_coeffs(slio_handle h, float* coeff, uint8_t* sel);
/* LMOptimization rows (:1578-1626; corners, then surfs) and the normal
 * equations A^T A (6x6) / A^T B (6) of the selected points, fp64 sums in a
 * fixed order rounded to float; *nsel = laserCloudSelNum.  Either handle may
 * be NULL. */
int slio_s2m_normal_equations(slio_handle h_corner, slio_handle h_surf,
                              const float transform[6], float AtA[36], float AtB[6],
                              int64_t* nsel);
/* LMOptimization's host step (:1627-1700): X = solve(AtA, AtB) (QR); on
 * iteration 0 the degeneracy projection matP (eigenvalues < 100) is formed,
 * later iterations reuse it; transform += X; *converged = deltaR < 0.05 deg
 * and deltaT < 0.05 cm.  Returns 1 (nothing done) with fewer than 50
 * correspondences, as the reference's `return false`.  A (numerically)
 * singular A^T A -- an R diagonal below 10 * FLT_EPSILON in the QR, where
 * cv::solve(DECOMP_QR) gives up and zeroes matX -- is a zero step (then
 * converged), not an error, as in the reference, which ignores cv::solve's
 * result. */
int slio_s2m_lm_step(const float AtA[36], const float AtB[6], int64_t nsel, int iter_count,
                     float transform[6], int* is_degenerate, float matP[36], int* converged);

/* Manifold helpers exported for tests (esekfom.hpp:59-73, 236-258). */
int slio_state_boxplus(const slio_state* x, const double dx[24], slio_state* out);
int slio_state_boxminus(const slio_state* x1, const slio_state* x2, double dx[24]);

/* ---- diagnostics ----------------------------------------------------------- */
/* Re-read the SLIO_NO_FUSE / SLIO_NO_FUSE0 / SLIO_PERSIST / SLIO_NO_MFMA /
 * SLIO_EVENT_WAIT / SLIO_NO_KNN_CERT switches of the update path (read once at
 * slio_create). */
int slio_debug_reload_switches(slio_handle h);
/* How the last slio_ikf_update_device ran: 1 one persistent launch for all
 * its passes (SLIO_PERSIST=1, single rank, fused configuration, every chunk's
 * workgroup resident at once), 0 a launch (or two) per pass. */
int slio_debug_update_path(slio_handle h);
/* Host clock stamps (CLOCK_MONOTONIC ns) of the last slio_ikf_update_device:
 * [0] entry, [1] state set up, [2] control block + information-form constants
 * ready (fused path), [3] first launch enqueued, [4] every launch enqueued,
 * [5] result seen, [6] return.  After slio_group_ikf_update, rank 0's handle
 * holds the group's: [0] entry, [1] every pass enqueued, [2] every rank's
 * result seen, [3] return, [4] / [5] / [6] host ns spent enqueueing the
 * ranks' pass launches / the reduce (events + in-device reduce, or the RCCL
 * group) / the filter steps.  out may be NULL; enable 1 / 0 turns stamping
 * on / off, -1 leaves it. */
int slio_debug_host_stamps(slio_handle h, int enable, int64_t out[8]);
/* kNN certificate counters (wrapping 32-bit; counting starts with the first
 * call, which turns it on for the handle -- it costs two same-address atomics
 * per workgroup):
 * out[0] queries whose 5 nearest a later pass certified from its earlier
 * search's 5 nearest and bound, out[1] queries searched in full in passes that write
 * certificates (device-resident passes after the first). */
int slio_debug_knn_cert(slio_handle h, uint32_t out[2]);
/* The device-side waits of the next updates on this handle (a persistent
 * update's workgroups waiting for the pass flag; on a group's rank 0, every
 * rank's gate between fused group passes) give up after `ticks` 100 MHz
 * clock ticks instead of 1 s (0 restores 1 s).  A test hook: 1 forces the
 * give-up path (SLIO_ETIMEOUT, counters reset). */
int slio_debug_wait_limit(slio_handle h, int64_t ticks);

#ifdef __cplusplus
}
#endif

#endif /* SLIO_H */
