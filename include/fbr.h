/* fbr.h — C-ABI of the MI355X-native feature-based scan-to-map registration path.
 *
 * Drop-in boundary for the per-scan hot loop of qpc001/Feature_Base_Pointcloud_Registration
 * (a LIO-SAM-derived localiser).  The reference's "operator API" for this path is in-process C++:
 *
 *   ImageProjection::cloudHandler()            src/imageProjection.cpp:182-226
 *     projectPointCloud() / cloudExtraction()  src/imageProjection.cpp:583-670
 *   FeatureExtraction::featureExtra()          src/featureExtraction.h:79-103
 *   mapOptimization::registration()            src/mapOptmization.h:263-343
 *   mapOptimization::allocateMemory() (map)    src/mapOptmization.h:245-260
 *
 * Each entry point below names the reference function it replaces.  Conventions:
 *   - plain C types only; host buffers are caller-owned; device memory is owned by the ctx;
 *   - every function returns an int status: 0 = FBR_OK, < 0 = error (fbr_strerror());
 *   - a ctx is bound to one HIP device and one HIP stream and is not thread-safe
 *     (one ctx per host thread and device, as the reference runs one scan at a time);
 *   - poses are the reference's transformTobeMapped layout [roll, pitch, yaw, x, y, z]
 *     (mapOptmization.h:131); fbr_affine_from_pose / fbr_pose_from_affine convert to and from the
 *     Eigen::Affine3f the reference's registration() takes, with PCL's exact formulas.
 */
#ifndef FBR_H_
#define FBR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FBR_ABI_VERSION 4  /* 4: fbr_batch_allgather takes wait_stream (the caller's reader of recv);
                              3: fbr_params.exact_voxel_order / pipeline_depth (were reserved_[0..1]);
                              2: fbr_selftest_math writes 6 floats per element (was 4) */

/* ---- status codes ------------------------------------------------------------------------- */
#define FBR_OK 0
#define FBR_ERR_INVALID_ARG (-1)  /* null pointer, negative size, bad parameter            */
#define FBR_ERR_HIP (-2)          /* a HIP runtime call failed                              */
#define FBR_ERR_NO_MAP (-3)       /* registration requested before fbr_set_map()           */
#define FBR_ERR_CAPACITY (-4)     /* input larger than the ctx was created for              */
#define FBR_ERR_UNSUPPORTED (-5)  /* configuration outside what the kernels handle          */
#define FBR_ERR_NO_DEVICE (-6)    /* no HIP device / extension not usable                   */
#define FBR_ERR_STATE (-7)        /* call order violated (e.g. features before projection)  */
#define FBR_ERR_MSG (-8)          /* PointCloud2 rejected by cachePointCloud's checks: not
                                     is_dense, or no "ring" field (imageProjection.cpp:256-281,
                                     where the reference calls ros::shutdown())               */

/* ---- registration outcome (fbr_reg_stats.status) -------------------------------------------- */
#define FBR_REG_OK 0                    /* scan2MapOptimization ran                           */
#define FBR_REG_NOT_ENOUGH_FEATURES 1   /* mapOptmization.h:1410/1440 gate: pose left at guess */
#define FBR_REG_SKIPPED_INTERVAL 2      /* mapOptmization.h:279 mappingProcessInterval gate    */
#define FBR_REG_FEATURE_CAPACITY 3      /* batch job: features exceeded the device capacity;   */
                                        /* its pose is left at the guess (single-scan calls    */
                                        /* return FBR_ERR_UNSUPPORTED instead)                 */

/* Raw lidar point: the PointXYZIRT payload of imageProjection.cpp:8-21 (x,y,z,intensity f32,
 * ring u16, time f32), laid out with natural alignment (24 bytes). */
typedef struct fbr_point_xyzirt {
  float x, y, z, intensity;
  uint16_t ring;
  uint16_t pad_;
  float time;
} fbr_point_xyzirt;

/* Work point: pcl::PointXYZI payload (include/utility.h:55). */
typedef struct fbr_point_xyzi {
  float x, y, z, intensity;
} fbr_point_xyzi;

/* Tunables.  Defaults (fbr_params_default) are config/params.yaml plus the constants the
 * reference hard-codes (SURVEY §5 "Config / flags"). */
typedef struct fbr_params {
  int32_t n_scan;                    /* N_SCAN                       params.yaml:19        */
  int32_t horizon_scan;              /* Horizon_SCAN                 params.yaml:20        */
  float edge_threshold;              /* edgeThreshold 1.0            params.yaml:45        */
  float surf_threshold;              /* surfThreshold 0.1            params.yaml:46        */
  int32_t edge_feature_min_valid_num;/* 10                           params.yaml:47        */
  int32_t surf_feature_min_valid_num;/* 100                          params.yaml:48        */
  float odometry_surf_leaf_size;     /* 0.4 per-ring surf VoxelGrid  params.yaml:51        */
  float mapping_corner_leaf_size;    /* 0.2                          params.yaml:52        */
  float mapping_surf_leaf_size;      /* 0.4                          params.yaml:53        */
  float z_tollerance;                /* 1000                         params.yaml:56        */
  float rotation_tollerance;         /* 1000                         params.yaml:57        */
  int32_t number_of_cores;           /* 4 (CPU paths only)           params.yaml:60        */
  double mapping_process_interval;   /* 0.15 s                       params.yaml:61        */
  float crop_half[3];                /* 30, 30, 10 m local-map box   mapOptmization.h:286  */
  int32_t max_iterations;            /* 30 Gauss-Newton iterations   mapOptmization.h:1417 */
  int32_t max_points_per_scan;       /* device capacity: raw points per scan               */
  int32_t max_batch;                 /* device capacity: scans per device batch            */
  int32_t exact_voxel_order;         /* 0: every VoxelGrid sums a voxel's points in index order
                                        (centroids to float rounding, the fast default); 1: in
                                        std::sort's order, as PCL does (bit-identical centroids and
                                        poses vs the oracle, ~0.45x the batch throughput)        */
  int32_t pipeline_depth;            /* batch launch slots 1..3 (0 = default 3; forced to 1 when
                                        max_batch = 1): launch n's front end overlaps the
                                        Gauss-Newton tails of up to depth-1 launches before it    */
  int32_t reserved_[2];
} fbr_params;

/* Per-scan registration statistics. */
typedef struct fbr_reg_stats {
  int32_t status;       /* FBR_REG_*                                                       */
  int32_t iterations;   /* LMOptimization calls made (<= max_iterations)                   */
  int32_t converged;    /* 1 if the loop ended on the 0.05 deg / 0.05 cm test               */
  int32_t degenerate;   /* isDegenerate after the last LMOptimization call                  */
  int32_t n_sel;        /* correspondences in the last LMOptimization call                  */
  int32_t n_corner_ds;  /* laserCloudCornerLastDSNum                                        */
  int32_t n_surf_ds;    /* laserCloudSurfLastDSNum                                          */
  int32_t n_corner_map; /* laserCloudCornerFromMapDSNum (cropped local map)                 */
  int32_t n_surf_map;   /* laserCloudSurfFromMapDSNum                                       */
  int32_t n_points;     /* valid projected points (cloud_deskewed size)                     */
  int32_t n_corner;     /* corner features before DS                                        */
  int32_t n_surf;       /* surface features before DS                                       */
} fbr_reg_stats;

typedef struct fbr_ctx fbr_ctx;

/* ---- sensor_msgs/PointCloud2 wire format ------------------------------ */
/* sensor_msgs/PointField datatypes */
#define FBR_PF_INT8 1
#define FBR_PF_UINT8 2
#define FBR_PF_INT16 3
#define FBR_PF_UINT16 4
#define FBR_PF_INT32 5
#define FBR_PF_UINT32 6
#define FBR_PF_FLOAT32 7
#define FBR_PF_FLOAT64 8

typedef struct fbr_point_field { /* sensor_msgs/PointField */
  const char* name;
  uint32_t offset;
  uint8_t datatype;              /* FBR_PF_* */
  uint32_t count;
} fbr_point_field;

typedef struct fbr_pointcloud2 { /* sensor_msgs/PointCloud2 without the header */
  uint32_t height, width;
  const fbr_point_field* fields;
  int32_t n_fields;
  uint8_t is_bigendian;          /* ignored, as pcl::fromROSMsg does (host byte order assumed) */
  uint32_t point_step, row_step;
  const uint8_t* data;
  uint64_t data_size;            /* bytes at data (>= (height-1)*row_step + width*point_step) */
  uint8_t is_dense;
} fbr_pointcloud2;

/* msg_flags bits reported by the *_msg entry points (warnings, the call still succeeds) */
#define FBR_MSG_NO_TIME 1        /* no "time" field: deskewFlag = -1, ROS_WARN (:285-298); time = 0 */
#define FBR_MSG_RING_UNMAPPED 2  /* "ring" exists but is not UINT16 x1: fromROSMsg leaves ring = 0 */
#define FBR_MSG_XYZI_UNMAPPED 4  /* x, y, z or intensity missing / not FLOAT32 x1: left 0          */

void fbr_params_default(fbr_params* p);
const char* fbr_strerror(int status);
int fbr_abi_version(void);
int fbr_device_count(int* count);

/* Create / destroy a context on HIP device `hip_device` (ParamServer + member construction,
 * utility.h:146-212, featureExtraction.h:48-77, mapOptmization.h:153-196). */
int fbr_create(fbr_ctx** out, const fbr_params* p, int hip_device);
int fbr_destroy(fbr_ctx* ctx);

/* Load the prior global feature map (already read from cloudCorner.pcd / cloudSurf.pcd) and
 * apply the start-up VoxelGrid (corner leaf mapping_corner_leaf_size, surf leaf
 * mapping_surf_leaf_size), replacing mapOptmization.h:245-260.  Builds the device search grid. */
int fbr_set_map(fbr_ctx* ctx, const fbr_point_xyzi* corner, int64_t n_corner,
                const fbr_point_xyzi* surf, int64_t n_surf);
/* pcl::io::loadPCDFile(HOME + savePCDDirectory + "cloudCorner.pcd" / "cloudSurf.pcd") followed by
 * fbr_set_map — the whole start-up block mapOptmization.h:245-260 (host-side PCD parsing). */
int fbr_load_map(fbr_ctx* ctx, const char* corner_pcd, const char* surf_pcd);

/* PCD v0.7 I/O for PointXYZI clouds (host only, no device needed).
 * fbr_pcd_read replaces pcl::io::loadPCDFile<PointXYZI> (mapOptmization.h:247-248): DATA ascii,
 * binary and binary_compressed (LZF); x, y, z and intensity are taken by name from any field
 * layout (F/U/I types, other fields skipped, missing intensity = 0).  Call with out == NULL to get
 * the point count in *n, then with a buffer of cap >= *n points (FBR_ERR_CAPACITY otherwise).
 * fbr_pcd_write_ascii replaces pcl::io::savePCDFileASCII (mapOptmization.h:511-515): PCL's header
 * and 8 significant digits per value.  fbr_pcd_write_binary writes DATA binary (exact floats). */
int fbr_pcd_read(const char* path, fbr_point_xyzi* out, int64_t cap, int64_t* n);
int fbr_pcd_write_ascii(const char* path, const fbr_point_xyzi* points, int64_t n);
int fbr_pcd_write_binary(const char* path, const fbr_point_xyzi* points, int64_t n);

/* cachePointCloud's conversion and checks (imageProjection.cpp:255-298) on the host:
 * pcl::fromROSMsg<PointXYZIRT> (fields mapped by name with matching datatype and count, points in
 * row-major order, unmapped fields 0), then the is_dense and "ring" checks (FBR_ERR_MSG) and the
 * "time" check (FBR_MSG_NO_TIME).  out == NULL queries *n.  The reference runs the ring/time
 * checks on the first message only (static flags); these entry points check every message. */
int fbr_msg_to_points(const fbr_pointcloud2* msg, fbr_point_xyzirt* out, int64_t cap, int64_t* n,
                      int32_t* msg_flags);
/* pcl::toROSMsg of a PointXYZI cloud (publishCloud, utility.h:255-264): height 1, width n,
 * fields x@0 y@4 z@8 intensity@16 (FLOAT32 x1), point_step 32, row_step 32n, with PCL's padding
 * (1.0f at offset 12, zeros after intensity).  data_out holds 32*n bytes. */
int fbr_points_to_msg_data(const fbr_point_xyzi* points, int64_t n, uint8_t* data_out);

/* Device variants of fbr_project / fbr_process_scan that take the raw PointCloud2: the message
 * bytes are copied to HBM as they are and unpacked by a kernel (field mapping as
 * fbr_msg_to_points), so the host does no per-point work (cachePointCloud + cloudHandler,
 * imageProjection.cpp:182-226). */
int fbr_project_msg(fbr_ctx* ctx, const fbr_pointcloud2* msg, int32_t* start_ring, int32_t* end_ring,
                    int32_t* col_ind, float* range, fbr_point_xyzi* cloud, int64_t* n_out,
                    int32_t* msg_flags);
int fbr_process_msg(fbr_ctx* ctx, const fbr_pointcloud2* msg, double stamp, float pose_inout[6],
                    fbr_reg_stats* stats, int32_t* msg_flags);

/* ---- IMU deskew --------------------------------------------------------
 * The reference carries LIO-SAM's IMU deskew but calls it nowhere: deskewInfo() is commented out
 * in cloudHandler (imageProjection.cpp:189-191), so imuAvailable stays 0 and deskewPoint() is the
 * identity (:548-549).  These entry points restore the path as it runs with that call enabled:
 *   fbr_imu_convert      imuConverter (utility.h:219-253), applied by imuHandler to each sample
 *   fbr_imu_deskew_info  deskewInfo + imuDeskewInfo (imageProjection.cpp:303-393) on the host:
 *                        a serial pass over the ~20 queued samples that builds the scan's table
 *   fbr_set_deskew       hands tables to the device: the compaction kernel then applies
 *                        deskewPoint / findRotation (:494-580) to every kept point, and
 *                        transformUpdate (mapOptmization.h:1444-1474) slerps roll and pitch towards
 *                        imuRollInit / imuPitchInit.
 * findPosition is all-zero in the reference (:528-542, positional deskew commented out), and the
 * odometry half of deskewInfo only fills initial-guess fields read by the disabled
 * updateInitialGuess; neither has an observable effect on this path. */
#define FBR_IMU_QUEUE 500 /* queueLength, imageProjection.cpp:23 */

typedef struct fbr_imu_sample { /* the sensor_msgs/Imu fields the path reads */
  double stamp;                 /* header.stamp.toSec()                                  */
  double linear_acceleration[3];
  double angular_velocity[3];
  double orientation[4];        /* x, y, z, w                                             */
} fbr_imu_sample;

typedef struct fbr_imu_extrinsics { /* ParamServer extrinsics (utility.h:172-178), row-major */
  double ext_rot[9];                /* extrinsicRot                                          */
  double ext_rpy[9];                /* extrinsicRPY (-> extQRPY)                             */
} fbr_imu_extrinsics;

/* fbr_deskew_table.status */
#define FBR_DESKEW_READY 0    /* deskewInfo() returned true: the scan is processed                */
#define FBR_DESKEW_WAIT_IMU 1 /* deskewInfo() returned false (the IMU queue does not cover the
                                 scan, :310-314): the reference's cloudHandler drops the scan     */

typedef struct fbr_deskew_table { /* imuDeskewInfo() state of one scan (imageProjection.cpp:52-57) */
  int32_t status;                 /* FBR_DESKEW_*                                                   */
  int32_t imu_available;          /* cloudInfo.imuAvailable                                         */
  int32_t imu_pointer_cur;        /* imuPointerCur                                                  */
  float imu_roll_init, imu_pitch_init, imu_yaw_init; /* cloudInfo.imu{Roll,Pitch,Yaw}Init          */
  double time_scan_cur;           /* timeScanCur                                                    */
  double imu_time[FBR_IMU_QUEUE]; /* imuTime                                                        */
  double imu_rot_x[FBR_IMU_QUEUE], imu_rot_y[FBR_IMU_QUEUE], imu_rot_z[FBR_IMU_QUEUE];
} fbr_deskew_table;

/* imuConverter: acceleration and angular velocity rotated by extrinsicRot, orientation =
 * extQRPY * q (Eigen, double).  FBR_ERR_INVALID_ARG for the |q| < 0.1 "please use a 9-axis IMU"
 * case, where the reference shuts the node down (:246-250). */
int fbr_imu_convert(const fbr_imu_extrinsics* ext, const fbr_imu_sample* in, fbr_imu_sample* out);
/* deskewInfo()'s IMU half on a queue of converted samples in arrival order.  *n_pop receives the
 * number of leading samples imuDeskewInfo pops (stamp < time_scan_cur - 0.01, :328-335), which the
 * caller removes from its queue (0 when the scan is dropped: deskewInfo returns before popping).
 * The table's imu_*_init fields are only overwritten when a sample at or before time_scan_cur
 * remains (:354-355): pass the previous scan's table to keep the reference's carry-over.
 * FBR_ERR_CAPACITY if the scan needs more than FBR_IMU_QUEUE samples (the reference overruns its
 * arrays there). */
int fbr_imu_deskew_info(const fbr_imu_sample* imu_queue, int64_t n_imu, double time_scan_cur,
                        double time_scan_next, fbr_deskew_table* out, int64_t* n_pop);
/* Deskew tables for the following calls: job j of a staged batch uses tables[j] (j < n_tables),
 * the single-scan calls use tables[0].  tables == NULL or n_tables == 0 restores the reference's
 * runtime behaviour (no deskew, imuAvailable = 0).  A PointCloud2 without a "time" field disables
 * the point deskew for that call (deskewFlag = -1, :296-297, :548) but not the IMU update. */
int fbr_set_deskew(fbr_ctx* ctx, const fbr_deskew_table* tables, int n_tables);

/* ---- LIO-SAM keyframe local map ------------------------------------
 * The reference's mapping back-end (laserCloudInfoHandler, mapOptmization.h:346-389) registers
 * each scan against a local map built from its keyframes instead of the cropped prior map:
 * extractSurroundingKeyFrames (:964-978) -> extractNearby (:872-907) or extractForLoopClosure
 * (:857-870) -> extractCloud (:909-955).  The keyframe store mirrors cloudKeyPoses3D/6D and
 * corner/surfCloudKeyFrames; GTSAM (saveKeyFramesAndFactor / correctPoses) stays with the caller,
 * which pushes each new key pose + its down-sampled feature clouds (fbr_keyframes_add) and
 * rewrites poses after a loop closure (fbr_keyframes_set_pose).  Selection runs on the host (a few
 * hundred poses), the transforms, concatenation, VoxelGrids and the kNN grid on the device. */
typedef struct fbr_keypose {   /* PointXYZIRPYT (mapOptmization.h:34-51) */
  float x, y, z;
  float intensity;             /* key index: set to the keyframe's position by fbr_keyframes_add,
                                  as saveKeyFramesAndFactor does (:1687, :1694)                   */
  float roll, pitch, yaw;
  float pad_;
  double time;                 /* timeLaserCloudInfoLast when the keyframe was saved (:1698)     */
} fbr_keypose;

typedef struct fbr_keyframe_params {
  float search_radius;         /* surroundingKeyframeSearchRadius 50 m   params.yaml:67        */
  float pose_density;          /* surroundingKeyframeDensity 2 m          params.yaml:66        */
  int32_t loop_closure;        /* loopClosureEnableFlag 0                 params.yaml:70        */
  int32_t submap_size;         /* surroundingKeyframeSize 25              params.yaml:71        */
  double recent_window;        /* 10 s of most recent keyframes           mapOptmization.h:900  */
} fbr_keyframe_params;

void fbr_keyframe_params_default(fbr_keyframe_params* p);
/* cloudKeyPoses3D/6D->push_back + corner/surfCloudKeyFrames.push_back (lidar-frame clouds). */
int fbr_keyframes_add(fbr_ctx* ctx, const fbr_keypose* pose, const fbr_point_xyzi* corner, int64_t n_corner,
                      const fbr_point_xyzi* surf, int64_t n_surf);
/* correctPoses (:1740-1770): new x, y, z, roll, pitch, yaw of keyframe `index` (index and time kept). */
int fbr_keyframes_set_pose(fbr_ctx* ctx, int64_t index, const fbr_keypose* pose);
int fbr_keyframes_count(fbr_ctx* ctx, int64_t* n);
int fbr_keyframes_reset(fbr_ctx* ctx);
/* extractSurroundingKeyFrames at timeLaserCloudInfoLast = `stamp`: the down-sampled local corner /
 * surf maps become the registration map of the following fbr_register / fbr_process_scan calls
 * (registered without the CropBox, as scan2MapOptimization does on them), until fbr_set_map /
 * fbr_load_map restores a prior map.  With no keyframe the previous map is kept (:967-968).
 * n_frames (optional) = entries of cloudToExtract. */
int fbr_extract_surrounding_keyframes(fbr_ctx* ctx, double stamp, const fbr_keyframe_params* kp,
                                      int64_t* n_corner_map, int64_t* n_surf_map, int32_t* n_frames);

/* Down-sampled global map actually used (sizes, then optional copies; pass NULL to skip).  After
 * fbr_extract_surrounding_keyframes: the keyframe local map (laserCloud{Corner,Surf}FromMapDS). */
int fbr_get_map(fbr_ctx* ctx, int64_t* n_corner, int64_t* n_surf, fbr_point_xyzi* corner,
                fbr_point_xyzi* surf);

/* A2+A4: projectPointCloud() + cloudExtraction() (imageProjection.cpp:583-670).
 * Fills the cloud_info fields (msg/cloud_info.msg:5-9,32): start_ring/end_ring [n_scan],
 * col_ind/range/cloud [n_out] (size the buffers for n_in points). */
int fbr_project(fbr_ctx* ctx, const fbr_point_xyzirt* points, int64_t n_in, int32_t* start_ring,
                int32_t* end_ring, int32_t* col_ind, float* range, fbr_point_xyzi* cloud,
                int64_t* n_out);

/* A6-A9: FeatureExtraction::featureExtra() on the ctx's last projection
 * (featureExtraction.h:79-294).  label[n_out] gets cloudLabel (1 corner, -1 picked surf, 0);
 * corner/surf get cloud_corner / cloud_surface (size corner for 20*6*n_scan points and surf for
 * n_out points).  Any output pointer may be NULL. */
int fbr_extract_features(fbr_ctx* ctx, int8_t* label, fbr_point_xyzi* corner, int64_t* n_corner,
                         fbr_point_xyzi* surf, int64_t* n_surf);

/* A10-A18: mapOptimization::registration() (mapOptmization.h:263-343) on given feature clouds,
 * ignoring the time gate.  pose_inout: [roll,pitch,yaw,x,y,z] guess in, registered pose out. */
int fbr_register(fbr_ctx* ctx, const fbr_point_xyzi* corner, int64_t n_corner,
                 const fbr_point_xyzi* surf, int64_t n_surf, float pose_inout[6],
                 fbr_reg_stats* stats);
/* Same, also returning the pose after every Gauss-Newton iteration (trace [max_iterations][6]). */
int fbr_register_trace(fbr_ctx* ctx, const fbr_point_xyzi* corner, int64_t n_corner,
                       const fbr_point_xyzi* surf, int64_t n_surf, float pose_inout[6],
                       fbr_reg_stats* stats, float* trace);

/* One scan through the whole path in stream mode (cloudHandler after the cache queue,
 * imageProjection.cpp:197-225): the FeatureExtraction scratch state carries over between calls
 * as in the reference; `stamp` feeds the mappingProcessInterval gate (mapOptmization.h:279).
 * Returns as soon as the pose is known (the Gauss-Newton solve that ends the run writes it to
 * host-mapped memory); Gauss-Newton iterations enqueued ahead of that point may still be draining
 * on the context's stream, and every other entry point waits for them first.  The caller's buffer
 * may be reused once the call returns. */
int fbr_process_scan(fbr_ctx* ctx, const fbr_point_xyzirt* points, int64_t n_in, double stamp,
                     float pose_inout[6], fbr_reg_stats* stats);
/* Forget the carried FeatureExtraction / time-gate state (as a freshly constructed node). */
int fbr_reset_stream(fbr_ctx* ctx);

/* Independent jobs (config C4): each job is one scan registered from its own guess against the
 * shared map, with fresh FeatureExtraction state.  Processed in device batches of max_batch; the
 * host scans are packed into pinned staging and copied on a second stream, double-buffered, so
 * batch k+1's host-to-device copy overlaps batch k's compute.  The caller's buffers may be reused
 * once the call returns. */
int fbr_process_batch(fbr_ctx* ctx, const fbr_point_xyzirt* const* scans, const int64_t* n_in,
                      int n_jobs, float* poses_inout /* [n_jobs][6] */,
                      fbr_reg_stats* stats /* [n_jobs] or NULL */);
/* Diagnostic: the kNN grid of the current map: {sparse (hashed chunks) 0/1, surf-grid box dims
 * x, y, z, box cells, stored chunks (sparse) or cells (dense), corner points, surf points}. */
int fbr_map_grid_info(fbr_ctx* ctx, int64_t info[8]);
/* Host-to-device scan bytes copied by the last fbr_process_batch (ingest measurement). */
int fbr_ingest_bytes(fbr_ctx* ctx, double* h2d_bytes);
/* Diagnostic process-wide counters: kernel launches, blocking host synchronisations of the
 * boundary code, and host polls of the device Gauss-Newton flags; reset != 0 zeroes them. */
int fbr_debug_counters(long long* launches, long long* host_syncs, long long* flag_polls, int reset);

/* Device-resident batch (throughput measurement): stage copies the scans and guesses to HBM (and
 * computes the per-job CropBox map statistics, which depend only on the guesses); launch enqueues
 * the whole path for the staged batch (asynchronous, inputs are not modified so it may be
 * re-launched); wait blocks; results copies the latest launch's poses/stats out.
 * Launches are pipelined fbr_params.pipeline_depth deep (1..3, default 3; 1 when max_batch = 1):
 * consecutive launches rotate over the work buffers and streams of the launch slots, and
 * fbr_batch_launch returns once the launch two before it is fully enqueued, leaving the tail of its own Gauss-Newton loop (whose length the device decides)
 * to the next launch / flush / wait call.  So launch n's projection and features run beside launch
 * n-1's last iterations.  The single-scan entry points (fbr_project, fbr_register*,
 * fbr_process_scan) share the device buffers and drop a staged batch (after enqueueing every
 * launch in flight): fbr_batch_launch then returns FBR_ERR_STATE until the next fbr_batch_stage.
 * Without deskew tables the staged scans live on the device as 16-B records (x, y, z, ring):
 * intensity and time reach no batch result (poses, statistics, feature masks) and are not copied;
 * a batch staged that way and then given deskew tables (fbr_set_deskew) is reported FBR_ERR_STATE
 * at launch (stage it again). */
int fbr_batch_stage(fbr_ctx* ctx, const fbr_point_xyzirt* const* scans, const int64_t* n_in,
                    int n_jobs, const float* poses_in /* [n_jobs][6] */);
int fbr_batch_launch(fbr_ctx* ctx);
/* Enqueue the rest of every launch in flight (host side only; no device synchronisation). */
int fbr_batch_flush(fbr_ctx* ctx);
int fbr_batch_wait(fbr_ctx* ctx);
/* A job whose features exceeded the device capacity (k_features' window / segment limits) does not
 * fail the batch: it gets status FBR_REG_FEATURE_CAPACITY and its guess as pose, and the others
 * their results (fbr_batch_results, fbr_process_batch). */
int fbr_batch_results(fbr_ctx* ctx, float* poses_out /* [n_jobs][6] */,
                      fbr_reg_stats* stats /* [n_jobs] or NULL */);
/* Whole feature masks for batch jobs (featureExtraction.h:178-285, cloudLabel).  By default a batch
 * resolves each segment's surf walk only within reach of its end, the only picks that reach a pose
 * or a statistic, so its label masks are incomplete.  With on != 0, the following fbr_batch_launch
 * calls run every walk whole (as fbr_extract_features does), at some cost in throughput; results
 * are the same either way. */
int fbr_batch_set_full_masks(fbr_ctx* ctx, int on);
/* cloudLabel of job `job` of the latest launch (1 corner, -1 picked surf, 0), one entry per
 * projected point: *n_out = the job's point count (cloud_info order).  FBR_ERR_STATE unless that
 * launch ran with full masks; FBR_ERR_CAPACITY (with *n_out set) if cap < *n_out.  Waits for the
 * launches in flight. */
int fbr_batch_labels(fbr_ctx* ctx, int job, int8_t* label, int64_t cap, int64_t* n_out);
/* Enqueue (on the ctx stream, after every launch in flight) a copy of the latest launch's per-job
 * pose records {pose[6] f32, iterations i32, status i32} = 32 B/job into `device_dst` (device
 * memory of the ctx's device, [n_jobs][8] x 4 B) — the payload of the cross-GPU pose all-gather. */
int fbr_batch_export(fbr_ctx* ctx, void* device_dst);
/* Pipelined form: export the records of the oldest launch not yet exported, if it is fully
 * enqueued (after fbr_batch_launch n: at least launch n - (pipeline_depth - 1); after fbr_batch_flush:
 * every launch), without waiting for the launches in flight; launches are exported in launch
 * order, each once.  The copy runs on that launch's stream after it, and after the
 * work queued so far on `wait_stream` (a HIP stream of the caller still reading device_dst, or
 * NULL); *export_stream receives the stream to wait on before reading device_dst, *launch_id the
 * launch number (0, 1, ... since the context was created), or -1 (nothing to export: no copy). */
int fbr_batch_export_ready(fbr_ctx* ctx, void* device_dst, void* wait_stream, void** export_stream,
                           int64_t* launch_id);
/* ---- multi-GPU pose gather ---------------------------------------------------
 * Scans shard across the GPUs of a node: one process (and one ctx) per GPU, each registering its
 * own contiguous block of jobs against its replica of the map; nothing is exchanged on the data
 * path.  The only collective is the all-gather of the 32-B pose records {pose[6] f32, iterations
 * i32, status i32} over RCCL (xGMI), after each launch.  librccl is loaded on the first call
 * (FBR_ERR_UNSUPPORTED if it cannot be); a one-GPU host never needs it.
 *   rank 0:     fbr_comm_unique_id(id), then hands id to the other ranks (any out-of-band channel);
 *   every rank: fbr_comm_create(&comm, ctx, id, nranks, rank, max_jobs_per_rank)  (blocks until
 *               all ranks joined), then per launch fbr_batch_allgather(ctx, comm, launch_id, recv,
 *               wait_stream, &stream) with the same launch_id on every rank.
 * max_jobs_per_rank must be at least the ctx's fbr_params.max_batch (FBR_ERR_CAPACITY otherwise), so
 * no staged batch can exceed the communicator's blocks once it exists. */
#define FBR_COMM_ID_BYTES 128
typedef struct fbr_comm fbr_comm;
int fbr_comm_unique_id(uint8_t id_out[FBR_COMM_ID_BYTES]);
int fbr_comm_create(fbr_comm** out, fbr_ctx* ctx, const uint8_t id[FBR_COMM_ID_BYTES], int nranks, int rank,
                    int max_jobs_per_rank);
/* One process driving several devices (one host thread, one ctx and one rank per device, SURVEY §7
 * step 7): the communicators of all n contexts at once, rank i = ctxs[i] (distinct devices), made
 * with one RCCL unique id inside an ncclGroupStart / ncclGroupEnd.  Each thread then calls
 * fbr_batch_allgather with its own ctx and out[i], the same launch ids on every thread; each
 * communicator is destroyed with fbr_comm_destroy. */
int fbr_comm_create_local(fbr_comm** out /* [n] */, fbr_ctx* const* ctxs, int n, int max_jobs_per_rank);
int fbr_comm_destroy(fbr_comm* comm);
/* Collective (every rank, same launch_id; -1 = the latest launch): the records of that launch of
 * every rank into recv = [nranks][max_jobs_per_rank][8] x 4 B (device memory of the ctx's device;
 * rank r's block holds its staged jobs in order, then zero records).  Records follow
 * fbr_batch_results (a job over the feature capacity: its guess, FBR_REG_FEATURE_CAPACITY).  The
 * launch is first enqueued to its end (the host follows its GN flags); the export and the
 * all-gather then run on that launch's stream, returned in *done_stream (wait on it before reading
 * recv), or, with done_stream NULL, joined into the ctx stream.  Consecutive calls are ordered on
 * the device (each after the previous one's all-gather).  recv is written only after the work
 * queued so far on `wait_stream` (a HIP stream of the caller still reading the previous result out
 * of recv, or NULL when recv is read only on *done_stream / the ctx stream), so one recv buffer may
 * serve every call.
 * The launch must still own its work slot (one of the last pipeline_depth launches of the staged
 * batch): FBR_ERR_STATE otherwise.  Every argument and state check runs before anything is
 * enqueued, but the call is a collective: a rank that returns an error has not joined the
 * all-gather, its peers stay blocked in it, and the caller must tear the group down (every rank:
 * fbr_comm_destroy, which aborts the RCCL communicator after a failed call). */
int fbr_batch_allgather(fbr_ctx* ctx, fbr_comm* comm, int64_t launch_id, void* recv, void* wait_stream,
                        void** done_stream);

/* Sum of the per-scan algorithmic byte counts of the last completed batch (roofline input). */
int fbr_batch_bytes(fbr_ctx* ctx, double* bytes_total, double* bytes_gn);

/* Kernel timing with HIP events recorded on the ctx stream around every launch of the named
 * kernel ("gn_residual", "project", ...). */
int fbr_set_profiling(fbr_ctx* ctx, int enable);
/* Restrict the timing to a comma-separated list of kernel names (NULL or "" = all kernels). */
int fbr_set_profiling_kernels(fbr_ctx* ctx, const char* names);
int fbr_kernel_time(fbr_ctx* ctx, const char* kernel, double* total_ms, int64_t* launches);
void* fbr_stream(fbr_ctx* ctx);

/* VoxelGrid<PointXYZI>::filter on the device (the kernel every DS in the path uses). */
int fbr_voxel_grid(fbr_ctx* ctx, const fbr_point_xyzi* in, int64_t n, float leaf,
                   fbr_point_xyzi* out, int64_t* n_out);

/* Diagnostic: device numerics probe.  For i < n writes out[6i..6i+5] = {sqrtf(|a|), a/b,
 * atan2f(a,b), a*b+b*a-a, sinf(a), cosf(a)} computed by the device kernels' primitives (tests
 * compare the bits with the host libm the reference uses). */
int fbr_selftest_math(int n, const float* a, const float* b, float* out);

/* Diagnostic: cv::eigen of n symmetric 6x6 float matrices a[36i..36i+35] (the degeneracy step,
 * mapOptmization.h:1353) by the single-lane and the wave-parallel device Jacobi; out[84i..] =
 * {6 eigenvalues, 36 eigenvector entries} of each (tests compare both with the host restatement). */
int fbr_selftest_eigen6(int n, const float* a, float* out);

/* Diagnostic: the degeneracy fast path of the iteration-0 solve.  out[i] = 1 when every eigenvalue
 * of the symmetric 6x6 float matrix a[36i..36i+35] is certified above thr (LDL^T of A - (thr +
 * 1e-3 ||A||_F) I in double), so isDegenerate (mapOptmization.h:1353-1366) is false without the
 * Jacobi; 0 = not certified (the device then runs cv::eigen's Jacobi). */
int fbr_selftest_eig_certified(int n, const float* a, float thr, int32_t* out);

/* Diagnostic: PCL VoxelGrid's point order inside voxels.  perm[0..n) = the index order the device's
 * emulation of std::sort's partition phase (libstdc++ introsort, fbr_introsort.h) leaves the
 * (keys[i], i) pairs in; a stable sort of that sequence by key is std::sort's result.  lds = 1
 * runs the LDS variant of the per-segment kernels (n <= 8192), 2 LDS keys with global-memory
 * positions (the mapping-DS kernel's, n <= 18432), 3 the per-ring filter's shape (512 threads, all
 * in LDS, n <= 4096, whole-workgroup partitions from 128 elements), 0 the global-memory one. */
int fbr_selftest_voxel_order(int64_t n, const uint32_t* keys, int lds, uint32_t* perm);
/* Diagnostic: the VoxelGrid kernels' stable LSD radix sorts on one array of n keys (the low
 * `nbits` significant), one workgroup: variant 0 = the per-ring filter's LDS sort (512 threads,
 * 8-bit digits, n <= 4096), 1 = the per-segment LDS sort (256 threads, 9-bit digits, n <= 4096),
 * 2 = the global-scratch sort (1024 threads), 3 = the mapping DS's in-place LDS sort (1024 x 18),
 * 4 = variant 3 with ballot-leader digit counts, 5 = variant 4 with round 3's wave-uniform early
 * exits in its count and scatter loops (the exact form round 3 reverted).  keys_inout receives
 * the sorted keys, perm the source index of every sorted position. */
int fbr_selftest_radix_sort(int64_t n, int nbits, int variant, uint32_t* keys_inout, uint32_t* perm);

/* Measurement helper: achievable HBM bandwidth of a device-wide float4 copy of `bytes` (read +
 * write counted), averaged over `iters` launches (the STREAM-copy figure bench.py reports next to
 * the 8 TB/s spec peak). */
int fbr_stream_copy_bandwidth(int hip_device, int64_t bytes, int iters, double* gbps);
/* Measurement helper: the VALU issue roof.  Every SIMD holds waves_per_simd (1..8) waves, each lane
 * running 8 independent chains of one VALU instruction (kind 0 v_fma_f32, 1 v_add_u32, 2
 * v_pk_fma_f32) for 32 * iters instructions; *ginst_per_s = wave-level instructions per second over
 * `reps` launches, *ms_per_launch (optional) the launch time (tools/valu_calib.py). */
int fbr_valu_peak(int hip_device, int waves_per_simd, int kind, int iters, int reps, double* ginst_per_s,
                  double* ms_per_launch);

/* pcl::getTransformation / pcl::getTranslationAndEulerAngles (row-major 4x4 float). */
void fbr_affine_from_pose(const float pose[6], float m[16]);
void fbr_pose_from_affine(const float m[16], float pose[6]);

#ifdef __cplusplus
}
#endif
#endif /* FBR_H_ */
