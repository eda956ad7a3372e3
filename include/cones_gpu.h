/* cones_gpu.h — C-ABI of the MI355X (gfx950) LiDAR cone-detection hot path.
 *
 * Drop-in for the bodies of the two ROS callbacks of dmn-sjk/cones_perception
 * (reference paths relative to its repository root):
 *   - GroundRemover::cloud_handler   src/ground_removal.cpp:50-89  (lines 51-79 replaced)
 *   - ConeDetector::cloud_handler    src/cone_detection.cpp:130-187 (lines 138-167 and the
 *     centroid arithmetic 261-279 replaced; the colour RPC 342-363 and the 4-topic publish
 *     177-186 stay in the node; the tracking 282-339 and the cone re-crop 222-238 are
 *     offered as cg_tracker_* and cg_recrop below)
 * The reference has no plugin API; its seam is those callback bodies, which call PCL
 * (fromROSMsg, VoxelGrid, search::KdTree, EuclideanClusterExtraction, toROSMsg) and libm.
 * INTEGRATION.md shows the patched callbacks. Plain C types only: no torch, no C++ in
 * signatures, no exceptions across the boundary.
 *
 * Threading: a handle is not thread-safe (the reference runs one callback at a time under
 * ros::spin, src/ground_removal.cpp:47, src/cone_detection.cpp:127). Single-frame calls are
 * synchronous. Batch calls are asynchronous on the given HIP stream.
 */
#ifndef CONES_GPU_H
#define CONES_GPU_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------------------- */
#define CG_OK          0
#define CG_E_INVALID   1   /* bad argument / unsupported cloud layout */
#define CG_E_DEVICE    2   /* HIP runtime error or no gfx950 device */
#define CG_E_OOM       3   /* device or pinned host allocation failed */
#define CG_E_CAPACITY  4   /* frame larger than the engine supports (N > 2^28 points) */

/* result flags (cg_detect_result.flags, batch header word CG_HDR_FLAGS) */
#define CG_F_VOXEL_PASSTHROUGH 0x1u  /* PCL VoxelGrid overflow guard hit: voxel cloud = input */
#define CG_F_GLOBAL_SCRATCH    0x2u  /* detector input too large for the LDS backend; ran from HBM */
#define CG_F_ORDER_CANONICAL   0x4u  /* >16 clusters: order is (size desc, seed asc); PCL's
                                        std::sort may order equal-size clusters differently */
#define CG_F_VOXEL_POINT_ORDER 0x8u  /* voxel sums ran in ascending point order, not in PCL's
                                        std::sort order (cg_set_voxel_order, the halo form) */

/* ---- parameters --------------------------------------------------------------------- */
/* Field names are the YAML keys, misspellings kept (config/ *.yaml). */
typedef struct cg_params {
    /* config/ground_removal_params.yaml; defaults src/ground_removal.cpp:18-19 */
    int32_t num_of_sectors;          /* read but inert: sector width is fixed at 22 deg (G1) */
    float   default_lowest_point;
    /* config/cones_detection_params_*.yaml; defaults src/cone_detection.cpp:27-43 */
    double  distance_treshold_max;
    double  distance_treshold_min;
    double  level_threshold;
    double  angle_threshold;         /* degrees */
    int32_t min_cluster_size;
    int32_t max_cluster_size;
    double  cone_position_extension_length;
    double  voxel_filter_leaf_size_x;
    double  voxel_filter_leaf_size_y;
    double  voxel_filter_leaf_size_z;
    double  cones_matching_dist_theshold;  /* tracking only (out of path); carried for the node */
} cg_params;

/* Class-member defaults of the reference (src/ground_removal.cpp:18-19,
 * src/cone_detection.cpp:27-43), i.e. what a node uses for a missing ROS param. */
void cg_params_init(cg_params* p);

/* ---- input cloud -------------------------------------------------------------------- */
/* Borrowed description of a sensor_msgs/PointCloud2. Fields are located by byte offset; pass
 * -1 for a field that is absent or not FLOAT32 x1 (pcl::fromROSMsg then leaves it at 0).
 * Reproducing src/cone_detection.cpp:142-151 (detector input without an intensity field gets
 * a fake FLOAT32 field at offset 0) is the caller's job: pass off_intensity = 0. */
typedef struct cg_cloud_view {
    const void* data;        /* PointCloud2::data (host memory for the single-frame calls) */
    uint32_t width, height;  /* N = width * height */
    uint32_t point_step, row_step;
    int32_t  off_x, off_y, off_z, off_intensity;
    uint8_t  is_dense;
} cg_cloud_view;

/* ---- handle ------------------------------------------------------------------------- */
typedef struct cg_handle cg_handle;

/* Create a handle on HIP device `device` (one stream, lazily grown device buffers). */
int  cg_create(const cg_params* params, int device, cg_handle** out);
int  cg_destroy(cg_handle* h);
int  cg_set_params(cg_handle* h, const cg_params* params);
/* Voxel summation order of the VoxelGrid stage (src/cone_detection.cpp:240-249). PCL sorts
 * index_vector with std::sort, an unstable introsort, so the float sums of a voxel's points
 * run in libstdc++'s permutation of the equal-idx points; CG_VOXEL_ORDER_PCL reproduces that
 * permutation and every voxel bit, CG_VOXEL_ORDER_POINT sums in ascending point index (same
 * voxels, clusters and cluster sets; voxel coordinates may differ in the last bits).
 * Default: CG_VOXEL_ORDER_PCL. */
#define CG_VOXEL_ORDER_POINT 0
#define CG_VOXEL_ORDER_PCL   1
int  cg_set_voxel_order(cg_handle* h, int order);
/* Thread-local message for the last failing call on this thread ("" if none). */
const char* cg_last_error(void);

/* ---- single-frame calls (ROS drop-in) ------------------------------------------------ */
/* GroundRemover::cloud_handler body (src/ground_removal.cpp:51-79): per-22-degree-sector
 * lowest z, keep points with !(z < low + 0.1), stable, then zero-pad back to N points
 * (pcl::PointXYZI() = x=y=z=0, data[3]=1, intensity=0). Output data is N x 32 B in PCL
 * PointXYZI layout (x,y,z @0,4,8; 1.0f @12; intensity @16; 12 zero bytes) — the bytes
 * toROSMsg would publish. Library-owned; valid until the next call on the handle. */
typedef struct cg_ground_result {
    uint32_t n_points;       /* N, preserved (G5) */
    uint32_t n_kept;         /* K */
    uint32_t width, height;  /* organized shape preserved (resize keeps width*height == N) */
    const uint8_t* data;     /* N * 32 bytes */
} cg_ground_result;
int cg_ground_remove(cg_handle* h, const cg_cloud_view* in, cg_ground_result* out);

/* ConeDetector::cloud_handler hot part (src/cone_detection.cpp:156-175, 189-220, 240-279):
 * filter_points_position -> VoxelGrid -> KdTree + EuclideanClusterExtraction -> per-cluster
 * xy centroid pushed 0.05 m outward. Arrays are library-owned, valid until the next call. */
typedef struct cg_detect_result {
    uint32_t n_points;           /* N of the input */
    uint32_t n_kept;             /* K (pipeline only; = N for cg_detect) */
    uint32_t n_filtered;         /* M, points surviving filter_points_position */
    uint32_t n_voxels;           /* V, points of the VoxelGrid output */
    uint32_t n_clusters;         /* C */
    uint32_t flags;              /* CG_F_* */
    const float*   voxels;           /* V x 4: x, y, z, intensity (PCL output order) */
    const int32_t* labels;           /* V: cluster rank in output order, or -1 */
    const int32_t* cluster_offsets;  /* C + 1 */
    const int32_t* cluster_indices;  /* cluster_offsets[C] voxel indices, ascending per cluster */
    const float*   centroids;        /* C x 2: x, y after the radial push (z = 0) */
} cg_detect_result;
/* Synchronous. A frame of <= 65,536 points is launched before its bytes are staged: the call
 * copies in->data into pinned memory chunk by chunk behind the launch, and each chunk's
 * workgroup reads its chunk over PCIe once published. in->data is read until the call
 * returns. A chunk workgroup waits at most 200 ms for its chunk (a host thread descheduled
 * that long); the call then runs the frame again with the whole message copied by DMA, so a
 * slow host makes the call slower, never failed. */
int cg_detect(cg_handle* h, const cg_cloud_view* in, cg_detect_result* out);

/* ground_removal -> cone_detection composition of launch/cones_perception.launch:17-37
 * (ground_removal:=true), fused: the detector sees exactly the groundless cloud the ground
 * node would publish (K kept points in order, then N-K zero points). */
int cg_pipeline(cg_handle* h, const cg_cloud_view* in, cg_detect_result* out);

/* ---- batch engine (device-resident frames) ------------------------------------------ */
/* n_frames uniform frames of n_points PointCloud2 points each, contiguous rows
 * (row_step = n_points * point_step), frame f at d_data + f * frame_stride (device memory). */
typedef struct cg_batch {
    const void* d_data;
    uint64_t frame_stride;
    uint32_t n_frames, n_points, point_step;
    int32_t  off_x, off_y, off_z, off_intensity;
    uint8_t  is_dense;
} cg_batch;

#define CG_MODE_PIPELINE 0   /* ground removal + detector (cg_pipeline semantics) */
#define CG_MODE_DETECT   1   /* detector only (cg_detect semantics) */

/* Enqueue one pass of the hot path over the batch on `hip_stream` (hipStream_t; NULL = the
 * handle's own stream). Results stay on the device until the next call on the handle. Frames
 * of up to 65,536 points run as one launch, one workgroup per frame. Frames of more run
 * through the multi-workgroup large-frame path one frame at a time: with PCL's voxel order (the
 * default) and up to 2^22 points, sized on the device and replayed from a captured hipGraph per
 * frame, nothing synchronised; otherwise the call synchronises the stream once per frame (the
 * frame's counts size its backend).
 * A handle's calls are ordered whatever stream each names: a call on another stream than the
 * handle's previous call waits for that stream's work queued so far (which must still exist). */
int cg_run_batch(cg_handle* h, const cg_batch* b, int mode, void* hip_stream);

/* n_calls batch calls in one: call i is cg_run_batch(handles[i], &batches[i], mode,
 * hip_streams[i]), in order (a handle may appear several times). Every call's arguments are
 * checked before any is enqueued; a call that fails stops the sequence, and *n_done (optional)
 * is the number of calls enqueued. For a server that enqueues many batches over several
 * handles and streams at once: one crossing of the ABI, and the device selected once. */
int cg_run_batches(cg_handle* const* handles, const cg_batch* batches, uint32_t n_calls, int mode,
                   void* const* hip_streams, uint32_t* n_done);

/* Per-frame header words in the device result buffer. */
#define CG_HDR_N      0
#define CG_HDR_K      1
#define CG_HDR_M      2
#define CG_HDR_V      3
#define CG_HDR_C      4
#define CG_HDR_FLAGS  5
#define CG_HDR_ERR    7   /* 0 for a good frame. Nonzero: the frame's results are void and
                             cg_batch_fetch fails with CG_E_DEVICE; a caller reading d_header
                             directly must drop such a frame. CG_HDR_E_WAIT: a large frame's
                             device-side wait gave up (never expected; ABI 0.2.0+) */
#define CG_HDR_WORDS  8
#define CG_HDR_E_WAIT 0x57414954u

typedef struct cg_batch_results {
    uint32_t n_frames;
    uint32_t capacity;                 /* per-frame slot length (points) of each array */
    const uint32_t* d_header;          /* n_frames x CG_HDR_WORDS */
    const float*    d_voxels;          /* n_frames x capacity x 4 */
    const int32_t*  d_labels;          /* n_frames x capacity */
    const int32_t*  d_cluster_offsets; /* n_frames x (capacity + 1) */
    const int32_t*  d_cluster_indices; /* n_frames x capacity */
    const float*    d_centroids;       /* n_frames x capacity x 2 */
} cg_batch_results;
int cg_batch_results_get(cg_handle* h, cg_batch_results* out);
/* Synchronise the batch stream and copy one frame's results to handle-owned host buffers. */
int cg_batch_fetch(cg_handle* h, uint32_t frame, cg_detect_result* out);

/* ---- one large frame tiled across ranks (C5; one process per GPU) ----------------------- */
/* A rank's tile: points [first, first + n) of a frame of n_total points, in device memory
 * (d_data = the tile's first point). Pipeline semantics (ground removal + detector), results
 * bit-identical to the single-GPU call on the whole frame. Protocol per frame:
 *   1. cg_tile_front on every rank -> keys; merge across ranks: words 0-17 MIN (sector-minimum
 *      keys, order-preserving), word 18 bitwise OR (sector bins holding points);
 *   2. cg_tile_decide with the merged keys -> counts; merge: K, survivors, finite survivors SUM,
 *      words 3-5 MIN (bounds minimum keys), words 6-8 MAX (bounds maximum keys);
 *   3. cg_tile_survivors copies the rank's survivors (x,y,z,i float4 + frame index) out; the
 *      survivors of all ranks are gathered (any order) on one rank, which runs
 *   4. cg_tile_backend with the merged counts; results as frame 0 of cg_batch_results_get /
 *      cg_batch_fetch. Calls synchronise the handle's stream. */
typedef struct cg_tile {
    const void* d_data;
    uint32_t first, n, n_total;
    uint32_t point_step;
    int32_t  off_x, off_y, off_z, off_intensity;
} cg_tile;
#define CG_TILE_KEYS   19
#define CG_TILE_COUNTS 9
int cg_tile_front(cg_handle* h, const cg_tile* t, uint32_t* keys);
int cg_tile_decide(cg_handle* h, const uint32_t* merged_keys, uint32_t* counts);
int cg_tile_survivors(cg_handle* h, float* d_points, uint32_t* d_index, uint32_t capacity);
int cg_tile_backend(cg_handle* h, const float* d_points, const uint32_t* d_index, uint32_t n_survivors,
                    const uint32_t* merged_counts, uint32_t n_total);
/* The same protocol with the keys and counts left on the device, for device-side merges (RCCL
 * all-reduce / all-gather on the caller's stream): nothing here synchronises. stream: the
 * caller's hipStream_t (NULL: the handle's own); every call on the frame passes the same one.
 *   cg_tile_front_async: step 1; the CG_TILE_KEYS keys to d_keys (device memory);
 *   cg_tile_decide_async: step 2 from merged keys in device memory; the CG_TILE_COUNTS
 *     counts to d_counts (device memory);
 *   cg_tile_survivors_async: step 3 for a survivor count n the caller already holds (its
 *     own entry of the gathered counts);
 *   cg_tile_backend_own: step 4 on this rank's own survivors, where they already are, when
 *     its tile is the whole frame (one rank): the counts are the rank's own. Like the
 *     single-GPU call it reads the frame's survivor count back once to size the backend. */
int cg_tile_front_async(cg_handle* h, const cg_tile* t, uint32_t* d_keys, void* hip_stream);
int cg_tile_decide_async(cg_handle* h, const uint32_t* d_merged_keys, uint32_t* d_counts, void* hip_stream);
int cg_tile_survivors_async(cg_handle* h, float* d_points, uint32_t* d_index, uint32_t n, void* hip_stream);
int cg_tile_backend_own(cg_handle* h, uint32_t n_total, void* hip_stream);

/* Spatial tiling with a halo exchange, in place of steps 3-4. The frame's
 * PCL voxel lattice (from the merged bounds) is cut into slabs of voxel columns along x; a
 * voxel lies in exactly one slab, and every rank voxelises and clusters its own slab:
 *   a. cg_halo_plan_frame with the merged counts -> the lattice, slabs, band width and the
 *      slab of the zero pads' voxel (host arithmetic, identical on every rank). A PCL
 *      overflow-guard frame (passthrough) has no lattice: use steps 3-4;
 *   b. cg_halo_owner: the slab of each of the rank's survivors (-1: non-finite, not
 *      voxelised). Survivors go to their slab's rank (all-to-all, in frame-index order);
 *   c. cg_halo_local on the slab's survivors (plus the pads on the pads' slab) -> one record
 *      per voxel in idx order: x, y, z, intensity (PCL centroid), idx, idx of the lowest voxel
 *      of its component within the slab, 0, 0;
 *   d. the records of a slab's lowest `band` voxel columns go to the rank of the slab below
 *      (point to point); there cg_halo_edges tests them against the own records of the top
 *      `band` columns -> pairs (own component idx, neighbour component idx), one per distinct
 *      component pair a halo voxel joins. n_pairs is exact; call again with capacity >=
 *      n_pairs when it exceeds capacity;
 *   e. every slab's records and pairs go to one rank: cg_halo_merge orders the voxels, unites
 *      the components and writes the clusters, results as cg_tile_backend's.
 * One slab (plan->slabs == 1: one rank, or a lattice narrower than two bands) has no boundary:
 * cg_halo_local then takes every survivor of the frame (n = merged_counts[1], non-finite ones
 * included, n_pads = plan->n_pads; d_rec and capacity unused) and writes the frame's results in
 * the handle itself, asynchronously on the handle's stream, with *n_vox = 0; steps b, d and e
 * are skipped.
 * Results are bit-identical to the single-GPU call on the whole frame in frame-index voxel
 * order (cg_set_voxel_order CG_VOXEL_ORDER_POINT). */
#define CG_HALO_REC_WORDS 8
typedef struct cg_halo_plan {
    uint32_t passthrough;   /* the voxel grid's overflow guard hit (no lattice) */
    int32_t  min_b[3];      /* pcl::VoxelGrid min_b_ and div_b_ of the whole frame */
    uint32_t div_b[3];
    uint32_t slabs;         /* slab s owns voxel columns [s * slab_w, (s + 1) * slab_w) (last: to div_b[0]) */
    uint32_t slab_w;
    uint32_t band;          /* voxel columns within which an edge can cross a slab boundary */
    int32_t  pad_slab;      /* slab of the zero pads' voxel; -1 when no pad reaches the detector */
    uint32_t n_pads;
    uint32_t key_bits;      /* bits of idx (plus one: non-finite points sort last) */
} cg_halo_plan;
int cg_halo_plan_frame(cg_handle* h, const uint32_t* merged_counts, uint32_t n_total, uint32_t n_ranks,
                       cg_halo_plan* plan);
int cg_halo_owner(cg_handle* h, const cg_halo_plan* plan, const float* d_points, uint32_t n, int32_t* d_slab);
int cg_halo_local(cg_handle* h, const cg_halo_plan* plan, const float* d_points, const uint32_t* d_index,
                  uint32_t n, uint32_t n_pads, const uint32_t* merged_counts, uint32_t n_total, uint32_t* d_rec,
                  uint32_t capacity, uint32_t* n_vox);
int cg_halo_edges(cg_handle* h, const uint32_t* d_own, uint32_t n_own, const uint32_t* d_halo, uint32_t n_halo,
                  uint32_t* d_pairs, uint32_t capacity, uint32_t* n_pairs);
int cg_halo_merge(cg_handle* h, const cg_halo_plan* plan, const uint32_t* d_rec, uint32_t n_rec,
                  const uint32_t* d_pairs, uint32_t n_pairs, const uint32_t* merged_counts, uint32_t n_total);

/* ---- colour classifier service ----------------------------------- */
/* ColorClassifier.handle_classify_color (scripts/color_classifier_server.py:81-124) with its
 * to_image (131-156) and the dam_net CNN it runs through TFLite (models/dam_net/dam_net.tflite),
 * on the GPU. The node's colour-service call (src/cone_detection.cpp:342-363) can be served by
 * it in process. Weights: the .tflite graph's constants packed as float32, in this order
 * (shapes as in the graph): conv2d kernel [16][3][3] (OHW, one input channel), conv2d bias [16],
 * conv2d_1 kernel [32][3][3][16] (OHWI), conv2d_1 bias [32], batch-norm MUL [32], batch-norm
 * ADD [32], dense kernel [3][64], dense bias [3]. cones_perception_amd.colornet reads them from
 * the .tflite file (the reference's ~model_path). */
#define CG_COLORNET_WEIGHTS 5059
#define CG_COLOR_SKIPPED     (-1)  /* empty cloud: the reference's response has no entry for it */
#define CG_COLOR_INDEX_ERROR (-2)  /* a point's image row falls outside the 15 rows: the reference raises IndexError */
#define CG_COLOR_RANGE_ERROR (-3)  /* an intensity outside [0, 255]: the reference's interp1d raises ValueError */
int cg_colornet_set(cg_handle* h, const float* weights, uint32_t n_weights);
/* points: host x, y, z, intensity float32, cone c's points at [offsets[c], offsets[c + 1]).
 * colors[c]: 1 yellow, 2 blue, 3 orange, 0 unknown (max probability < 0.8), or a negative code
 * above. probs (n_cones x 3) and images (n_cones x 15 x 12 uint8, to_image's pixels) are
 * optional (NULL). Synchronous. */
int cg_classify_colors(cg_handle* h, const float* points, const uint32_t* offsets, uint32_t n_cones,
                       int32_t* colors, float* probs, uint8_t* images);

/* ---- detector node after the hot path (src/cone_detection.cpp:171-186, 222-339) -------- */
/* Cone re-crop, ConeDetector::get_reconstructed_cone (src/cone_detection.cpp:222-238): for each
 * cone centre (x, y), every point of the last single-frame call's detector input (the "whole
 * cloud" get_centroid_clouds receives: the cg_detect input after decoding, or the groundless
 * cloud of a cg_pipeline call, zero pads included) with
 *     cx - 0.228f/1.5 <= x <= cx + 0.228f/1.5  and the same in y   (double compares),
 * in cloud order, as x, y, z, intensity. This is what the colour classifier receives.
 * Arrays are library-owned, valid until the next call on the handle. */
typedef struct cg_crop_result {
    uint32_t n_centers;
    const uint32_t* offsets;  /* n_centers + 1 */
    const float*    points;   /* offsets[n_centers] x 4 */
} cg_crop_result;
int cg_recrop(cg_handle* h, const float* centers_xy, uint32_t n_centers, cg_crop_result* out);
/* The same for frame `frame` of the last cg_run_batch on the handle (pipeline or detect
 * mode). The batch's input must still be in the caller's device memory; the call waits for
 * the batch's stream. */
int cg_batch_recrop(cg_handle* h, uint32_t frame, const float* centers_xy, uint32_t n_centers,
                    cg_crop_result* out);

/* Tracking and the four colour clouds, ConeDetector::get_centroid_clouds
 * (src/cone_detection.cpp:251-339). Host code; no device. One frame is two calls, split where
 * the reference calls the colour service (src/cone_detection.cpp:320-327):
 *   cg_tracker_match  with the frame's centroids in cluster order (cg_detect_result.centroids):
 *                     status[c] = CG_TRACK_DROPPED (not published: no previous frame, or no
 *                     previous cone within cones_matching_dist_theshold while
 *                     use_points_buffer), a colour 0..3 (published in that cloud: colour known
 *                     from the previous frame, or 0 = unknown when classify_colors is off), or
 *                     CG_TRACK_NEED_COLOR (re-crop with cg_recrop and classify);
 *   cg_tracker_commit with the colour service's response for the CG_TRACK_NEED_COLOR
 *                     centroids in request order: n_colors <= n_need colours, applied to the
 *                     first n_colors of them, the rest unknown (src/cone_detection.cpp:328,
 *                     357-358; the reference's server skips empty crops, so a response can be
 *                     short); NULL: the service call failed, all unknown; more colours than
 *                     n_need: CG_E_INVALID. Builds the clouds in the reference's push order
 *                     and rolls the previous-frame state.
 * cg_tracker_cloud then returns colour cloud `color` as (x, y) pairs (z = 0, intensity = 0):
 * the points the node publishes on cones_topics[color] (src/cone_detection.cpp:46-49). */
#define CG_NUM_COLORS        4     /* perception_handling::Color: unknown, yellow, blue, orange */
#define CG_TRACK_DROPPED    (-1)
#define CG_TRACK_NEED_COLOR (-2)
typedef struct cg_track_params {
    uint8_t classify_colors;              /* ~classify_colors: node default 1, launch files 0 */
    uint8_t use_points_buffer;            /* ~use_points_buffer: node default 0, launch files 1 */
    double  cones_matching_dist_theshold; /* default 0.5 */
} cg_track_params;
typedef struct cg_tracker cg_tracker;
void cg_track_params_init(cg_track_params* p);   /* the node's class-member defaults */
int  cg_tracker_create(const cg_track_params* p, cg_tracker** out);
int  cg_tracker_destroy(cg_tracker* t);
int  cg_tracker_set_params(cg_tracker* t, const cg_track_params* p);
int  cg_tracker_match(cg_tracker* t, const float* centroids_xy, uint32_t n, int32_t* status, uint32_t* n_need);
int  cg_tracker_commit(cg_tracker* t, const int32_t* colors, uint32_t n_colors);
int  cg_tracker_cloud(const cg_tracker* t, int color, const float** xy, uint32_t* n);

/* Exported library version string. */
/* "cones_gpu MAJOR.MINOR.PATCH (gfx950)"; INTEGRATION.md, ABI history */
const char* cg_version(void);

/* ---- synthetic frames (harness; src-free of any GPU call) ---------------------------- */
typedef struct cg_synth_cfg {
    uint32_t rings, cols;            /* N = rings * cols */
    float    elev_min_deg, elev_max_deg, mount_height, wall_radius, range_noise;
    uint32_t point_step;             /* 16 (xyzi) or 32 (PCL PointXYZI layout) */
    uint32_t column_major;           /* 1: point = col*rings + ring; 0: ring*cols + col */
    uint32_t cones_per_row;
    uint32_t clutter;                /* extra posts (dense scenes) */
    uint64_t seed;
} cg_synth_cfg;
void cg_synth_default(cg_synth_cfg* c);
int  cg_synth_frames(const cg_synth_cfg* cfg, uint64_t first_frame, uint32_t n_frames,
                     void* out, uint64_t frame_stride, uint32_t n_threads);

#ifdef __cplusplus
}
#endif
#endif /* CONES_GPU_H */
