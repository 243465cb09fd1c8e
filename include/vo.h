/*
 * vo.h — C-ABI of libvo, the MI355X-native stereo visual-odometry front end.
 *
 * Drop-in boundary.  The reference (ivario123/r7020e-visual-
 * odometry, MATLAB) has no native interface: its per-frame path calls
 * MathWorks toolbox functions from VO.m.  Each entry point below replaces one
 * of those calls; a MATLAB maintainer binds them through the MEX gateways
 * shown in INTEGRATION.md (path shadowing), a Python user through ctypes
 * (r7020e-visual-odometry_amd/vo.py).
 *
 *   entry point            replaces (reference call site)
 *   ---------------------  ---------------------------------------------------
 *   vo_sift                detectSIFTFeatures + extractFeatures(...,"SIFT")
 *                          VO.m:79-84
 *   vo_match               matchFeatures(F1, F2)  VO.m:87,283,293,311,323
 *   vo_track               find_remaining_points  VO.m:280-334 (4 matches +
 *                          gathers), fused on device
 *   vo_triangulate         triangulate(x1, x2, P1, P2)  VO.m:113-116,
 *                          CreateLandmarksFromFeatures.m:7
 *   vo_estworldpose        estworldpose(imagePts, worldPts, intrinsics)
 *                          VO.m:123-127 (P3P + MSAC)
 *   vo_landmarks           new-landmark filter VO.m:145-158 +
 *                          CreateLandmarksFromFeatures.m:1-21
 *   vo_step / vo_step_batch the whole loop body VO.m:70-161 (features stay
 *                          device-resident between frames)
 *   vo_step_submit_dev /   the same loop body, pipelined: batch n+1's SIFT
 *   vo_step_collect        overlaps batch n's geometry and host pose chain
 *   vo_sift_match_batch    VO.m:79-87 for a batch of independent stereo pairs
 *                          (the benchmark workload, BASELINE.json configs[1])
 *   vo_sift_ex /           the same calls taking MATLAB's column-major storage
 *   vo_match_f32 /         (images, n x 128 single descriptors) without a host
 *   vo_step_batch_ex       transpose or conversion (zero-copy MEX gateways)
 *   vo_set_landmark_frame  sharded sequences: camera-frame landmark rows, moved
 *   vo_landmarks_to_world* to the world after the gathered pose chain
 *   vo_landmarks_world_dev (CreateLandmarksFromFeatures.m:17, VO.m:130; the
 *   vo_chain_poses         _dev form on the rank's own rows, on the device)
 *
 * Conventions
 *  - Return value: VO_OK (0) or a negative VO_ERR_* code.  vo_last_error()
 *    gives a message.  VO_ERR_TOO_FEW_POINTS / VO_ERR_NO_CONSENSUS mirror the
 *    errors estworldpose throws (the reference crashes; we report and the
 *    step holds the previous pose).
 *  - Buffers are caller-allocated host memory with explicit capacities, unless
 *    a function name ends in _dev (device pointers, stream-ordered).
 *  - Images: uint8, row-major with leading dimension `ld` (bytes per row).
 *    (MATLAB is column-major: the MEX shim passes the transpose view, see
 *    INTEGRATION.md.)
 *  - Image coordinates are MATLAB 1-based pixel coordinates (x = column).
 *  - Index pairs are 1-based uint32 [P][2] row-major, ascending in column 0,
 *    exactly as matchFeatures returns them.
 *  - Matrices are row-major doubles: P1/P2 3x4 premultiply camera matrices,
 *    K 3x3, rigid transforms 4x4 (R2022b rigidtform3d.A convention).
 *  - One context per device; a context is not thread-safe.
 */
#ifndef VO_H
#define VO_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VO_OK                  0
#define VO_ERR_ARG            -1
#define VO_ERR_HIP            -2
#define VO_ERR_TOO_FEW_POINTS -3
#define VO_ERR_NO_CONSENSUS   -4
#define VO_ERR_CAPACITY       -5
#define VO_ERR_STATE          -6

/* vo_step_out.flags / vo_pair_stats.flags: a capacity was exceeded and the frame's feature
 * sets are incomplete (results then differ from an uncapped run) */
#define VO_FLAG_KEYPOINTS   1    /* an image detected more than max_keypoints keypoints */
#define VO_FLAG_CANDIDATES  2    /* an image's extremum candidates exceeded 4 x max_keypoints */

#define VO_DESC_LEN 128
#define VO_MAX_BATCH 512         /* largest max_batch of vo_create */
#define VO_STEP_DEPTH 3          /* batches vo_step_submit_dev keeps in flight */

/* detectSIFTFeatures / extractFeatures defaults (MATLAB R2022b+).
 * contrast_threshold is in OpenCV units: MATLAB's ContrastThreshold 0.0133
 * equals 0.04 / NumLayersInOctave. */
typedef struct {
    int32_t n_octave_layers;      /* NumLayersInOctave, 3 */
    float   sigma;                /* Sigma, 1.6 */
    float   contrast_threshold;   /* 0.04  (= 0.0133 * 3) */
    float   edge_threshold;       /* EdgeThreshold, 10 */
    int32_t upsample;             /* 1: first octave is the x2 upsampled image */
    int32_t max_keypoints;        /* capacity per image (keypoints beyond it are dropped, flagged) */
} vo_sift_params;

/* matchFeatures defaults: Method Exhaustive, Metric SSD, MatchThreshold 1.0
 * (percent), MaxRatio 0.6, Unique false. */
typedef struct {
    float match_threshold;        /* percent; SSD threshold = 0.04 * match_threshold on unit vectors */
    float max_ratio;              /* 0.6 */
} vo_match_params;

/* estworldpose defaults (VO.m:123-127 calls it with no options: MaxNumTrials 1000).
 * The BASELINE configs[2] bench passes max_num_trials = 2048 explicitly. */
typedef struct {
    int32_t  max_num_trials;      /* 1000 (MATLAB default); hypothesis slots the context allocates */
    double   confidence;          /* percent, 99 */
    double   max_reprojection_error; /* pixels, 1 */
    uint32_t seed;                /* Philox key (frame index is mixed in by vo_step) */
} vo_ransac_params;

typedef struct {
    double P1[12];   /* left camera 3x4 (VO.m:27-29) */
    double P2[12];   /* right camera 3x4 (VO.m:30-32) */
    double K[9];     /* left intrinsics (VO.m:35-38,50) */
} vo_calib;

typedef struct {
    float   x, y;        /* Location, 1-based */
    float   size;        /* keypoint diameter in image pixels (OpenCV KeyPoint.size) */
    float   angle;       /* orientation in degrees [0,360) (OpenCV convention) */
    float   response;    /* |DoG| at the refined extremum (Metric) */
    int32_t octave;      /* octave index, -1 = upsampled */
    int32_t layer;       /* layer within octave 1..n_octave_layers */
    float   scale;       /* Scale = size / 2 in image pixels */
} vo_keypoint;

typedef struct vo_ctx vo_ctx;

/* Defaults for every parameter block. */
void vo_default_sift_params(vo_sift_params* p);
void vo_default_match_params(vo_match_params* p);
void vo_default_ransac_params(vo_ransac_params* p);

/* Create a context on HIP device `device` for images of rows x cols, able to
 * process up to max_batch (1..VO_MAX_BATCH) stereo frames per call.  calib may be NULL (then
 * vo_step/vo_landmarks are unavailable until vo_set_calib). Returns NULL on
 * failure (message via vo_last_error(NULL)). */
vo_ctx* vo_create(int device, int rows, int cols, int max_batch,
                  const vo_calib* calib, const vo_sift_params* sift,
                  const vo_match_params* match, const vo_ransac_params* ransac);
void vo_destroy(vo_ctx* ctx);
int  vo_set_calib(vo_ctx* ctx, const vo_calib* calib);
const char* vo_last_error(const vo_ctx* ctx);

/* detectSIFTFeatures + extractFeatures for one image (host buffers).
 * kps[capacity], desc[capacity][128] (uint8 values; MATLAB gets them as
 * single).  *n_out = number of keypoints (may exceed capacity: then only
 * `capacity` are written and VO_ERR_CAPACITY is returned). */
int vo_sift(vo_ctx* ctx, const uint8_t* img, int rows, int cols, int ld,
            vo_keypoint* kps, uint8_t* desc, int capacity, int* n_out);

/* The same for an image in MATLAB's own storage: col_major = 1 means pixel (r, c) at
 * img[c * ld + r] (ld >= rows; a MEX gateway passes mxGetUint8s(I) with ld = rows, no
 * transpose on the host; the device transposes).  col_major = 0 is vo_sift. */
int vo_sift_ex(vo_ctx* ctx, const uint8_t* img, int rows, int cols, int ld, int col_major,
               vo_keypoint* kps, uint8_t* desc, int capacity, int* n_out);

/* matchFeatures(F1, F2) on SIFT descriptors (uint8 rows of 128).
 * pairs[capacity][2] 1-based; *n_pairs = matches found. */
int vo_match(vo_ctx* ctx, const uint8_t* F1, int n1, const uint8_t* F2, int n2,
             uint32_t* pairs, int capacity, int* n_pairs);

/* matchFeatures(F1, F2) on single-precision descriptor matrices exactly as MATLAB holds
 * extractFeatures' output (VO.m:83-87): n x 128 single with integer values 0..255.
 * col_major = 1: element (i, k) at F[i + k * ld] (MATLAB storage; ld >= n), so a MEX gateway
 * passes mxGetSingles(prhs[k]) with ld = n and no transpose or conversion; col_major = 0:
 * F[i * ld + k] (ld >= 128).  The matrices are copied to the device as they lie and packed to
 * u8 rows there.  Non-integer or out-of-range values -> VO_ERR_ARG.  Same results as vo_match. */
int vo_match_f32(vo_ctx* ctx, const float* F1, int n1, int ld1, const float* F2, int n2, int ld2,
                 int col_major, uint32_t* pairs, int capacity, int* n_pairs);

/* find_remaining_points (VO.m:280-334) on device.  old = previous frame's
 * stereo-aligned set (n_old rows, left/right row-aligned); cur = current
 * frame's full left (n_cl) / right (n_cr) sets.  Writes K row-aligned rows:
 * idx_out[K][3] = 1-based rows {old_row, cur_left_row, cur_right_row}
 * (old left and right stay row-aligned through VO.m:287-329), *K_out. */
int vo_track(vo_ctx* ctx,
             const uint8_t* old_l_desc, const uint8_t* old_r_desc, int n_old,
             const uint8_t* cur_l_desc, int n_cl, const uint8_t* cur_r_desc, int n_cr,
             uint32_t* idx_out, int capacity, int* K_out);

/* triangulate: n points, x1/x2 [n][2] float (1-based pixels), P1/P2 3x4
 * row-major -> X [n][3] double (values rounded through single, as MATLAB
 * returns single for single inputs). */
int vo_triangulate(vo_ctx* ctx, const float* x1, const float* x2, int n,
                   const double P1[12], const double P2[12], double* X);

/* estworldpose: img [n][2] double (1-based pixels), world [n][3] double,
 * K 3x3 -> T 4x4 camera pose in world (rigidtform3d.A), inliers[n] (0/1),
 * *n_inliers.  frame_key is mixed into the Philox key.  Returns
 * VO_ERR_TOO_FEW_POINTS (n < 4) or VO_ERR_NO_CONSENSUS like MATLAB throws. */
int vo_estworldpose(vo_ctx* ctx, const double* img, const double* world, int n,
                    const double K[9], const vo_ransac_params* params, uint32_t frame_key,
                    double T[16], uint8_t* inliers, int* n_inliers);

/* new-landmark filter (VO.m:145-158) + CreateLandmarksFromFeatures.
 * l_pos/r_pos [S][2] current stereo-matched locations; old_l/old_r [K][2]
 * remaining_old_features locations; pose 4x4 world pose.  Appends rows to
 * out[capacity][3]; *rows_out = rows appended (max(2, last kept odd index),
 * zero rows kept exactly as the reference does). */
int vo_landmarks(vo_ctx* ctx, const float* l_pos, const float* r_pos, int S,
                 const float* old_l, const float* old_r, int K,
                 const double pose[16], double* out, int capacity, int* rows_out);

/* ---- fused per-frame step (the VO.m loop body) ----------------------- */
typedef struct {
    int32_t status;          /* VO_OK, or VO_ERR_* for this frame (pose held) */
    int32_t n_left, n_right; /* detected keypoints */
    int32_t n_stereo;        /* stereo matches S (VO.m:87) */
    int32_t n_tracked;       /* K after find_remaining_points (0 on frame 1) */
    int32_t n_inliers;       /* MSAC inliers */
    int32_t n_landmarks;     /* landmark rows appended this frame */
    int32_t flags;           /* VO_FLAG_* capacity flags of this frame's two images */
    double  rel_pose[16];    /* rel_pose.A (identity on frame 1) */
    double  pose[16];        /* world pose after this frame (pose.A) */
} vo_step_out;

/* Process one stereo frame.  Keeps `features` (stereo subset) on device for
 * the next call.  Landmarks accumulate inside the context (vo_get_landmarks). */
int vo_step(vo_ctx* ctx, const uint8_t* left, const uint8_t* right, int ld, vo_step_out* out);

/* Process B consecutive frames (host buffers, B*rows*ld bytes each).  The
 * per-frame work is batched across frames on the GPU; only the 4x4 pose
 * chain is sequential (host).  Equivalent to B calls of vo_step. */
int vo_step_batch(vo_ctx* ctx, const uint8_t* lefts, const uint8_t* rights, int ld, int B,
                  vo_step_out* outs);
/* Same with a storage-order flag: col_major = 1 takes B column-major (MATLAB) frames, frame n
 * at lefts + n * ld * cols, pixel (r, c) at [c * ld + r]. */
int vo_step_batch_ex(vo_ctx* ctx, const uint8_t* lefts, const uint8_t* rights, int ld, int col_major, int B,
                     vo_step_out* outs);
/* Same, inputs already in device memory (tightly packed rows*cols each). */
int vo_step_batch_dev(vo_ctx* ctx, const uint8_t* d_lefts, const uint8_t* d_rights, int B,
                      vo_step_out* outs);

/* Pipelined form of vo_step_batch_dev (same results, bit for bit).  submit enqueues the
 * device half of B frames and returns; collect waits for the oldest submitted batch and
 * runs the host half (pose chain, landmark append), writing its B outputs.  Consecutive
 * batches alternate two buffer sets, so batch n+1's SIFT overlaps batch n's tracking /
 * MSAC / landmark kernels and the host work of collect(n); batch n+2's SIFT waits for batch
 * n's geometry on the device, not for collect(n).  At most VO_STEP_DEPTH (3) batches may be
 * pending (submit(n+3) needs collect(n) first); other calls on the context are refused
 * while any is pending.  Inputs of a submit made while another batch is pending must be
 * ready on the device at the call (the first submit is ordered after vo_stream()). */
int vo_step_submit_dev(vo_ctx* ctx, const uint8_t* d_lefts, const uint8_t* d_rights, int B);
int vo_step_collect(vo_ctx* ctx, vo_step_out* outs, int capacity, int* n);
int vo_steps_pending(const vo_ctx* ctx);

/* Visualisation data of frame `frame` of the most recently collected batch (valid until
 * that buffer set is reused, i.e. the next-but-one submit; VO_ERR_STATE once that batch is
 * submitted, so a driver that visualises keeps at most two batches pending): the tracked points'
 * previous-frame left positions, current left image points and triangulated world points
 * (remaining_old_features.l_pos / .pos of VO.m:106-116), and every current left detection
 * (l_pos, VO.m:79).  Any output pointer may be NULL. */
int vo_fetch_tracks(vo_ctx* ctx, int frame, float* old_l, float* cur_l, double* world, float* det, int capacity,
                    int* n_tracked, int* n_det);

/* Landmarks accumulated so far ([rows][3] double, world frame). */
int vo_get_landmarks(vo_ctx* ctx, double* out, int capacity, int* rows);

/* Sharded sequences: CreateLandmarksFromFeatures.m:17 transforms the
 * new points by the world pose, which a rank that starts mid-sequence does not know until
 * the relative poses of every earlier rank are gathered and chained.  With
 * vo_set_landmark_frame(ctx, 1) the context keeps each appended row in the CAMERA frame
 * instead: X [rows][3] float (the triangulated point, as CreateLandmarksFromFeatures.m:7
 * returns it) and keep[rows] (0 = one of the reference's zero rows, :2).  After the chain,
 * vo_landmarks_to_world applies :17 with the frame's world pose; the result equals the
 * world-frame rows a single-process run appends, bit for bit.  Mode 0 (default) = world rows
 * (vo_get_landmarks).  Changing the mode clears the accumulated rows.  Camera-frame rows stay
 * in device memory; vo_get_landmark_rows copies them to the host. */
int vo_set_landmark_frame(vo_ctx* ctx, int camera);
int vo_get_landmark_rows(vo_ctx* ctx, float* X, uint8_t* keep, int capacity, int* rows);
/* CreateLandmarksFromFeatures.m:17 on the device for the context's own camera-frame rows:
 * poses[f] (n_frames x 16 row-major double) is the chained world pose of the f-th frame the
 * context collected since vo_reset / vo_set_landmark_frame (n_frames must equal that count;
 * frames without rows, e.g. a shard's halo frame, still take a slot).  Writes the world rows
 * as float32 x, y, z to DEVICE memory d_out [capacity][3] -- the values are single-rounded,
 * so float32 holds exactly the doubles vo_landmarks_to_world returns; keep = 0 rows are the
 * reference's zero rows.  *rows = row count (d_out NULL: count only).  Synchronises the
 * context's stream before returning, so d_out is ready for any other stream (RCCL). */
int vo_landmarks_world_dev(vo_ctx* ctx, const double* poses, int n_frames, float* d_out, long capacity, long* rows);
/* Host-only, stateless: out[i] = keep[i] ? single(pose * [X[i]; 1]) : 0 (row-major 4x4 pose). */
int vo_landmarks_to_world(const double pose[16], const float* X, const uint8_t* keep, int n, double* out);
/* The same for a whole gathered sequence: frame f's rows_per_frame[f] consecutive rows with
 * poses[f] (n_frames x 16 row-major); sum(rows_per_frame) must equal n_rows. */
int vo_landmarks_to_world_frames(const double* poses, const int32_t* rows_per_frame, int n_frames, const float* X,
                                 const uint8_t* keep, long n_rows, double* out);
/* Host-only: the VO.m:130 world-pose chain over gathered relative poses (n x 16 row-major),
 * pose = pose * rel[f] for frames whose status is VO_OK (status NULL: every frame), the pose
 * after frame f into out[f]; pose0 NULL = identity.  Same arithmetic as vo_step_collect. */
int vo_chain_poses(const double* rel, const int32_t* status, int n, const double* pose0, double* out);
/* Reset loop state (features, pose, landmarks). */
int vo_reset(vo_ctx* ctx);
/* Global index of the next frame (the MSAC Philox key of frame i is
 * seed, frame i); a rank that starts a sequence shard at frame k sets k here. */
int vo_set_frame_index(vo_ctx* ctx, long frame_index);

/* ---- benchmark workload: SIFT + stereo match on B independent pairs ---- */
typedef struct {
    int32_t n_left, n_right, n_stereo, flags;   /* flags: VO_FLAG_* */
} vo_pair_stats;

/* Device buffers: d_lefts/d_rights are B tightly packed rows*cols images.
 * Stream-ordered on the context's stream; stats (host) are written after the
 * call completes (the call synchronises only when stats != NULL). */
int vo_sift_match_batch_dev(vo_ctx* ctx, const uint8_t* d_lefts, const uint8_t* d_rights, int B,
                            vo_pair_stats* stats);

/* Device-side results of the last batched call, for parity tests:
 * keypoints and descriptors of image i (2*frame + side) and stereo pairs of
 * a frame.  Host output buffers. */
int vo_fetch_keypoints(vo_ctx* ctx, int image, vo_keypoint* kps, uint8_t* desc, int capacity, int* n);
int vo_fetch_stereo_pairs(vo_ctx* ctx, int frame, uint32_t* pairs, int capacity, int* n);
/* Extremum candidates of image i in the last batched call (uncapped: above 4 x max_keypoints
 * the list was truncated, VO_FLAG_CANDIDATES) and how many passed refinement (contrast, edge
 * and the outer-level extremum test) -- the counts the feature kernels' byte model prices. */
int vo_fetch_candidate_counts(vo_ctx* ctx, int image, int* n_cand, int* n_accepted);
/* Gaussian scale-space level G(octave, level) of image i from the last batched
 * call (rows x cols floats, tightly packed; out == NULL only reports the size).
 * Diagnostic: the scale space has no MATLAB counterpart (detectSIFTFeatures
 * keeps it internal, VO.m:79-80); parity tests compare it with the oracle. */
int vo_fetch_gaussian(vo_ctx* ctx, int image, int octave, int level, float* out, int capacity, int* rows, int* cols);

/* HIP stream the context launches on (hipStream_t as void*), and per-kernel
 * timing over the last call (for bench.py's roofline; ms). */
void* vo_stream(vo_ctx* ctx);
int vo_set_profiling(vo_ctx* ctx, int enable);

/* Batch calls run SIFT in two phases on two internal streams forked from
 * vo_stream(): the scale space (bandwidth-bound) and the feature stages +
 * stereo matching (latency-bound).  vo_set_concurrency(n) additionally splits a
 * batch into n parts (1..4, default 1) so the features of part k overlap the
 * scale space of part k+1.  vo_sift_match_batch_dev without stats is
 * asynchronous: consecutive calls alternate between two buffer sets, so the
 * scale space of call N+1 overlaps the feature stages of call N; inputs are
 * read after earlier work on vo_stream() and must stay valid until the call
 * completes (vo_fetch_* / any synchronising call wait for it).  Results are
 * identical for any n and any call pattern. */
int vo_set_concurrency(vo_ctx* ctx, int n_streams);
int vo_kernel_times(vo_ctx* ctx, const char** names, double* ms, int* calls, int capacity, int* n);

#ifdef __cplusplus
}
#endif
#endif /* VO_H */
