/*
 * oracle.h — CPU restatement of the reference's per-frame hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so.  The product path
 * (libvo.so) never links, loads or calls anything under oracle/.
 *
 * PARITY STATUS: "parity unpinned" against MATLAB.  The reference's hot path
 * lives in closed MathWorks toolboxes: no MATLAB, no golden
 * vectors, no images of KITTI-00 in the reference.  This oracle restates
 *   VO.m:64-232 (loop body), VO.m:280-334 (find_remaining_points),
 *   CreateLandmarksFromFeatures.m:1-21,
 * plus a written spec of each toolbox call's documented
 * behaviour (OpenCV-4.x-style SIFT, matchFeatures SSD+ratio, DLT
 * triangulation, P3P+MSAC).  It is pinned by known-answer tests
 * (tests/test_oracle_kat.py) and by its own committed golden fixtures
 * (tests/golden/), which the GPU path must reproduce bit for bit.
 */
#ifndef VO_ORACLE_H
#define VO_ORACLE_H

#include <stdint.h>
#include "vo.h"

#ifdef __cplusplus
extern "C" {
#endif

/* SIFT detect + describe (VO.m:79-84). Returns number of keypoints (may be >
 * capacity; only capacity written), or <0 on error. */
int oracle_sift(const uint8_t* img, int rows, int cols, int ld, const vo_sift_params* p,
                vo_keypoint* kps, uint8_t* desc, int capacity);

/* Intermediate access for KATs: Gaussian blur of a float image with the
 * spec kernel for sigma (reflect-101), and the spec kernel itself. */
int oracle_gauss_kernel(double sigma, float* k, int cap);  /* returns radius; k[0..radius] */
void oracle_blur(const float* src, float* dst, int rows, int cols, const float* k, int radius);
void oracle_upsample(const uint8_t* img, int rows, int cols, int ld, float* out);
int oracle_num_octaves(int rows, int cols, int upsample);

/* Build the whole pyramid: gauss[o][0..L+2], dog[o][0..L+1] concatenated in
 * the product's arena layout; for KATs. Returns floats
 * written or required size if out==NULL. */
long oracle_pyramid(const uint8_t* img, int rows, int cols, int ld, const vo_sift_params* p, float* out);

/* matchFeatures (VO.m:87 ...). pairs 1-based. returns n_pairs (may exceed cap). */
int oracle_match(const uint8_t* F1, int n1, const uint8_t* F2, int n2, const vo_match_params* p,
                 uint32_t* pairs, int capacity);
/* matchFeatures on general single features (libvo vo_match_f32 for non-u8-valued rows) */
int oracle_match_f32(const float* F1, int n1, int ld1, const float* F2, int n2, int ld2, int col_major,
                     const vo_match_params* p, uint32_t* pairs, int capacity);

/* find_remaining_points (VO.m:280-334). idx_out[K][3] 1-based. returns K. */
int oracle_track(const uint8_t* old_l, const uint8_t* old_r, int n_old,
                 const uint8_t* cur_l, int n_cl, const uint8_t* cur_r, int n_cr,
                 const vo_match_params* p, uint32_t* idx_out, int capacity);

/* triangulate (VO.m:113-116). */
void oracle_triangulate(const float* x1, const float* x2, int n, const double P1[12],
                        const double P2[12], double* X);

/* P3P on 3 points: bearing-free form using pixel coords + K; returns number
 * of solutions (<=4) written to Rs[4][9], ts[4][3] (X_cam = R X_world + t). */
int oracle_p3p(const double img[3][2], const double world[3][3], const double K[9],
               double Rs[4][9], double ts[4][3]);

/* estworldpose (VO.m:123-127). returns VO_OK / VO_ERR_*. */
int oracle_estworldpose(const double* img, const double* world, int n, const double K[9],
                        const vo_ransac_params* p, uint32_t frame_key, double T[16],
                        uint8_t* inliers, int* n_inliers);

/* landmarks (VO.m:145-160 + CreateLandmarksFromFeatures.m). returns rows. */
int oracle_landmarks(const float* l_pos, const float* r_pos, int S, const float* old_l,
                     const float* old_r, int K, const double P1[12], const double P2[12],
                     const double pose[16], double* out, int capacity);

/* The same split in two (sharded sequences): camera-frame rows X[rows][3] + keep[rows]
 * (CreateLandmarksFromFeatures.m:1-16), then the world transform (:17). */
int oracle_landmark_rows(const float* l_pos, const float* r_pos, int S, const float* old_l,
                         const float* old_r, int K, const double P1[12], const double P2[12],
                         float* X, uint8_t* keep, int capacity);
void oracle_landmarks_to_world(const double pose[16], const float* X, const uint8_t* keep, int n, double* out);

/* Whole loop over a sequence (VO.m:64-232): frames [F][rows*cols] u8 tightly
 * packed.  outs[F]; landmarks appended to lm_out (capacity rows). Frame f uses
 * MSAC key key0 + f (key0 = global index of frame 0).  Returns landmark rows.
 * With lm_cam_X/lm_cam_keep non-NULL the rows are appended there in the camera frame
 * instead (lm_out unused). */
long oracle_run_sequence(const uint8_t* lefts, const uint8_t* rights, int F, int rows, int cols,
                         const vo_calib* calib, const vo_sift_params* sp, const vo_match_params* mp,
                         const vo_ransac_params* rp, vo_step_out* outs, double* lm_out, long lm_cap,
                         uint32_t key0, float* lm_cam_X, uint8_t* lm_cam_keep);

/* spec primitive evaluation for KATs (spec_eval.c) */
void oracle_spec_eval(int fn, const double* in, double* out, int n);
void oracle_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t* out);
int oracle_gauss_radius(double sigma);

/* SIFT + stereo match of one pair (bench workload, configs[1]). */
int oracle_sift_match_pair(const uint8_t* left, const uint8_t* right, int rows, int cols,
                           const vo_sift_params* sp, const vo_match_params* mp,
                           int* n_left, int* n_right);

#ifdef __cplusplus
}
#endif
#endif
