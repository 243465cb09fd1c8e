// vo_geom.h — device buffers and launchers for the tracking + geometry part of
// the per-frame path: find_remaining_points (VO.m:280-334) as index
// composition over match jobs, DLT triangulation (VO.m:113-116), P3P + MSAC
// (VO.m:123-127), and the landmark filter / CreateLandmarksFromFeatures
// (VO.m:145-160).  All batched over the frames of a call.
#pragma once
#include "vo_internal.h"

namespace vo {

// index lists per frame (each [kp_cap] ints), see geom.hip for the sequence
enum TrackList {
    TL_OL1, TL_OR1, TL_CL, TL_OL2, TL_OR2, TL_CR, TL_CL2, TL_CR2, TL_OLF, TL_ORF, TL_CLF, TL_CRF, TL_COUNT
};

struct MsacHyp {
    double R[9];
    double t[3];
    double score;
    int valid;
    int n_in;
};

struct FrameGeom {
    int status;
    int n_inliers;
    int best;
    int n_tracked;
    double T[16];          // rel_pose (camera pose of cur in prev frame)
};

struct GeomBuffers {
    int max_frames = 0, kp_cap = 0, n_hyp = 0;
    int* lists = nullptr;        // [max_frames][TL_COUNT][kp_cap]
    int* list_n = nullptr;       // [max_frames][4]  n after lm, rm, cm, last
    int* step_i = nullptr;       // [4][max_frames][kp_cap] match outputs
    int* step_j = nullptr;
    int* step_n = nullptr;       // [4][max_frames]
    double* world = nullptr;     // [max_frames][kp_cap][3]
    double* imgpt = nullptr;     // [max_frames][kp_cap][2]
    float* oldpos = nullptr;     // [max_frames][kp_cap][4]  old left xy, old right xy
    uint8_t* inliers = nullptr;  // [max_frames][kp_cap]
    MsacHyp* hyp = nullptr;      // [max_frames][n_hyp]
    FrameGeom* fg = nullptr;     // [max_frames]
    // landmarks
    float* spos = nullptr;       // [max_frames][kp_cap][4] stereo subset positions (lx, ly, rx, ry)
    int* s_n = nullptr;          // [max_frames]
    int* lm_new = nullptr;       // [max_frames][kp_cap]  compacted indices of new stereo matches
    int* lm_M = nullptr;         // [max_frames]
    float* lm_X = nullptr;       // [max_frames][kp_cap][3] camera-frame points of odd rows
    uint8_t* lm_keep = nullptr;  // [max_frames][kp_cap]
    int* lm_rows = nullptr;      // [max_frames]
    // the batch's landmark rows packed in frame order (one D2H copy per batch): row r of frame f
    // at sum_{g<f} min(lm_rows[g], kp_cap) + r
};

hipError_t geom_alloc(GeomBuffers& g, int max_frames, int kp_cap, int n_hyp);
void geom_free(GeomBuffers& g);

// Fill the 4 x max_frames tracking match jobs starting at jobs[first].
// Frame f: cur images 2f (left) / 2f+1 (right); prev frame = f-1, frame 0's
// prev is the carried frame (image slots 2*max_frames, 2*max_frames+1; pair
// slot max_frames).
void geom_fill_track_jobs(const GeomBuffers& g, MatchJob* jobs, int max_frames, int first, const SiftBuffers& sb,
                          int* pair_i, int* pair_j, int* pair_n, int kp_cap);

struct StepArgs {
    const SiftBuffers* sb;
    const int* pair_i; const int* pair_j; const int* pair_n;   // stereo pairs per pair slot
    int max_frames, B, kp_cap;
    int first_has_prev;            // frame 0 of this call has a previous frame (carry)
    long frame_index0;             // global index of frame 0 (Philox key)
    vo_calib calib;
    vo_ransac_params rp;
};

// Enqueue tracking (4 matches + compositions), triangulation, MSAC and the
// landmark kernels for frames [0, B).  match jobs at d_jobs + first.
void geom_enqueue(GeomBuffers& g, const MatchBuffers& mb, const MatchJob* d_track_jobs, const StepArgs& a,
                  const vo_match_params& mp, hipStream_t s);
// tracking only (4 matches + compositions); lists/list_n valid afterwards.
void track_enqueue(GeomBuffers& g, const MatchBuffers& mb, const MatchJob* d_track_jobs, const StepArgs& a,
                   const vo_match_params& mp, hipStream_t s);
static inline int* track_list(const GeomBuffers& g, int f, int l) { return g.lists + ((size_t)f * TL_COUNT + l) * g.kp_cap; }

// Pack frames [0, B)'s landmark rows contiguously into pX [B * kp_cap][3] / pkeep [B * kp_cap]
// (the submitting batch's own buffers: they outlive the buffer set's reuse by the batch after next).
void lm_pack_launch(GeomBuffers& g, int B, float* pX, uint8_t* pkeep, hipStream_t s);

// CreateLandmarksFromFeatures.m:17 on the device for a run of frames: frame f's rows
// [off[f], off[f+1]) of the camera-frame store (X [rows][3], keep [rows]) go to the world with
// poses[f] (row-major 4x4, f64), rounded through single into out [rows][3] (zero rows for keep 0).
void lm_world_launch(const double* poses, const long long* off, int n_frames, const float* X, const uint8_t* keep,
                     float* out, hipStream_t s);

// Standalone launchers used by the single-call ABI functions (frame slot 0).
// pos: [n][4] (x1, y1, x2, y2) device floats.
void triangulate_launch(const float* pos, int n, const vo_calib& c, double* X, hipStream_t s);
void estworldpose_launch(GeomBuffers& g, const double* img, const double* world, const int* n, const double K[9],
                         const vo_ransac_params& rp, uint32_t frame_key, hipStream_t s);
// landmark filter + CreateLandmarksFromFeatures on g.spos/g.s_n (frame 0) vs
// g.oldpos with *kn old rows.
void landmarks_launch(GeomBuffers& g, const int* kn, const vo_calib& c, hipStream_t s);

}  // namespace vo
