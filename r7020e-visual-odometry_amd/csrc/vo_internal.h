// vo_internal.h — device data layout and kernel launch interfaces of libvo.
// Layout rationale: DESIGN.md §4.  All kernels are hand-written HIP for gfx950
// (wave64), compiled with -ffp-contract=off so every float operation is the
// IEEE basic op the spec (include/vo_spec.h) names.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <vector>
#include <string>
#include "vo.h"
#include "vo_spec.h"

#define VO_WAVE 64

namespace vo {

// ---------------------------------------------------------------------------
// Per-kernel HIP-event timing (vo_set_profiling).  When enabled every launch
// made through VO_LAUNCH is bracketed by two events on its stream; the
// durations are summed per kernel name after the call synchronises.
// ---------------------------------------------------------------------------
struct Profiler {
    bool on = false;
    std::vector<hipEvent_t> pool;
    int used = 0;
    std::vector<std::pair<const char*, int>> marks;   // (kernel name, start event index)
    std::vector<std::string> names;
    std::vector<double> ms;
    std::vector<int> calls;
    void begin(const char* name, hipStream_t s);
    void end(hipStream_t s);
    void collect();      // after the stream has synchronised
    void reset_totals();
    ~Profiler();
};
extern Profiler* g_prof;

#define VO_LAUNCH_NAMED(name, kernel, grid, block, shmem, stream, ...)                     \
    do {                                                                                   \
        if (::vo::g_prof && ::vo::g_prof->on) ::vo::g_prof->begin(name, stream);           \
        hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);               \
        if (::vo::g_prof && ::vo::g_prof->on) ::vo::g_prof->end(stream);                   \
    } while (0)
#define VO_LAUNCH(kernel, grid, block, shmem, stream, ...) \
    VO_LAUNCH_NAMED(#kernel, kernel, grid, block, shmem, stream, __VA_ARGS__)

// ---------------------------------------------------------------------------
// Scale-space arena, image-major: the whole pyramid of one image is contiguous,
// G(o,i,img) = arena + img*istride + g_off[o][i], so any contiguous range of
// images is a pointer shift (sub-batches run concurrently on separate streams).
// DoG planes are not stored: D(o,i) = G(o,i+1) - G(o,i) where it is consumed.
// Rows are padded to a multiple of 256 floats (1 KiB): every row starts on a
// cache-line boundary and spans a whole number of the level blur's 256-column
// strips, so lanes past the last column store into padding instead of branching.
// ---------------------------------------------------------------------------
struct OctGeom {
    int rows, cols, pitch;
    int dmax;                           // descriptor window radius cap, (int)sqrt(cols^2 + rows^2)
    size_t plane;                       // rows * pitch (floats)
    size_t g_off[VO_SIFT_MAX_LAYERS];   // L+3 Gaussian levels
};

struct Pyramid {
    int n_oct, L, n_img;
    OctGeom oct[VO_SIFT_MAX_OCTAVES];
    float kern[VO_SIFT_MAX_LAYERS][VO_SIFT_MAX_RADIUS + 1];  // level blur kernels (level 0 = base)
    int krad[VO_SIFT_MAX_LAYERS];
    size_t istride;                      // floats per image (all octaves and levels)
    size_t total;                        // floats in the arena
    size_t tmp_plane;                    // floats per image of the horizontal-pass scratch
    // extrema word layout: per (octave, layer, interior row) the words of 64
    // absolute columns [64k, 64k+64); bits of border columns are 0
    int wbase[VO_SIFT_MAX_OCTAVES * 4 + 1];   // prefix over (o, layer-1) blocks; size n_oct*L+1
    int wrow[VO_SIFT_MAX_OCTAVES];            // words per row in octave o
    int n_words;                              // words per image
    // extremum-test units: (strip of 128 columns, band of VO_EXT_BAND interior rows)
    int ebase[VO_SIFT_MAX_OCTAVES + 1];       // prefix of units per octave
    int estrips[VO_SIFT_MAX_OCTAVES];         // strips per row in octave o
    int n_units;                              // units per image
    int n_seg;                                // 1024-word compaction segments per image
    int dcap;                                 // largest descriptor window radius the parameters allow
};

// Feature-stage build switch (A/B builds; the product uses the default):
//  VO_ACC_LIST   1: k_refine lists the accepted candidates and k_orient / k_expand walk the list
#ifndef VO_ACC_LIST
#define VO_ACC_LIST 1
#endif



// k_desc's per-keypoint window tables in LDS (desc_tables), u32 words: a header of DT_HDR words
// (DT_ORI .. DT_LAYER below), the row table (2 dcap + 10 entries) and the separable window
// weights (dcap + 1 floats); stride rounded to 16 B.
#define DT_HDR 12
enum { DT_ORI, DT_PX, DT_PY, DT_RADIUS, DT_COS, DT_SIN, DT_NSAMP, DT_NROWS, DT_O, DT_LAYER };
static inline __host__ __device__ int dt_rtab_off() { return DT_HDR; }
static inline __host__ __device__ int dt_wtab_off(int dcap) { return DT_HDR + 2 * dcap + 10; }
static inline __host__ __device__ int dt_stride(int dcap) { return (DT_HDR + 3 * dcap + 11 + 3) & ~3; }

#ifndef VO_EXT_BAND
#define VO_EXT_BAND 30            // interior rows per extremum-test wave (a multiple of 3)
#endif
#ifndef VO_EXT_INNER
#define VO_EXT_INNER 1            // extremum test: 1 = k_ext_inner + k_refine's outer-level check, 0 = k_ext_stream (all L+3 levels)
#endif
#ifndef VO_NPK_COMPACT
#define VO_NPK_COMPACT 1          // peak counts also as a 4-B array (koff, scanned in place) for k_scan_cands
#endif
#ifndef VO_EXT_BSTORE
#define VO_EXT_BSTORE 1           // extremum test: mask words by unconditional buffer stores (0: branchy stores)
#endif
#define VO_SEG_WORDS 1024

// Packed candidate: c | r << 12 | layer << 24 | o << 27  (c, r < 4096)
__host__ __device__ inline uint32_t pack_cand(int o, int layer, int r, int c) {
    return (uint32_t)c | ((uint32_t)r << 12) | ((uint32_t)layer << 24) | ((uint32_t)o << 27);
}

// Refined candidate with its orientation peaks (output of refine_orient).
struct CandOut {
    float xo, yo, scl, response;
    int o, layer, r, c;
    int npk, pad0, pad1, pad2;
    float ang[VO_SIFT_MAX_PEAKS + 2];
};

// Internal keypoint record used by the descriptor kernel.
struct KpInt {
    float xo, yo, scl, angle;
    int o, layer, pad0, pad1;
};

// Per-descriptor metadata for matching: exact integer sums.
struct DescMeta {
    int32_t sum;      // sum of the 128 u8 values
    float inv_norm;   // 1/sqrtf((float)sum of squares), 0 if zero
};

// Buffers of the SIFT stage for a batch of n_img images.
struct SiftBuffers {
    float* arena = nullptr;
    float* tmp = nullptr;              // horizontal-pass scratch [n_img][tmp_plane]
    unsigned long long* mask = nullptr;  // [n_img][n_words]
    uint32_t* woff = nullptr;          // [n_img][n_seg] segment counts, then exclusive offsets
    uint32_t* cand = nullptr;          // [n_img][cand_cap]
    int* n_cand = nullptr;             // [n_img]  (uncapped count)
    int* acc = nullptr;                // [n_img][cand_cap] accepted candidates' indices (k_refine, any order)
    int* n_acc = nullptr;              // [n_img]
    CandOut* cout = nullptr;           // [n_img][cand_cap]
    uint32_t* koff = nullptr;          // [n_img][cand_cap]
    int* n_kp = nullptr;               // [n_img]  (uncapped count)
    vo_keypoint* kp = nullptr;         // [n_img][kp_cap]
    KpInt* kpi = nullptr;              // [n_img][kp_cap]
    uint8_t* desc = nullptr;           // [n_img][kp_cap][128]
    DescMeta* meta = nullptr;          // [n_img][kp_cap]
    int cand_cap = 0, kp_cap = 0, n_img = 0;
};

// Image source for the first octave: image i of the batch is
// (i & 1 ? right : left) + (i >> 1) * frame_stride, row-major with ld.
struct ImageSrc {
    const uint8_t* left;
    const uint8_t* right;
    size_t frame_stride;
    int ld;
    int pad;
};

void build_pyramid_geometry(Pyramid& py, int rows, int cols, int n_img, const vo_sift_params& p);
// Parameters the SIFT kernels' fixed-point and window bounds admit (vo_create refuses others):
// sigma finite and > 0, and every orientation window small enough for k_orient's u32 column sums.
bool sift_params_supported(const vo_sift_params& p);
// View of images [img0, img0 + n) of b: every per-image array shifted (image-major layout).
SiftBuffers sift_view(const SiftBuffers& b, const Pyramid& py, int img0, int n);
hipError_t sift_alloc(SiftBuffers& b, const Pyramid& py, int kp_cap, int cand_cap);
void sift_free(SiftBuffers& b);
// Enqueue the whole detect+describe pipeline for n_img images (<= allocated).
// d_py is a device copy of py.
void sift_enqueue(const Pyramid& py, SiftBuffers& b, const ImageSrc& src, int n_img,
                  const vo_sift_params& p, hipStream_t s, const Pyramid* d_py);
// The phases of sift_enqueue: the scale space of the large octaves (base, level blurs, octave
// bases; ev_o0, if given, is recorded once octave 0 is complete); its tail (the LDS-sized octaves
// and the extremum test of octaves [ext_o_begin, n_oct)); the extremum test of an octave range;
// and the feature stages (mask compaction, refinement, orientation, descriptors).  The batched
// path runs the extremum test of octave 0 on the feature stream as soon as ev_o0 fires, beside
// the scale space of octaves 1.., and the rest at the scale space's tail (vo_api.hip).
void sift_enqueue_pyramid(const Pyramid& py, SiftBuffers& b, const ImageSrc& src, int n_img,
                          const vo_sift_params& p, hipStream_t s, const Pyramid* d_py, hipEvent_t ev_o0 = nullptr);
void sift_enqueue_pyramid_tail(const Pyramid& py, SiftBuffers& b, int n_img, const vo_sift_params& p, hipStream_t s,
                               const Pyramid* d_py, int ext_o_begin);
void sift_enqueue_extrema(const Pyramid& py, SiftBuffers& b, int n_img, const vo_sift_params& p, hipStream_t s,
                          const Pyramid* d_py, int o_begin, int o_end);
// the LDS-sized octaves o >= sift_small_octave(py) (one k_small_pyr launch; n_oct when none)
int sift_small_octave(const Pyramid& py);
void sift_enqueue_small(const Pyramid& py, SiftBuffers& b, int n_img, hipStream_t s, const Pyramid* d_py);
void sift_enqueue_features(const Pyramid& py, SiftBuffers& b, int n_img, const vo_sift_params& p, hipStream_t s,
                           const Pyramid* d_py);

// One octave's levels 1..5 + extremum test + next octave base in one pass (octave.hip).
struct OctArgs {
    float* arena;
    size_t istride;                     // floats per image
    int R, C, pitch, pad0;
    size_t goff[6];                     // this octave's G_0..G_5 plane offsets
    float* nbase;                       // next octave's G_0 plane (image 0), or nullptr
    int Rn, Cn, pitchn, pad1;
    unsigned long long* mask;
    int n_words, wr;                    // words per image, words per mask row of this octave
    int wb[3];                          // word base of layers 1..3 of this octave
    float thr;                          // extremum threshold (DoG units)
    float k[6][16];                     // taps of levels 1..5 (k[i][0..r_i])
    int n_strips, pad2;
};
#if VO_EXPERIMENTAL
// test build only (libvo_exp.so): the fused octave (octave.hip) and the eager MSAC kernels, each
// selected by vo_exp_set; the product libvo.so has neither the kernels nor a switch
bool octave_fused_ok(const Pyramid& py, int o);
void octave_fused_launch(const Pyramid& py, const Pyramid* d_py, const SiftBuffers& b, int o, int n_img, float thr,
                         hipStream_t s);
extern int g_exp_fused_octave, g_exp_msac_eager;
#endif
// hipFuncSetAttribute(MaxDynamicSharedMemorySize, 160 KB) once per (kernel, device)
void raise_lds_limit(const void* fn);

// ---------------------------------------------------------------------------
// Matching.  A match job compares F1 rows (desc[idx1[i]] for i < *n1) against
// F2 rows.  idx == nullptr means identity.  Counts are read on device.
// ---------------------------------------------------------------------------
struct MatchJob {
    const uint8_t* d1; const DescMeta* m1; const int* idx1; const int* n1;
    const uint8_t* d2; const DescMeta* m2; const int* idx2; const int* n2;
    int* out_i;      // [cap] F1 positions (0-based, position in the F1 list)
    int* out_j;      // [cap] F2 positions
    int* out_n;      // matches found
    int cap;
    int pad;
};

// Per (row, F2 chunk) top-2 in the cosine domain: best/second are the largest
// c = ((float)dot * inv|a|) * inv|b| values (SSD = 2 - 2c is non-increasing in c).
struct MatchTop2 { float best; int idx; float second; int pad; };

struct MatchBuffers {
    MatchJob* jobs = nullptr;        // device copy of the jobs [max_jobs]
    MatchTop2* partial = nullptr;    // [max_jobs][n_chunks][row_cap]
    int* res = nullptr;              // [max_jobs][row_cap] accepted F2 index per F1 row, -1 if none
    int max_jobs = 0, row_cap = 0, n_chunks = 0;
};

#ifndef VO_MATCH_CHUNK
#define VO_MATCH_CHUNK 4096          // F2 columns per task (512/1024/2048 swept before; 4096: the tracking steps' ~2.1 k
                                     // columns in one chunk, match -10 % isolated, full path +1.3 %, r06_y)
#endif

hipError_t match_alloc(MatchBuffers& b, int max_jobs, int row_cap);
// View whose job slot 0 is slot k0 of b (partial-result rows of jobs k0, k0+1, ...).
MatchBuffers match_view(const MatchBuffers& b, int k0);
void match_free(MatchBuffers& b);
// d_jobs: device array of n_jobs jobs (prepared once per context); job k uses
// partial-result slot k.
// The index composition after tracking step `step` of find_remaining_points (VO.m:287-290,
// 297-300, 305-308, 314-317, 326-333) over lists [frame][TL_COUNT][kp_cap] (vo_geom.h), applied
// by match_launch's finishing kernel to the step's compacted pairs of job f (= frame f).
struct MatchCompose {
    int* lists; int* list_n;
    const int* pair_i; const int* pair_j;    // stereo pairs per pair slot (frame f-1's, or slot M)
    int M, kp_cap, step;
    int f0;                                  // frame of job 0 (a launch split at VO_MP_MAX_JOBS jobs)
};
void match_launch(const MatchBuffers& b, const MatchJob* d_jobs, int n_jobs, const vo_match_params& p,
                  hipStream_t s, const MatchCompose* compose);
void match_launch(const MatchBuffers& b, const MatchJob* d_jobs, int n_jobs, const vo_match_params& p,
                  hipStream_t s);
void desc_meta_launch(const uint8_t* desc, DescMeta* meta, int n, hipStream_t s);
void pack_f32_desc_launch(const float* F, int n, int ld, int col_major, uint8_t* out, int* bad, hipStream_t s);
// matchFeatures on general single features (not u8-valued): normalised rows A [n1][128], F2
// normalised and transposed into BT [128][n2], res[i] = accepted F2 column of row i or -1
void match_f32_launch(const float* F1, int n1, int ld1, const float* F2, int n2, int ld2, int col_major, float* A, float* BT,
                      int* res, const vo_match_params& p, hipStream_t s);

}  // namespace vo
