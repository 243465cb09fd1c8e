// vo_api.hip — the C-ABI of libvo (include/vo.h): context, staging and the
// orchestration of the per-frame pipeline on one HIP stream.
#include "vo_internal.h"
#include "vo_geom.h"
#include <climits>
#include <cstdio>
#include <cstring>
#include <cstdarg>
#include <string>
#include <vector>
#include <deque>
#include <algorithm>

namespace vo {

Profiler* g_prof = nullptr;

void Profiler::begin(const char* name, hipStream_t s)
{
    if (used + 2 > (int)pool.size()) {
        int add = std::max(64, (int)pool.size());
        for (int i = 0; i < add; ++i) { hipEvent_t e; hipEventCreate(&e); pool.push_back(e); }
    }
    marks.push_back({name, used});
    hipEventRecord(pool[used], s);
    used += 1;
}

void Profiler::end(hipStream_t s)
{
    hipEventRecord(pool[used], s);
    used += 1;
}

void Profiler::collect()
{
    for (auto& m : marks) {
        float t = 0.0f;
        hipEventElapsedTime(&t, pool[m.second], pool[m.second + 1]);
        std::string n(m.first);
        size_t k = 0;
        for (; k < names.size(); ++k) if (names[k] == n) break;
        if (k == names.size()) { names.push_back(n); ms.push_back(0.0); calls.push_back(0); }
        ms[k] += t;
        calls[k] += 1;
    }
    marks.clear();
    used = 0;
}

void Profiler::reset_totals() { names.clear(); ms.clear(); calls.clear(); marks.clear(); used = 0; }

Profiler::~Profiler() { for (auto e : pool) hipEventDestroy(e); }

}  // namespace vo

using namespace vo;

struct vo_ctx {
    int device = 0, rows = 0, cols = 0, max_batch = 0;
    vo_sift_params sp;
    vo_match_params mp;
    vo_ransac_params rp;
    vo_calib calib;
    bool has_calib = false;
    hipStream_t stream = nullptr;
    // sub-batch concurrency: a batch's frames are split over n_sub streams that
    // fork from / join into `stream` (latency-bound SIFT stages of one part
    // overlap bandwidth-bound stages of another)
    static constexpr int MAX_SUB = 4;
    int n_sub = 1;
    hipStream_t sub[MAX_SUB] = {};                 // sub[0]: scale-space stream, sub[1]: feature stream
    hipEvent_t ev_fork = nullptr, ev_join[MAX_SUB] = {}, ev_o0[MAX_SUB] = {}, ev_small[MAX_SUB] = {};
    // Asynchronous batch pipeline (vo_sift_match_batch_dev): calls alternate between two
    // buffer sets; set 0 is the context's own buffers (sb, mb, stereo jobs, pairs), set 1
    // is `aux`.  A call's scale space waits only for the previous use of its own set, so
    // the pyramid of call N+1 overlaps the latency-bound feature stages of call N.
    // Set 1 is a full replica of set 0's per-frame state (image slots incl. the carried
    // frame, pair slots incl. the carry slot, stereo + tracking jobs, geometry buffers), so
    // the full per-frame path can also alternate sets (vo_step_submit_dev).
    struct AuxSet {
        SiftBuffers sb;
        MatchBuffers mb;
        MatchJob* d_jobs = nullptr;      // [0, M) stereo, [M, 5M) tracking (job_track layout)
        int* pair_i = nullptr; int* pair_j = nullptr; int* pair_n = nullptr;   // max_batch + 1 slots
        GeomBuffers gb;
    } aux;
    hipEvent_t ev_done[2] = {};
    hipEvent_t ev_arena[2] = {};     // set's scale-space arena read for the last time (after k_desc)
    int next_set = 0, last_set = 0;
    Pyramid py;
    Pyramid* d_py = nullptr;
    SiftBuffers sb;                  // 2*max_batch + 2 image slots (last 2 = carried frame)
    MatchBuffers mb;
    MatchJob* d_jobs = nullptr;      // job tables (see JOB_* offsets)
    int* d_pair_i = nullptr;         // stereo pairs per frame slot [slots][kp_cap]
    int* d_pair_j = nullptr;
    int* d_pair_n = nullptr;         // [slots]
    uint8_t* d_img = nullptr;        // image staging [2*max_batch][rows*cols]
    uint8_t* d_cm = nullptr;         // column-major (MATLAB) image staging, allocated on first use
    size_t cm_cap = 0;
    // vo_match staging
    uint8_t* d_fd[2] = {nullptr, nullptr};
    DescMeta* d_fm[2] = {nullptr, nullptr};
    int* d_fn = nullptr;             // [2]
    float* d_ff[2] = {nullptr, nullptr};   // vo_match_f32 staging (single descriptors as MATLAB holds them)
    // vo_match_f32 on general (non-u8-valued) features: normalised F1, transposed F2, per-row result
    // (allocated on first use)
    float* d_fa = nullptr;
    float* d_fbt = nullptr;
    int* d_fres = nullptr;
    int* d_bad = nullptr;
    int* d_mi = nullptr; int* d_mj = nullptr; int* d_mn = nullptr;
    GeomBuffers gb;
    // Pipelined full path (vo_step_submit_dev / vo_step_collect): batch n uses buffer set
    // n & 1; its geometry runs on `stream` while the later batches' SIFT runs on sub[0..1].
    // Up to VO_STEP_DEPTH batches are in flight, so each batch also owns a result slot
    // (n mod VO_STEP_DEPTH): pinned host copies of the per-frame results, its packed landmark
    // rows on the device, and the event that ends the batch (geometry, carry into the other
    // set, result copies).  A slot outlives its buffer set's reuse by batch n+2.
    struct StepHost {
        FrameGeom* fg = nullptr; int* nkp = nullptr; int* ncand = nullptr; int* np = nullptr; int* rows = nullptr;
        float* pX = nullptr; uint8_t* pkeep = nullptr;     // the batch's packed landmark rows (pinned)
        float* d_pX = nullptr; uint8_t* d_pkeep = nullptr; // ... and on the device (k_lm_pack)
        hipEvent_t ev = nullptr;                           // end of the batch on `stream`
    };
    StepHost sh[VO_STEP_DEPTH];
    hipStream_t copy_stream = nullptr;
    struct Pending { int set, slot, B; bool first_tracked; };
    std::deque<Pending> pending;
    int next_step_set = 0, next_slot = 0;
    std::vector<void*> lm_retired;                   // landmark stores replaced by a larger one (freed at reset)
    int last_step_set = -1, last_step_B = 0;          // the most recently collected batch (vo_fetch_tracks)
    std::string err;
    Profiler prof;
    int last_B = 0;
    // loop state (vo_step)
    long frame_index = 0;
    bool have_features = false;
    double pose[16];
    std::vector<double> landmarks;
    // camera-frame landmark rows (vo_set_landmark_frame(ctx, 1)): sharded sequences.  The rows
    // stay in device memory (appended by collect from the packed batch rows, a device-to-device
    // copy on `stream`), so the world transform after the gathered chain runs on the device and
    // only the world rows move (vo_landmarks_world_dev)
    int lm_camera = 0;
    float* d_lmX = nullptr;                       // [lm_cap][3]
    uint8_t* d_lmkeep = nullptr;                  // [lm_cap]
    size_t lm_cap = 0, lm_n = 0;
    std::vector<long long> lm_frame_off{0};       // row offset of every collected frame (+ end)
    double* d_lmw_pose = nullptr;                 // vo_landmarks_world_dev staging: poses, offsets
    long long* d_lmw_off = nullptr;
    int lmw_cap = 0;
};

static std::string g_create_err;

static int fail(vo_ctx* c, int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (c) c->err = buf; else g_create_err = buf;
    return code;
}

#define HIPC(c, x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return fail(c, VO_ERR_HIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); } while (0)

static const double I4[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};

extern "C" {

void vo_default_sift_params(vo_sift_params* p)
{
    p->n_octave_layers = 3; p->sigma = 1.6f; p->contrast_threshold = 0.04f; p->edge_threshold = 10.0f;
    p->upsample = 1; p->max_keypoints = 16384;
}
void vo_default_match_params(vo_match_params* p) { p->match_threshold = 1.0f; p->max_ratio = 0.6f; }
void vo_default_ransac_params(vo_ransac_params* p)
{
    p->max_num_trials = 1000; p->confidence = 99.0; p->max_reprojection_error = 1.0; p->seed = 0x5EED;
}

const char* vo_last_error(const vo_ctx* c) { return c ? c->err.c_str() : g_create_err.c_str(); }

void* vo_stream(vo_ctx* c) { return c ? (void*)c->stream : nullptr; }

// job table layout: [0, B) stereo; [B, B + 4*B) tracking steps; last: vo_match
static int job_stereo(const vo_ctx*, int f) { return f; }
static int job_track(const vo_ctx* c, int step, int f) { return c->max_batch + step * c->max_batch + f; }
static int job_single(const vo_ctx* c) { return 5 * c->max_batch; }

static void destroy_streams(vo_ctx* c)
{
    for (int k = 0; k < vo_ctx::MAX_SUB; ++k) {
        if (c->sub[k]) hipStreamDestroy(c->sub[k]);
        if (c->ev_join[k]) hipEventDestroy(c->ev_join[k]);
        if (c->ev_o0[k]) hipEventDestroy(c->ev_o0[k]);
        if (c->ev_small[k]) hipEventDestroy(c->ev_small[k]);
        c->sub[k] = nullptr; c->ev_join[k] = nullptr; c->ev_o0[k] = nullptr; c->ev_small[k] = nullptr;
    }
    if (c->ev_fork) hipEventDestroy(c->ev_fork);
    c->ev_fork = nullptr;
    for (int k = 0; k < 2; ++k) {
        if (c->ev_done[k]) hipEventDestroy(c->ev_done[k]);
        if (c->ev_arena[k]) hipEventDestroy(c->ev_arena[k]);
        c->ev_arena[k] = nullptr;
        c->ev_done[k] = nullptr;
    }
    for (int k = 0; k < VO_STEP_DEPTH; ++k) {
        if (c->sh[k].ev) hipEventDestroy(c->sh[k].ev);
        c->sh[k].ev = nullptr;
    }
    if (c->copy_stream) hipStreamDestroy(c->copy_stream);
    c->copy_stream = nullptr;
}

static void destroy_buffers(vo_ctx* c)
{
    sift_free(c->sb);
    match_free(c->mb);
    sift_free(c->aux.sb);
    match_free(c->aux.mb);
    hipFree(c->aux.d_jobs); hipFree(c->aux.pair_i); hipFree(c->aux.pair_j); hipFree(c->aux.pair_n);
    geom_free(c->aux.gb);
    for (int k = 0; k < VO_STEP_DEPTH; ++k) {
        hipHostFree(c->sh[k].fg); hipHostFree(c->sh[k].nkp); hipHostFree(c->sh[k].ncand); hipHostFree(c->sh[k].np); hipHostFree(c->sh[k].rows);
        hipHostFree(c->sh[k].pX); hipHostFree(c->sh[k].pkeep);
        hipFree(c->sh[k].d_pX); hipFree(c->sh[k].d_pkeep);
        const hipEvent_t ev = c->sh[k].ev;               // owned by destroy_streams
        c->sh[k] = vo_ctx::StepHost();
        c->sh[k].ev = ev;
    }
    for (void* p : c->lm_retired) hipFree(p);
    c->lm_retired.clear();
    geom_free(c->gb);
    hipFree(c->d_py); hipFree(c->d_jobs); hipFree(c->d_pair_i); hipFree(c->d_pair_j); hipFree(c->d_pair_n);
    hipFree(c->d_img); hipFree(c->d_cm); hipFree(c->d_fd[0]); hipFree(c->d_fd[1]); hipFree(c->d_fm[0]); hipFree(c->d_fm[1]);
    hipFree(c->d_ff[0]); hipFree(c->d_ff[1]); hipFree(c->d_bad);
    hipFree(c->d_fa); hipFree(c->d_fbt); hipFree(c->d_fres);
    hipFree(c->d_fn); hipFree(c->d_mi); hipFree(c->d_mj); hipFree(c->d_mn);
    hipFree(c->d_lmX); hipFree(c->d_lmkeep); hipFree(c->d_lmw_pose); hipFree(c->d_lmw_off);
    c->d_lmX = nullptr; c->d_lmkeep = nullptr; c->d_lmw_pose = nullptr; c->d_lmw_off = nullptr;
    c->lm_cap = 0; c->lmw_cap = 0;
}

vo_ctx* vo_create(int device, int rows, int cols, int max_batch, const vo_calib* calib, const vo_sift_params* sift,
                  const vo_match_params* match, const vo_ransac_params* ransac)
{
    if (rows < 16 || cols < 16 || rows > 2048 || cols > 2048 || max_batch < 1 || max_batch > VO_MAX_BATCH) {
        fail(nullptr, VO_ERR_ARG, "vo_create: bad size rows=%d cols=%d max_batch=%d", rows, cols, max_batch);
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) { fail(nullptr, VO_ERR_HIP, "hipSetDevice(%d) failed", device); return nullptr; }
    vo_ctx* c = new vo_ctx();
    c->device = device; c->rows = rows; c->cols = cols; c->max_batch = max_batch;
    if (sift) c->sp = *sift; else vo_default_sift_params(&c->sp);
    if (match) c->mp = *match; else vo_default_match_params(&c->mp);
    if (ransac) c->rp = *ransac; else vo_default_ransac_params(&c->rp);
    if (calib) { c->calib = *calib; c->has_calib = true; }
    memcpy(c->pose, I4, sizeof(I4));
    if (c->sp.n_octave_layers < 1 || c->sp.n_octave_layers > 5 || c->sp.max_keypoints < 16 ||
        !sift_params_supported(c->sp)) {
        fail(nullptr, VO_ERR_ARG, "vo_create: bad sift params");
        delete c;
        return nullptr;
    }
    auto bail = [&](const char* what, hipError_t e) -> vo_ctx* {
        fail(nullptr, VO_ERR_HIP, "vo_create: %s: %s", what, hipGetErrorString(e));
        destroy_buffers(c);
        destroy_streams(c);
        if (c->stream) hipStreamDestroy(c->stream);
        delete c;
        return nullptr;
    };
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return bail("stream", e);
    for (int k = 0; k < vo_ctx::MAX_SUB; ++k) {
        // every stream at the default priority: the forked SIFT streams must not rank below the
        // geometry / copy streams of the pipelined loop body (at the lowest priority the full
        // per-frame path dropped from 7.3 k to 5.4 k stereo frames/s), and the scale-space stream
        // at the highest priority measured within noise.  No CU masks: with masks that bind
        // (contiguous CU ranges), every split of the CUs between the two streams was 9-38 %
        // slower -- both streams are bound per CU and need the whole chip
        e = hipStreamCreateWithFlags(&c->sub[k], hipStreamNonBlocking);
        if (e != hipSuccess) return bail("stream", e);
        if ((e = hipEventCreateWithFlags(&c->ev_join[k], hipEventDisableTiming)) != hipSuccess) return bail("event", e);
        if ((e = hipEventCreateWithFlags(&c->ev_o0[k], hipEventDisableTiming)) != hipSuccess) return bail("event", e);
        if ((e = hipEventCreateWithFlags(&c->ev_small[k], hipEventDisableTiming)) != hipSuccess) return bail("event", e);
    }
    if ((e = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming)) != hipSuccess) return bail("event", e);
    for (int k = 0; k < 2; ++k) {
        if ((e = hipEventCreateWithFlags(&c->ev_done[k], hipEventDisableTiming)) != hipSuccess) return bail("event", e);
        if ((e = hipEventCreateWithFlags(&c->ev_arena[k], hipEventDisableTiming)) != hipSuccess) return bail("event", e);
    }
    if ((e = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking)) != hipSuccess) return bail("stream", e);
    const int n_slots = 2 * max_batch + 2;
    const int kp_cap = c->sp.max_keypoints;
    build_pyramid_geometry(c->py, rows, cols, n_slots, c->sp);
    if ((e = hipMalloc((void**)&c->d_py, sizeof(Pyramid))) != hipSuccess) return bail("pyramid", e);
    if ((e = hipMemcpy(c->d_py, &c->py, sizeof(Pyramid), hipMemcpyHostToDevice)) != hipSuccess) return bail("pyramid copy", e);
    if ((e = sift_alloc(c->sb, c->py, kp_cap, 4 * kp_cap)) != hipSuccess) return bail("sift buffers", e);
    const int n_jobs = 5 * max_batch + 1;
    if ((e = match_alloc(c->mb, n_jobs, kp_cap)) != hipSuccess) return bail("match buffers", e);
    if ((e = hipMalloc((void**)&c->d_jobs, sizeof(MatchJob) * n_jobs)) != hipSuccess) return bail("jobs", e);
    const int pair_slots = max_batch + 1;
    if ((e = hipMalloc((void**)&c->d_pair_i, sizeof(int) * (size_t)pair_slots * kp_cap)) != hipSuccess) return bail("pairs", e);
    if ((e = hipMalloc((void**)&c->d_pair_j, sizeof(int) * (size_t)pair_slots * kp_cap)) != hipSuccess) return bail("pairs", e);
    if ((e = hipMalloc((void**)&c->d_pair_n, sizeof(int) * pair_slots)) != hipSuccess) return bail("pairs", e);
    if ((e = hipMemset(c->d_pair_n, 0, sizeof(int) * pair_slots)) != hipSuccess) return bail("pairs", e);
    if ((e = hipMalloc((void**)&c->d_img, (size_t)2 * max_batch * rows * cols)) != hipSuccess) return bail("staging", e);
    for (int k = 0; k < 2; ++k) {
        if ((e = hipMalloc((void**)&c->d_fd[k], (size_t)kp_cap * VO_DESC_LEN)) != hipSuccess) return bail("staging", e);
        if ((e = hipMalloc((void**)&c->d_fm[k], sizeof(DescMeta) * kp_cap)) != hipSuccess) return bail("staging", e);
        if ((e = hipMalloc((void**)&c->d_ff[k], sizeof(float) * kp_cap * VO_DESC_LEN)) != hipSuccess) return bail("staging", e);
    }
    if ((e = hipMalloc((void**)&c->d_fn, sizeof(int) * 2)) != hipSuccess) return bail("staging", e);
    if ((e = hipMalloc((void**)&c->d_bad, sizeof(int))) != hipSuccess) return bail("staging", e);
    if ((e = hipMalloc((void**)&c->d_mi, sizeof(int) * kp_cap)) != hipSuccess) return bail("staging", e);
    if ((e = hipMalloc((void**)&c->d_mj, sizeof(int) * kp_cap)) != hipSuccess) return bail("staging", e);
    if ((e = hipMalloc((void**)&c->d_mn, sizeof(int))) != hipSuccess) return bail("staging", e);
    if ((e = geom_alloc(c->gb, max_batch, kp_cap, c->rp.max_num_trials)) != hipSuccess) return bail("geometry buffers", e);
    // job tables
    std::vector<MatchJob> jobs(n_jobs);
    memset(jobs.data(), 0, sizeof(MatchJob) * n_jobs);
    const size_t dstride = (size_t)kp_cap * VO_DESC_LEN;
    for (int f = 0; f < max_batch; ++f) {
        MatchJob& J = jobs[job_stereo(c, f)];
        const int il = 2 * f, ir = 2 * f + 1;
        J.d1 = c->sb.desc + il * dstride; J.m1 = c->sb.meta + (size_t)il * kp_cap; J.idx1 = nullptr; J.n1 = c->sb.n_kp + il;
        J.d2 = c->sb.desc + ir * dstride; J.m2 = c->sb.meta + (size_t)ir * kp_cap; J.idx2 = nullptr; J.n2 = c->sb.n_kp + ir;
        J.out_i = c->d_pair_i + (size_t)f * kp_cap; J.out_j = c->d_pair_j + (size_t)f * kp_cap; J.out_n = c->d_pair_n + f;
        J.cap = kp_cap;
    }
    geom_fill_track_jobs(c->gb, jobs.data(), c->max_batch, job_track(c, 0, 0), c->sb, c->d_pair_i, c->d_pair_j, c->d_pair_n,
                         kp_cap);
    {
        MatchJob& J = jobs[job_single(c)];
        J.d1 = c->d_fd[0]; J.m1 = c->d_fm[0]; J.idx1 = nullptr; J.n1 = c->d_fn;
        J.d2 = c->d_fd[1]; J.m2 = c->d_fm[1]; J.idx2 = nullptr; J.n2 = c->d_fn + 1;
        J.out_i = c->d_mi; J.out_j = c->d_mj; J.out_n = c->d_mn; J.cap = kp_cap;
    }
    if ((e = hipMemcpy(c->d_jobs, jobs.data(), sizeof(MatchJob) * n_jobs, hipMemcpyHostToDevice)) != hipSuccess) return bail("jobs copy", e);
    // second buffer set of the asynchronous pipelines (a full replica of set 0's per-frame state)
    {
        vo_ctx::AuxSet& X = c->aux;
        const int xn = 5 * max_batch;
        if ((e = sift_alloc(X.sb, c->py, kp_cap, 4 * kp_cap)) != hipSuccess) return bail("sift buffers (set 1)", e);
        if ((e = match_alloc(X.mb, max_batch, kp_cap)) != hipSuccess) return bail("match buffers (set 1)", e);
        if ((e = hipMalloc((void**)&X.d_jobs, sizeof(MatchJob) * xn)) != hipSuccess) return bail("jobs (set 1)", e);
        if ((e = hipMalloc((void**)&X.pair_i, sizeof(int) * (size_t)pair_slots * kp_cap)) != hipSuccess) return bail("pairs", e);
        if ((e = hipMalloc((void**)&X.pair_j, sizeof(int) * (size_t)pair_slots * kp_cap)) != hipSuccess) return bail("pairs", e);
        if ((e = hipMalloc((void**)&X.pair_n, sizeof(int) * pair_slots)) != hipSuccess) return bail("pairs", e);
        if ((e = hipMemset(X.pair_n, 0, sizeof(int) * pair_slots)) != hipSuccess) return bail("pairs", e);
        if ((e = geom_alloc(X.gb, max_batch, kp_cap, c->rp.max_num_trials)) != hipSuccess) return bail("geometry buffers (set 1)", e);
        std::vector<MatchJob> xj(xn);
        memset(xj.data(), 0, sizeof(MatchJob) * xn);
        for (int f = 0; f < max_batch; ++f) {
            MatchJob& J = xj[f];
            const int il = 2 * f, ir = 2 * f + 1;
            J.d1 = X.sb.desc + il * dstride; J.m1 = X.sb.meta + (size_t)il * kp_cap; J.idx1 = nullptr; J.n1 = X.sb.n_kp + il;
            J.d2 = X.sb.desc + ir * dstride; J.m2 = X.sb.meta + (size_t)ir * kp_cap; J.idx2 = nullptr; J.n2 = X.sb.n_kp + ir;
            J.out_i = X.pair_i + (size_t)f * kp_cap; J.out_j = X.pair_j + (size_t)f * kp_cap; J.out_n = X.pair_n + f;
            J.cap = kp_cap;
        }
        geom_fill_track_jobs(X.gb, xj.data(), max_batch, job_track(c, 0, 0), X.sb, X.pair_i, X.pair_j, X.pair_n, kp_cap);
        if ((e = hipMemcpy(X.d_jobs, xj.data(), sizeof(MatchJob) * xn, hipMemcpyHostToDevice)) != hipSuccess)
            return bail("jobs copy (set 1)", e);
    }
    for (int k = 0; k < VO_STEP_DEPTH; ++k) {
        vo_ctx::StepHost& H = c->sh[k];
        if ((e = hipEventCreateWithFlags(&H.ev, hipEventDisableTiming)) != hipSuccess) return bail("event", e);
        if ((e = hipMalloc((void**)&H.d_pX, sizeof(float) * 3 * max_batch * kp_cap)) != hipSuccess) return bail("packed rows", e);
        if ((e = hipMalloc((void**)&H.d_pkeep, (size_t)max_batch * kp_cap)) != hipSuccess) return bail("packed rows", e);
        if ((e = hipHostMalloc((void**)&H.fg, sizeof(FrameGeom) * max_batch, 0)) != hipSuccess) return bail("pinned", e);
        if ((e = hipHostMalloc((void**)&H.nkp, sizeof(int) * 2 * max_batch, 0)) != hipSuccess) return bail("pinned", e);
        if ((e = hipHostMalloc((void**)&H.ncand, sizeof(int) * 2 * max_batch, 0)) != hipSuccess) return bail("pinned", e);
        if ((e = hipHostMalloc((void**)&H.np, sizeof(int) * max_batch, 0)) != hipSuccess) return bail("pinned", e);
        if ((e = hipHostMalloc((void**)&H.rows, sizeof(int) * max_batch, 0)) != hipSuccess) return bail("pinned", e);
        if ((e = hipHostMalloc((void**)&H.pX, sizeof(float) * 3 * max_batch * kp_cap, 0)) != hipSuccess) return bail("pinned", e);
        if ((e = hipHostMalloc((void**)&H.pkeep, (size_t)max_batch * kp_cap, 0)) != hipSuccess) return bail("pinned", e);
    }
    return c;
}

void vo_destroy(vo_ctx* c)
{
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    destroy_buffers(c);
    destroy_streams(c);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

int vo_set_concurrency(vo_ctx* c, int n_streams)
{
    if (!c || n_streams < 1 || n_streams > vo_ctx::MAX_SUB) return VO_ERR_ARG;
    c->n_sub = n_streams;
    return VO_OK;
}

int vo_set_calib(vo_ctx* c, const vo_calib* calib)
{
    if (!c || !calib) return VO_ERR_ARG;
    c->calib = *calib;
    c->has_calib = true;
    return VO_OK;
}

int vo_set_profiling(vo_ctx* c, int enable)
{
    if (!c) return VO_ERR_ARG;
    c->prof.on = enable != 0;
    c->prof.reset_totals();
    return VO_OK;
}

static int finish(vo_ctx* c);
int vo_kernel_times(vo_ctx* c, const char** names, double* ms, int* calls, int capacity, int* n)
{
    if (!c) return VO_ERR_ARG;
    hipSetDevice(c->device);
    if (c->prof.on) {                                  // asynchronous calls may still be in flight
        g_prof = &c->prof;
        int rc = finish(c);
        if (rc) return rc;
    }
    int m = (int)c->prof.names.size();
    if (n) *n = m;
    for (int i = 0; i < m && i < capacity; ++i) {
        if (names) names[i] = c->prof.names[i].c_str();
        if (ms) ms[i] = c->prof.ms[i];
        if (calls) calls[i] = c->prof.calls[i];
    }
    return VO_OK;
}

// Synchronise the stream, collect profiling, translate errors.
static int finish(vo_ctx* c)
{
    hipError_t e = hipStreamSynchronize(c->stream);
    for (int k = 0; k < 2 && e == hipSuccess; ++k) e = hipStreamSynchronize(c->sub[k]);
    if (e != hipSuccess) return fail(c, VO_ERR_HIP, "stream sync: %s", hipGetErrorString(e));
    e = hipGetLastError();
    if (e != hipSuccess) return fail(c, VO_ERR_HIP, "launch: %s", hipGetErrorString(e));
    if (c->prof.on) c->prof.collect();
    g_prof = nullptr;
    return VO_OK;
}
// quiesce: calls that run on `stream` over the context's own buffers first wait for any
// batch still in flight on either buffer set (no host synchronisation)
// Calls other than the step pipeline's own are refused while step batches are pending
// (they reuse buffer set 0).
static int begin_call(vo_ctx* c, bool quiesce = true, bool step = false)
{
    hipSetDevice(c->device);
    if (!step && !c->pending.empty())
        return fail(c, VO_ERR_STATE, "asynchronous step batches pending (vo_step_collect first)");
    g_prof = c->prof.on ? &c->prof : nullptr;
    if (quiesce)
        for (int k = 0; k < 2; ++k) hipStreamWaitEvent(c->stream, c->ev_done[k], 0);
    return VO_OK;
}
#define BEGIN_CALL(...) do { int rc_ = begin_call(__VA_ARGS__); if (rc_) return rc_; } while (0)

// MATLAB images are column-major: pixel (r, c) of image n at src[n * ld * cols + c * ld + r]
// (ld >= rows).  32 x 32 LDS tile transpose into tightly packed row-major frames.
__global__ __launch_bounds__(256) void k_cm_to_rm_u8(const uint8_t* __restrict__ src, int ld, int rows, int cols,
                                                     uint8_t* __restrict__ dst)
{
    __shared__ uint8_t t[32][33];
    const int n = blockIdx.z, r0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
    const uint8_t* s = src + (size_t)n * ld * cols;
    uint8_t* d = dst + (size_t)n * rows * cols;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int k = ty; k < 32; k += 8) {
        const int c = c0 + k, r = r0 + tx;                  // lanes walk a source column (contiguous)
        if (c < cols && r < rows) t[k][tx] = s[(size_t)c * ld + r];
    }
    __syncthreads();
    for (int k = ty; k < 32; k += 8) {
        const int r = r0 + k, c = c0 + tx;                  // lanes walk a destination row
        if (r < rows && c < cols) d[(size_t)r * cols + c] = t[tx][k];
    }
}

// host images -> tightly packed row-major device frames at dst (n frames).  col_major: the
// buffer as MATLAB holds it (copied as it lies into the context's column-major staging, then
// transposed on the device).
static int stage_images(vo_ctx* c, const uint8_t* img, int ld, int col_major, int n, uint8_t* dst)
{
    const int rows = c->rows, cols = c->cols;
    if (!col_major) {
        HIPC(c, hipMemcpy2DAsync(dst, cols, img, ld, cols, (size_t)rows * n, hipMemcpyHostToDevice, c->stream));
        return VO_OK;
    }
    // exactly the bytes the frames span: the last column of the last frame ends `rows` bytes
    // into its ld-byte slot (a padded view, ld > rows, must not be read past its end)
    const size_t need = (size_t)ld * ((size_t)cols * n - 1) + rows;
    if (need > c->cm_cap) {
        HIPC(c, hipStreamSynchronize(c->stream));
        hipFree(c->d_cm);
        c->d_cm = nullptr;
        c->cm_cap = 0;
        HIPC(c, hipMalloc((void**)&c->d_cm, need));
        c->cm_cap = need;
    }
    HIPC(c, hipMemcpyAsync(c->d_cm, img, need, hipMemcpyHostToDevice, c->stream));
    VO_LAUNCH(k_cm_to_rm_u8, dim3((rows + 31) / 32, (cols + 31) / 32, n), dim3(256), 0, c->stream, c->d_cm, ld, rows, cols, dst);
    return VO_OK;
}

int vo_sift_ex(vo_ctx* c, const uint8_t* img, int rows, int cols, int ld, int col_major, vo_keypoint* kps, uint8_t* desc,
               int capacity, int* n_out)
{
    if (!c || !img || rows != c->rows || cols != c->cols || (col_major != 0 && col_major != 1) ||
        ld < (col_major ? rows : cols))
        return fail(c, VO_ERR_ARG, "vo_sift: bad arguments");
    BEGIN_CALL(c);
    int rc_stage = stage_images(c, img, ld, col_major, 1, c->d_img);
    if (rc_stage) return rc_stage;
    ImageSrc src{c->d_img, c->d_img, (size_t)rows * cols, cols, 0};
    sift_enqueue(c->py, c->sb, src, 1, c->sp, c->stream, c->d_py);
    c->last_set = 0;                                   // vo_fetch_* now read this result (set 0)
    int n = 0, n_cand = 0;
    HIPC(c, hipMemcpyAsync(&n, c->sb.n_kp, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemcpyAsync(&n_cand, c->sb.n_cand, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    int rc = finish(c);
    if (rc) return rc;
    if (n_out) *n_out = n;
    int m = std::min(std::min(n, c->sb.kp_cap), capacity);
    if (m > 0) {
        if (kps) HIPC(c, hipMemcpy(kps, c->sb.kp, sizeof(vo_keypoint) * m, hipMemcpyDeviceToHost));
        if (desc) HIPC(c, hipMemcpy(desc, c->sb.desc, (size_t)m * VO_DESC_LEN, hipMemcpyDeviceToHost));
    }
    if (n_cand > c->sb.cand_cap)
        return fail(c, VO_ERR_CAPACITY, "vo_sift: %d extremum candidates exceed the candidate list (%d = 4 x max_keypoints)",
                    n_cand, c->sb.cand_cap);
    if (n > c->sb.kp_cap) return fail(c, VO_ERR_CAPACITY, "vo_sift: %d keypoints exceed max_keypoints %d", n, c->sb.kp_cap);
    if (n > capacity) return fail(c, VO_ERR_CAPACITY, "vo_sift: %d keypoints exceed capacity %d", n, capacity);
    return VO_OK;
}

int vo_sift(vo_ctx* c, const uint8_t* img, int rows, int cols, int ld, vo_keypoint* kps, uint8_t* desc, int capacity,
            int* n_out)
{
    return vo_sift_ex(c, img, rows, cols, ld, 0, kps, desc, capacity, n_out);
}

// matchFeatures on the two staged descriptor sets d_fd[0] (n1 rows) / d_fd[1] (n2 rows)
static int match_staged(vo_ctx* c, int n1, int n2, uint32_t* pairs, int capacity, int* n_pairs, const char* who)
{
    int nn[2] = {n1, n2};
    HIPC(c, hipMemcpyAsync(c->d_fn, nn, sizeof(nn), hipMemcpyHostToDevice, c->stream));
    desc_meta_launch(c->d_fd[0], c->d_fm[0], n1, c->stream);
    desc_meta_launch(c->d_fd[1], c->d_fm[1], n2, c->stream);
    match_launch(c->mb, c->d_jobs + job_single(c), 1, c->mp, c->stream);
    int P = 0;
    HIPC(c, hipMemcpyAsync(&P, c->d_mn, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    int rc = finish(c);
    if (rc) return rc;
    if (n_pairs) *n_pairs = P;
    int m = std::min(P, capacity);
    if (m > 0 && pairs) {
        std::vector<int> ii(m), jj(m);
        HIPC(c, hipMemcpy(ii.data(), c->d_mi, sizeof(int) * m, hipMemcpyDeviceToHost));
        HIPC(c, hipMemcpy(jj.data(), c->d_mj, sizeof(int) * m, hipMemcpyDeviceToHost));
        for (int k = 0; k < m; ++k) { pairs[2 * k] = (uint32_t)ii[k] + 1; pairs[2 * k + 1] = (uint32_t)jj[k] + 1; }
    }
    if (P > capacity) return fail(c, VO_ERR_CAPACITY, "%s: %d pairs exceed capacity %d", who, P, capacity);
    return VO_OK;
}

int vo_match(vo_ctx* c, const uint8_t* F1, int n1, const uint8_t* F2, int n2, uint32_t* pairs, int capacity, int* n_pairs)
{
    if (!c || n1 < 0 || n2 < 0 || (n1 && !F1) || (n2 && !F2)) return fail(c, VO_ERR_ARG, "vo_match: bad arguments");
    if (n1 > c->sb.kp_cap || n2 > c->sb.kp_cap) return fail(c, VO_ERR_CAPACITY, "vo_match: more rows than max_keypoints");
    BEGIN_CALL(c);
    if (n1) HIPC(c, hipMemcpyAsync(c->d_fd[0], F1, (size_t)n1 * VO_DESC_LEN, hipMemcpyHostToDevice, c->stream));
    if (n2) HIPC(c, hipMemcpyAsync(c->d_fd[1], F2, (size_t)n2 * VO_DESC_LEN, hipMemcpyHostToDevice, c->stream));
    return match_staged(c, n1, n2, pairs, capacity, n_pairs, "vo_match");
}

int vo_match_f32(vo_ctx* c, const float* F1, int n1, int ld1, const float* F2, int n2, int ld2, int col_major,
                 uint32_t* pairs, int capacity, int* n_pairs)
{
    if (!c || n1 < 0 || n2 < 0 || (n1 && !F1) || (n2 && !F2) || (col_major != 0 && col_major != 1))
        return fail(c, VO_ERR_ARG, "vo_match_f32: bad arguments");
    if ((n1 && ld1 < (col_major ? n1 : VO_DESC_LEN)) || (n2 && ld2 < (col_major ? n2 : VO_DESC_LEN)))
        return fail(c, VO_ERR_ARG, "vo_match_f32: leading dimension too small");
    if (n1 > c->sb.kp_cap || n2 > c->sb.kp_cap) return fail(c, VO_ERR_CAPACITY, "vo_match_f32: more rows than max_keypoints");
    BEGIN_CALL(c);
    HIPC(c, hipMemsetAsync(c->d_bad, 0, sizeof(int), c->stream));
    const float* src[2] = {F1, F2};
    const int n[2] = {n1, n2}, ld[2] = {ld1, ld2};
    for (int s = 0; s < 2; ++s) {
        if (!n[s]) continue;
        // the matrix as it lies in host memory (MATLAB: n x 128 column-major, ld = n), one copy
        const size_t elems = col_major ? (size_t)ld[s] * (VO_DESC_LEN - 1) + n[s] : (size_t)ld[s] * (n[s] - 1) + VO_DESC_LEN;
        if (elems > (size_t)c->sb.kp_cap * VO_DESC_LEN) return fail(c, VO_ERR_CAPACITY, "vo_match_f32: matrix exceeds staging");
        HIPC(c, hipMemcpyAsync(c->d_ff[s], src[s], sizeof(float) * elems, hipMemcpyHostToDevice, c->stream));
        pack_f32_desc_launch(c->d_ff[s], n[s], ld[s], col_major, c->d_fd[s], c->d_bad, c->stream);
    }
    int bad = 0;
    HIPC(c, hipMemcpyAsync(&bad, c->d_bad, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    int rc = finish(c);
    if (rc) return rc;
    // u8-valued rows (libvo / SIFT descriptors, what VO.m passes): the exact-integer spec of the
    // hot path; any other single features: the float SSD spec (match_f32_launch)
    if (!bad) return match_staged(c, n1, n2, pairs, capacity, n_pairs, "vo_match_f32");
    if (!c->d_fa || !c->d_fbt || !c->d_fres) {
        // all three or none: a failed allocation leaves the context without any of them, so the
        // next call allocates again instead of launching on a null buffer
        const size_t fb = sizeof(float) * (size_t)c->sb.kp_cap * VO_DESC_LEN;
        float* fa = nullptr; float* fbt = nullptr; int* fres = nullptr;
        hipError_t e;
        if ((e = hipMalloc((void**)&fa, fb)) != hipSuccess || (e = hipMalloc((void**)&fbt, fb)) != hipSuccess ||
            (e = hipMalloc((void**)&fres, sizeof(int) * c->sb.kp_cap)) != hipSuccess) {
            hipFree(fa); hipFree(fbt); hipFree(fres);
            return fail(c, VO_ERR_HIP, "vo_match_f32: %s", hipGetErrorString(e));
        }
        hipFree(c->d_fa); hipFree(c->d_fbt); hipFree(c->d_fres);
        c->d_fa = fa; c->d_fbt = fbt; c->d_fres = fres;
    }
    match_f32_launch(c->d_ff[0], n1, ld1, c->d_ff[1], n2, ld2, col_major, c->d_fa, c->d_fbt, c->d_fres, c->mp, c->stream);
    std::vector<int> res((size_t)n1 + 1);
    if (n1) HIPC(c, hipMemcpyAsync(res.data(), c->d_fres, sizeof(int) * n1, hipMemcpyDeviceToHost, c->stream));
    rc = finish(c);
    if (rc) return rc;
    int P = 0;
    for (int i = 0; i < n1; ++i) {
        if (res[i] < 0) continue;
        if (pairs && P < capacity) { pairs[2 * P] = (uint32_t)i + 1; pairs[2 * P + 1] = (uint32_t)res[i] + 1; }
        ++P;
    }
    if (n_pairs) *n_pairs = P;
    if (P > capacity) return fail(c, VO_ERR_CAPACITY, "vo_match_f32: %d pairs exceed capacity %d", P, capacity);
    return VO_OK;
}

// SIFT + stereo match on B frames already in device memory.
// buffers of set `set` of the asynchronous batch pipeline
// vo_pair_stats.flags / vo_step_out.flags of one frame's n images: VO_FLAG_KEYPOINTS if an
// image detected more keypoints than max_keypoints, VO_FLAG_CANDIDATES if its extremum test
// (k_ext_inner's partial candidates included) produced more candidates than the list holds,
// so k_seg_emit dropped some in scan order and the keypoint set is incomplete
static int capacity_flags(const SiftBuffers& sb, const int* nkp, const int* ncand, int n)
{
    int fl = 0;
    for (int i = 0; i < n; ++i) {
        if (nkp[i] > sb.kp_cap) fl |= VO_FLAG_KEYPOINTS;
        if (ncand[i] > sb.cand_cap) fl |= VO_FLAG_CANDIDATES;
    }
    return fl;
}

struct SetRef {
    SiftBuffers* sb; MatchBuffers* mb; MatchJob* jobs; int* pair_i; int* pair_j; int* pair_n;
    GeomBuffers* gb; MatchJob* track_jobs;
};
static SetRef set_ref(vo_ctx* c, int set)
{
    if (set == 0)
        return {&c->sb, &c->mb, c->d_jobs + job_stereo(c, 0), c->d_pair_i, c->d_pair_j, c->d_pair_n, &c->gb,
                c->d_jobs + job_track(c, 0, 0)};
    return {&c->aux.sb, &c->aux.mb, c->aux.d_jobs, c->aux.pair_i, c->aux.pair_j, c->aux.pair_n, &c->aux.gb,
            c->aux.d_jobs + job_track(c, 0, 0)};
}

// SIFT of 2B images + stereo matching of B frames into buffer set `set`.  The frames are
// split into `parts` (vo_set_concurrency); every part's scale space runs on sub[0] and its
// feature stages + stereo matching on sub[1] once that part's scale space is done, so the
// features of part k overlap the scale space of part k+1 (and of the next call, which uses
// the other set).  Inputs are ordered after earlier work on `stream`; the set's previous
// contents are released by its ev_done.  With `join`, `stream` waits for the result.
// Where the extremum test of octaves 1.. runs: 1 (default) on the feature stream after the
// scale space, 0 at the scale space's tail.  With the faster k_desc / k_orient of round 3 the
// scale-space stream became the critical path again, and moving that 0.4 ms of test off it
// gave 7.51-7.55 vs 7.66-7.77 ms per 64-frame step (A/B on one box).
#ifndef VO_EXT_SPLIT
#define VO_EXT_SPLIT 1
#endif
// Where the LDS-sized octaves (k_small_pyr: one 1024-thread workgroup per image, ~120 KB of LDS,
// 0.13 ms isolated but ~1 ms in situ while it waits for a CU with that much free LDS) run:
// 0 at the scale space's tail; 1 at the head of the feature stream's second part (measured
// slower: the feature stream is the critical one at 128 frames per step); 2 on a
// stream of their own (sub[2]) after the level blurs, so neither stream waits for its
// placement -- only the extremum test of the small octaves does.
#ifndef VO_ARENA_EVENT
#define VO_ARENA_EVENT 1          // the scale space of a set waits for its arena's last reader, not the whole feature stream
#endif
#ifndef VO_SMALL_STREAM
#define VO_SMALL_STREAM 0
#endif
static int enqueue_sift_stereo(vo_ctx* c, int set, const uint8_t* d_l, const uint8_t* d_r, int B, bool join,
                               bool fork = true)
{
    const size_t fs = (size_t)c->rows * c->cols;
    const int parts = std::min(c->n_sub, B);
    SetRef S = set_ref(c, set);
    hipStream_t sp = c->sub[0], st = c->sub[1], ss = c->sub[2];
    if (fork) {                                                 // inputs / earlier work on `stream`
        HIPC(c, hipEventRecord(c->ev_fork, c->stream));
        HIPC(c, hipStreamWaitEvent(sp, c->ev_fork, 0));
    }
#if VO_ARENA_EVENT
    // the set's arena free: its previous call's last reader (k_desc) is done -- the stereo match
    // of that call (descriptors only) may still run; everything else of the set is written by st,
    // in order behind it
    HIPC(c, hipStreamWaitEvent(sp, c->ev_arena[set], 0));
#else
    HIPC(c, hipStreamWaitEvent(sp, c->ev_done[set], 0));      // set free (its previous features done)
#endif
    const int o_small = sift_small_octave(c->py);
    const bool ext_on_st = VO_EXT_SPLIT || VO_SMALL_STREAM != 0;   // the test of octaves 1.. on st
    // scale space on sp; octave 0's extremum test on st as soon as octave 0 is built (beside the
    // scale space of octaves 1..), the other octaves' on st after the scale space (VO_EXT_SPLIT)
    // -- the split that balances the two streams
    for (int p = 0; p < parts; ++p) {
        const int f0 = B * p / parts, nf = B * (p + 1) / parts - f0;
        ImageSrc src{d_l + f0 * fs, d_r + f0 * fs, fs, c->cols, 0};
        SiftBuffers v = sift_view(*S.sb, c->py, 2 * f0, 2 * nf);
        sift_enqueue_pyramid(c->py, v, src, 2 * nf, c->sp, sp, c->d_py, c->ev_o0[p]);
        if (VO_SMALL_STREAM == 0) sift_enqueue_small(c->py, v, 2 * nf, sp, c->d_py);
        if (!ext_on_st) sift_enqueue_extrema(c->py, v, 2 * nf, c->sp, sp, c->d_py, 1, c->py.n_oct);
        HIPC(c, hipEventRecord(c->ev_join[p], sp));
        if (VO_SMALL_STREAM == 2) {
            HIPC(c, hipStreamWaitEvent(ss, c->ev_join[p], 0));
            sift_enqueue_small(c->py, v, 2 * nf, ss, c->d_py);
            HIPC(c, hipEventRecord(c->ev_small[p], ss));
        }
    }
    for (int p = 0; p < parts; ++p) {
        const int f0 = B * p / parts, nf = B * (p + 1) / parts - f0;
        SiftBuffers v = sift_view(*S.sb, c->py, 2 * f0, 2 * nf);
        // (a synchronous profiled call -- bench.py's isolated pass -- starts it after the whole
        // scale space, so its per-kernel durations stay undisturbed)
        const bool iso = c->prof.on && join;
        if (iso && VO_SMALL_STREAM == 2) HIPC(c, hipStreamWaitEvent(st, c->ev_small[p], 0));
        HIPC(c, hipStreamWaitEvent(st, iso ? c->ev_join[p] : c->ev_o0[p], 0));
        sift_enqueue_extrema(c->py, v, 2 * nf, c->sp, st, c->d_py, 0, 1);
        HIPC(c, hipStreamWaitEvent(st, c->ev_join[p], 0));
        if (VO_SMALL_STREAM == 1) sift_enqueue_small(c->py, v, 2 * nf, st, c->d_py);
        if (ext_on_st) {
            sift_enqueue_extrema(c->py, v, 2 * nf, c->sp, st, c->d_py, 1, o_small);
            if (VO_SMALL_STREAM == 2) HIPC(c, hipStreamWaitEvent(st, c->ev_small[p], 0));
            sift_enqueue_extrema(c->py, v, 2 * nf, c->sp, st, c->d_py, o_small, c->py.n_oct);
        }
        sift_enqueue_features(c->py, v, 2 * nf, c->sp, st, c->d_py);
        if (p == parts - 1) HIPC(c, hipEventRecord(c->ev_arena[set], st));
        match_launch(match_view(*S.mb, f0), S.jobs + f0, nf, c->mp, st);
    }
    HIPC(c, hipEventRecord(c->ev_done[set], st));
    if (join) HIPC(c, hipStreamWaitEvent(c->stream, c->ev_done[set], 0));
    c->last_set = set;
    return VO_OK;
}

int vo_sift_match_batch_dev(vo_ctx* c, const uint8_t* d_lefts, const uint8_t* d_rights, int B, vo_pair_stats* stats)
{
    if (!c || !d_lefts || !d_rights || B < 1 || B > c->max_batch) return fail(c, VO_ERR_ARG, "vo_sift_match_batch_dev: bad arguments");
    BEGIN_CALL(c, false);
    const int set = c->next_set;
    c->next_set ^= 1;
    const bool sync = stats != nullptr;      // profiling events are collected by vo_kernel_times
    int rc = enqueue_sift_stereo(c, set, d_lefts, d_rights, B, sync);
    if (rc) return rc;
    c->last_B = B;
    if (!sync) {
        g_prof = nullptr;
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return fail(c, VO_ERR_HIP, "launch: %s", hipGetErrorString(e));
        return VO_OK;
    }
    SetRef S = set_ref(c, set);
    std::vector<int> nk(2 * B), nc(2 * B), np(B);
    HIPC(c, hipMemcpyAsync(nk.data(), S.sb->n_kp, sizeof(int) * 2 * B, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemcpyAsync(nc.data(), S.sb->n_cand, sizeof(int) * 2 * B, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemcpyAsync(np.data(), S.pair_n, sizeof(int) * B, hipMemcpyDeviceToHost, c->stream));
    rc = finish(c);
    if (rc) return rc;
    if (stats) {
        for (int f = 0; f < B; ++f) {
            stats[f].n_left = nk[2 * f]; stats[f].n_right = nk[2 * f + 1]; stats[f].n_stereo = np[f];
            stats[f].flags = capacity_flags(c->sb, nk.data() + 2 * f, nc.data() + 2 * f, 2);
        }
    }
    return VO_OK;
}

int vo_fetch_keypoints(vo_ctx* c, int image, vo_keypoint* kps, uint8_t* desc, int capacity, int* n)
{
    if (!c || image < 0 || image >= c->sb.n_img) return fail(c, VO_ERR_ARG, "vo_fetch_keypoints: bad image");
    hipSetDevice(c->device);
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipEventSynchronize(c->ev_done[c->last_set]));
    // batch results live in the last call's buffer set (set 1 holds stereo frames only)
    const SiftBuffers& B = (c->last_set == 1 && image < 2 * c->max_batch) ? c->aux.sb : c->sb;
    int cnt = 0;
    HIPC(c, hipMemcpy(&cnt, B.n_kp + image, sizeof(int), hipMemcpyDeviceToHost));
    if (n) *n = cnt;
    int m = std::min(std::min(cnt, B.kp_cap), capacity);
    if (m > 0) {
        if (kps) HIPC(c, hipMemcpy(kps, B.kp + (size_t)image * B.kp_cap, sizeof(vo_keypoint) * m, hipMemcpyDeviceToHost));
        if (desc) HIPC(c, hipMemcpy(desc, B.desc + (size_t)image * B.kp_cap * VO_DESC_LEN, (size_t)m * VO_DESC_LEN, hipMemcpyDeviceToHost));
    }
    return VO_OK;
}

int vo_fetch_candidate_counts(vo_ctx* c, int image, int* n_cand, int* n_accepted)
{
    if (!c || image < 0 || image >= c->sb.n_img) return fail(c, VO_ERR_ARG, "vo_fetch_candidate_counts: bad image");
    hipSetDevice(c->device);
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipEventSynchronize(c->ev_done[c->last_set]));
    const SiftBuffers& B = (c->last_set == 1 && image < 2 * c->max_batch) ? c->aux.sb : c->sb;
    int v[2] = {0, 0};
    HIPC(c, hipMemcpy(&v[0], B.n_cand + image, sizeof(int), hipMemcpyDeviceToHost));
    HIPC(c, hipMemcpy(&v[1], B.n_acc + image, sizeof(int), hipMemcpyDeviceToHost));
    if (n_cand) *n_cand = v[0];
    if (n_accepted) *n_accepted = v[1];
    return VO_OK;
}

int vo_fetch_gaussian(vo_ctx* c, int image, int octave, int level, float* out, int capacity, int* rows, int* cols)
{
    if (!c || image < 0 || image >= c->sb.n_img || octave < 0 || octave >= c->py.n_oct || level < 0 ||
        level >= c->py.L + 3)
        return fail(c, VO_ERR_ARG, "vo_fetch_gaussian: bad image/octave/level");
    hipSetDevice(c->device);
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipEventSynchronize(c->ev_done[c->last_set]));
    const SiftBuffers& B = (c->last_set == 1 && image < 2 * c->max_batch) ? c->aux.sb : c->sb;
    const OctGeom& g = c->py.oct[octave];
    if (rows) *rows = g.rows;
    if (cols) *cols = g.cols;
    if (!out) return VO_OK;
    if (capacity < g.rows * g.cols) return fail(c, VO_ERR_CAPACITY, "vo_fetch_gaussian: capacity %d < %d", capacity, g.rows * g.cols);
    const float* src = B.arena + (size_t)image * c->py.istride + g.g_off[level];
    HIPC(c, hipMemcpy2D(out, sizeof(float) * g.cols, src, sizeof(float) * g.pitch, sizeof(float) * g.cols, g.rows,
                        hipMemcpyDeviceToHost));
    return VO_OK;
}

int vo_fetch_stereo_pairs(vo_ctx* c, int frame, uint32_t* pairs, int capacity, int* n)
{
    if (!c || frame < 0 || frame >= c->max_batch) return fail(c, VO_ERR_ARG, "vo_fetch_stereo_pairs: bad frame");
    hipSetDevice(c->device);
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipEventSynchronize(c->ev_done[c->last_set]));
    SetRef S = set_ref(c, c->last_set);
    int P = 0;
    HIPC(c, hipMemcpy(&P, S.pair_n + frame, sizeof(int), hipMemcpyDeviceToHost));
    if (n) *n = P;
    int m = std::min(P, capacity);
    if (m > 0 && pairs) {
        std::vector<int> ii(m), jj(m);
        HIPC(c, hipMemcpy(ii.data(), S.pair_i + (size_t)frame * c->sb.kp_cap, sizeof(int) * m, hipMemcpyDeviceToHost));
        HIPC(c, hipMemcpy(jj.data(), S.pair_j + (size_t)frame * c->sb.kp_cap, sizeof(int) * m, hipMemcpyDeviceToHost));
        for (int k = 0; k < m; ++k) { pairs[2 * k] = (uint32_t)ii[k] + 1; pairs[2 * k + 1] = (uint32_t)jj[k] + 1; }
    }
    return VO_OK;
}

}  // extern "C"

// ---- tracking / geometry / loop --------------------------------------------
static vo_calib calib_of(const double P1[12], const double P2[12], const double* K)
{
    vo_calib c;
    memcpy(c.P1, P1, sizeof(c.P1));
    memcpy(c.P2, P2, sizeof(c.P2));
    if (K) memcpy(c.K, K, sizeof(c.K));
    else for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) c.K[3 * i + j] = P1[4 * i + j];
    return c;
}

static StepArgs step_args(vo_ctx* c, int B, int set = 0)
{
    SetRef S = set_ref(c, set);
    StepArgs a;
    a.sb = S.sb;
    a.pair_i = S.pair_i; a.pair_j = S.pair_j; a.pair_n = S.pair_n;
    a.max_frames = c->max_batch; a.B = B; a.kp_cap = c->sb.kp_cap;
    a.first_has_prev = c->have_features ? 1 : 0;
    a.frame_index0 = c->frame_index;
    a.calib = c->calib;
    a.rp = c->rp;
    return a;
}

static void mat4_mul(const double* A, const double* B, double* C)
{
    double T[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            T[4 * i + j] = A[4 * i] * B[j] + A[4 * i + 1] * B[4 + j] + A[4 * i + 2] * B[8 + j] + A[4 * i + 3] * B[12 + j];
    memcpy(C, T, sizeof(T));
}

// world transform of one landmark row, rounded through single (CreateLandmarksFromFeatures.m:17)
static void lm_world(const double* pose, const float* X, double* out)
{
    const double x0 = X[0], x1 = X[1], x2 = X[2];
    for (int a = 0; a < 3; ++a) {
        double w = pose[4 * a] * x0 + pose[4 * a + 1] * x1 + pose[4 * a + 2] * x2 + pose[4 * a + 3];
        out[a] = (double)(float)w;
    }
}

// copy frame f's SIFT results + stereo pairs into the carry slots (prev of the next call's frame 0)
// Frame f of set `from` becomes the carried (previous) frame of set `to`: its keypoints,
// descriptors and stereo pairs are copied into `to`'s carry slots (image slots 2M, 2M+1,
// pair slot M), which frame 0 of the next batch tracks against.
static int enqueue_carry(vo_ctx* c, int from, int f, int to)
{
    const int M = c->max_batch, K = c->sb.kp_cap;
    SetRef A = set_ref(c, from), Z = set_ref(c, to);
    for (int side = 0; side < 2; ++side) {
        const int src = 2 * f + side, dst = 2 * M + side;
        HIPC(c, hipMemcpyAsync(Z.sb->kp + (size_t)dst * K, A.sb->kp + (size_t)src * K, sizeof(vo_keypoint) * K,
                               hipMemcpyDeviceToDevice, c->stream));
        HIPC(c, hipMemcpyAsync(Z.sb->desc + (size_t)dst * K * VO_DESC_LEN, A.sb->desc + (size_t)src * K * VO_DESC_LEN,
                               (size_t)K * VO_DESC_LEN, hipMemcpyDeviceToDevice, c->stream));
        HIPC(c, hipMemcpyAsync(Z.sb->meta + (size_t)dst * K, A.sb->meta + (size_t)src * K, sizeof(DescMeta) * K,
                               hipMemcpyDeviceToDevice, c->stream));
        HIPC(c, hipMemcpyAsync(Z.sb->n_kp + dst, A.sb->n_kp + src, sizeof(int), hipMemcpyDeviceToDevice, c->stream));
    }
    HIPC(c, hipMemcpyAsync(Z.pair_i + (size_t)M * K, A.pair_i + (size_t)f * K, sizeof(int) * K, hipMemcpyDeviceToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(Z.pair_j + (size_t)M * K, A.pair_j + (size_t)f * K, sizeof(int) * K, hipMemcpyDeviceToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(Z.pair_n + M, A.pair_n + f, sizeof(int), hipMemcpyDeviceToDevice, c->stream));
    return VO_OK;
}

// The VO.m loop body for B frames whose images are in device memory, split into a
// device half (submit: everything up to the per-frame results, asynchronous) and a host
// half (collect: pose chain VO.m:130-134 and landmark append CreateLandmarksFromFeatures.m:20).
// Batch n uses buffer set n & 1 and result slot n mod VO_STEP_DEPTH.  Its scale space (sub[0])
// waits only for the arena's last reader of batch n-2 (ev_arena); its feature stages and stereo
// matching (sub[1]) overwrite the keypoints, descriptors and stereo pairs that batch n-2's
// geometry reads, so they wait for the end of that batch on the GPU (its slot event) -- not for
// the host to collect it, so the scale space of batch n runs straight after batch n-1's while
// batch n-2's geometry finishes.  Its tracking, triangulation, MSAC and landmark kernels run on
// `stream` after the SIFT and after the previous batch's carry; then frame B-1 is carried into
// the other set, the landmark rows are packed into the slot and the small per-frame results
// are copied to the slot's pinned host memory.  With fork, the SIFT is also ordered after
// earlier work on `stream` (the synchronous calls' H2D copies).
static int submit_batch(vo_ctx* c, const uint8_t* d_l, const uint8_t* d_r, int B, bool fork)
{
    if (!c->has_calib) return fail(c, VO_ERR_STATE, "vo_step: no calibration (vo_set_calib)");
    if (c->pending.size() >= VO_STEP_DEPTH)
        return fail(c, VO_ERR_STATE, "vo_step_submit_dev: %d batches already pending (collect first)", VO_STEP_DEPTH);
    const int set = c->next_step_set, slot = c->next_slot;
    SetRef S = set_ref(c, set);
    for (const vo_ctx::Pending& q : c->pending)         // batch n-2 (same set), still in flight
        if (q.set == set) HIPC(c, hipStreamWaitEvent(c->sub[1], c->sh[q.slot].ev, 0));
    int rc = enqueue_sift_stereo(c, set, d_l, d_r, B, true, fork);   // `stream` waits for this set's SIFT
    if (rc) return rc;
    StepArgs a = step_args(c, B, set);
    geom_enqueue(*S.gb, *S.mb, S.track_jobs, a, c->mp, c->stream);
    vo_ctx::StepHost& H = c->sh[slot];
    HIPC(c, hipMemcpyAsync(H.fg, S.gb->fg, sizeof(FrameGeom) * B, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemcpyAsync(H.nkp, S.sb->n_kp, sizeof(int) * 2 * B, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemcpyAsync(H.ncand, S.sb->n_cand, sizeof(int) * 2 * B, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemcpyAsync(H.np, S.pair_n, sizeof(int) * B, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemcpyAsync(H.rows, S.gb->lm_rows, sizeof(int) * B, hipMemcpyDeviceToHost, c->stream));
    lm_pack_launch(*S.gb, B, H.d_pX, H.d_pkeep, c->stream);
    if ((rc = enqueue_carry(c, set, B - 1, set ^ 1))) return rc;
    HIPC(c, hipEventRecord(H.ev, c->stream));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(c, VO_ERR_HIP, "launch: %s", hipGetErrorString(e));
    c->pending.push_back({set, slot, B, c->have_features});
    c->next_step_set ^= 1;
    c->next_slot = (slot + 1) % VO_STEP_DEPTH;
    c->have_features = true;
    c->frame_index += B;
    return VO_OK;
}

static int collect_batch(vo_ctx* c, vo_step_out* outs, int capacity, int* n_out)
{
    if (c->pending.empty()) return fail(c, VO_ERR_STATE, "vo_step_collect: no batch pending");
    const vo_ctx::Pending P = c->pending.front();
    if (capacity < P.B) return fail(c, VO_ERR_CAPACITY, "vo_step_collect: %d frames pending, capacity %d", P.B, capacity);
    const int K = c->sb.kp_cap, B = P.B;
    const vo_ctx::StepHost& H = c->sh[P.slot];
    if (c->prof.on) {                                  // profiling: events of every stream are collected
        g_prof = &c->prof;
        int rc = finish(c);
        if (rc) return rc;
    } else {
        HIPC(c, hipEventSynchronize(H.ev));
    }
    // the batch's landmark rows, packed on the device in frame order (k_lm_pack): one copy each
    // of X and keep into pinned memory (per-frame copies into pageable vectors cost ~2 x B
    // staged transfers per batch)
    size_t total = 0;
    std::vector<size_t> roff(B + 1, 0);
    for (int f = 0; f < B; ++f) roff[f + 1] = roff[f] + (size_t)std::min(H.rows[f], K);
    total = roff[B];
    if (c->lm_camera) {
        // camera-frame rows stay on the device: the tracked frames' packed rows are appended to
        // the store by one device-to-device copy on `stream` (ordered before the next submit
        // into this slot, which reuses the packed buffer: it needs this collect first)
        const size_t first = (P.first_tracked ? 0 : roff[1]), add = total - first;
        if (add > 0) {
            if (c->lm_n + add > c->lm_cap) {
                size_t cap = std::max<size_t>({c->lm_n + add, 2 * c->lm_cap, (size_t)1 << 16});
                float* nX = nullptr; uint8_t* nk = nullptr;
                if (hipMalloc((void**)&nX, sizeof(float) * 3 * cap) != hipSuccess ||
                    hipMalloc((void**)&nk, cap) != hipSuccess) {
                    hipFree(nX);
                    return fail(c, VO_ERR_HIP, "vo_step_collect: landmark store of %zu rows", cap);
                }
                // the store at least doubles; the old one is copied on `stream` (in order with the
                // appends) and retired until reset / destroy, so growth never waits for the pipeline
                hipError_t ge = hipSuccess;
                if (c->lm_n > 0) {
                    ge = hipMemcpyAsync(nX, c->d_lmX, sizeof(float) * 3 * c->lm_n, hipMemcpyDeviceToDevice, c->stream);
                    if (ge == hipSuccess) ge = hipMemcpyAsync(nk, c->d_lmkeep, c->lm_n, hipMemcpyDeviceToDevice, c->stream);
                }
                if (ge != hipSuccess) {
                    (void)hipStreamSynchronize(c->stream);   // the copies may be queued: let them drain
                    hipFree(nX); hipFree(nk);
                    return fail(c, VO_ERR_HIP, "vo_step_collect: landmark store growth: %s", hipGetErrorString(ge));
                }
                if (c->d_lmX) c->lm_retired.push_back(c->d_lmX);
                if (c->d_lmkeep) c->lm_retired.push_back(c->d_lmkeep);
                c->d_lmX = nX; c->d_lmkeep = nk; c->lm_cap = cap;
            }
            HIPC(c, hipMemcpyAsync(c->d_lmX + 3 * c->lm_n, H.d_pX + 3 * first, sizeof(float) * 3 * add,
                                   hipMemcpyDeviceToDevice, c->stream));
            HIPC(c, hipMemcpyAsync(c->d_lmkeep + c->lm_n, H.d_pkeep + first, add, hipMemcpyDeviceToDevice, c->stream));
            c->lm_n += add;
        }
    } else if (total > 0) {
        HIPC(c, hipMemcpyAsync(H.pX, H.d_pX, sizeof(float) * 3 * total, hipMemcpyDeviceToHost, c->copy_stream));
        HIPC(c, hipMemcpyAsync(H.pkeep, H.d_pkeep, total, hipMemcpyDeviceToHost, c->copy_stream));
        HIPC(c, hipStreamSynchronize(c->copy_stream));
    }
    c->pending.pop_front();
    c->last_step_set = P.set;
    c->last_step_B = B;
    for (int f = 0; f < B; ++f) {
        vo_step_out& o = outs[f];
        memset(&o, 0, sizeof(o));
        o.n_left = H.nkp[2 * f]; o.n_right = H.nkp[2 * f + 1]; o.n_stereo = H.np[f];
        o.flags = capacity_flags(c->sb, H.nkp + 2 * f, H.ncand + 2 * f, 2);
        memcpy(o.rel_pose, I4, sizeof(I4));
        const bool tracked = f > 0 || P.first_tracked;
        if (c->lm_camera) {
            const size_t r = tracked ? roff[f + 1] - roff[f] : 0;
            c->lm_frame_off.push_back(c->lm_frame_off.back() + (long long)r);
        }
        if (tracked) {
            o.status = H.fg[f].status;
            o.n_tracked = H.fg[f].n_tracked;
            o.n_inliers = H.fg[f].n_inliers;
            if (o.status == VO_OK) {
                memcpy(o.rel_pose, H.fg[f].T, sizeof(H.fg[f].T));
                mat4_mul(c->pose, H.fg[f].T, c->pose);
            }
            const int r = (int)(roff[f + 1] - roff[f]);
            const float* Xf = H.pX + roff[f] * 3;
            const uint8_t* kf = H.pkeep + roff[f];
            o.n_landmarks = r;
            if (!c->lm_camera) {
                size_t base = c->landmarks.size();
                c->landmarks.resize(base + (size_t)r * 3, 0.0);
                for (int m = 0; m < r; ++m)
                    if (kf[m]) lm_world(c->pose, Xf + (size_t)m * 3, &c->landmarks[base + (size_t)m * 3]);
            }
        }
        memcpy(o.pose, c->pose, sizeof(c->pose));
    }
    if (n_out) *n_out = B;
    return VO_OK;
}

// synchronous form: submit + collect (nothing else may be pending)
static int run_batch(vo_ctx* c, const uint8_t* d_l, const uint8_t* d_r, int B, vo_step_out* outs)
{
    if (!c->pending.empty()) return fail(c, VO_ERR_STATE, "vo_step: asynchronous batches pending (vo_step_collect first)");
    int rc = submit_batch(c, d_l, d_r, B, true);
    if (rc) return rc;
    return collect_batch(c, outs, B, nullptr);
}

extern "C" {

int vo_step_batch_dev(vo_ctx* c, const uint8_t* d_l, const uint8_t* d_r, int B, vo_step_out* outs)
{
    if (!c || !d_l || !d_r || !outs || B < 1 || B > c->max_batch) return fail(c, VO_ERR_ARG, "vo_step_batch_dev: bad arguments");
    BEGIN_CALL(c);
    int rc = run_batch(c, d_l, d_r, B, outs);
    g_prof = nullptr;
    return rc;
}

int vo_step_batch_ex(vo_ctx* c, const uint8_t* lefts, const uint8_t* rights, int ld, int col_major, int B, vo_step_out* outs)
{
    if (!c || !lefts || !rights || !outs || B < 1 || B > c->max_batch || (col_major != 0 && col_major != 1) ||
        ld < (col_major ? c->rows : c->cols))
        return fail(c, VO_ERR_ARG, "vo_step_batch: bad arguments");
    BEGIN_CALL(c);
    const size_t fs = (size_t)c->rows * c->cols;
    uint8_t* dl = c->d_img;
    uint8_t* dr = c->d_img + fs * B;
    int rc = stage_images(c, lefts, ld, col_major, B, dl);
    if (!rc) rc = stage_images(c, rights, ld, col_major, B, dr);
    if (!rc) rc = run_batch(c, dl, dr, B, outs);
    g_prof = nullptr;
    return rc;
}

int vo_step_batch(vo_ctx* c, const uint8_t* lefts, const uint8_t* rights, int ld, int B, vo_step_out* outs)
{
    return vo_step_batch_ex(c, lefts, rights, ld, 0, B, outs);
}

int vo_step(vo_ctx* c, const uint8_t* left, const uint8_t* right, int ld, vo_step_out* out)
{
    return vo_step_batch(c, left, right, ld, 1, out);
}

int vo_step_submit_dev(vo_ctx* c, const uint8_t* d_l, const uint8_t* d_r, int B)
{
    if (!c || !d_l || !d_r || B < 1 || B > c->max_batch) return fail(c, VO_ERR_ARG, "vo_step_submit_dev: bad arguments");
    BEGIN_CALL(c, false, true);
    // the first batch of a pipeline is ordered after earlier work on `stream`; later ones
    // overlap the previous batch's geometry (their inputs must be ready at the call)
    int rc = submit_batch(c, d_l, d_r, B, c->pending.empty());
    if (!c->prof.on) g_prof = nullptr;
    return rc;
}

int vo_step_collect(vo_ctx* c, vo_step_out* outs, int capacity, int* n)
{
    if (!c || !outs) return fail(c, VO_ERR_ARG, "vo_step_collect: bad arguments");
    hipSetDevice(c->device);
    int rc = collect_batch(c, outs, capacity, n);
    g_prof = nullptr;
    return rc;
}

int vo_steps_pending(const vo_ctx* c) { return c ? (int)c->pending.size() : 0; }

int vo_fetch_tracks(vo_ctx* c, int frame, float* old_l, float* cur_l, double* world, float* det, int capacity,
                    int* n_tracked, int* n_det)
{
    if (!c || capacity < 0) return fail(c, VO_ERR_ARG, "vo_fetch_tracks: bad arguments");
    if (c->last_step_set < 0 || frame < 0 || frame >= c->last_step_B)
        return fail(c, VO_ERR_STATE, "vo_fetch_tracks: frame %d not in the last collected batch", frame);
    for (const vo_ctx::Pending& q : c->pending)
        if (q.set == c->last_step_set)
            return fail(c, VO_ERR_STATE, "vo_fetch_tracks: the collected batch's buffer set is reused by a pending batch");
    hipSetDevice(c->device);
    SetRef S = set_ref(c, c->last_step_set);
    const int K = c->sb.kp_cap;
    int n = 0, nd = 0;
    HIPC(c, hipMemcpy(&n, S.gb->list_n + 4 * frame + 3, sizeof(int), hipMemcpyDeviceToHost));
    HIPC(c, hipMemcpy(&nd, S.sb->n_kp + 2 * frame, sizeof(int), hipMemcpyDeviceToHost));
    n = std::min(std::max(n, 0), K);
    nd = std::min(std::max(nd, 0), K);
    if (n_tracked) *n_tracked = n;
    if (n_det) *n_det = nd;
    const int m = std::min(n, capacity), md = std::min(nd, capacity);
    if (m > 0 && (old_l || cur_l || world)) {
        std::vector<float> op((size_t)m * 4);
        std::vector<double> ip((size_t)m * 2);
        HIPC(c, hipMemcpy(op.data(), S.gb->oldpos + (size_t)frame * K * 4, sizeof(float) * 4 * m, hipMemcpyDeviceToHost));
        HIPC(c, hipMemcpy(ip.data(), S.gb->imgpt + (size_t)frame * K * 2, sizeof(double) * 2 * m, hipMemcpyDeviceToHost));
        if (world) HIPC(c, hipMemcpy(world, S.gb->world + (size_t)frame * K * 3, sizeof(double) * 3 * m, hipMemcpyDeviceToHost));
        for (int k = 0; k < m; ++k) {
            if (old_l) { old_l[2 * k] = op[4 * k]; old_l[2 * k + 1] = op[4 * k + 1]; }
            if (cur_l) { cur_l[2 * k] = (float)ip[2 * k]; cur_l[2 * k + 1] = (float)ip[2 * k + 1]; }
        }
    }
    if (det && md > 0) {
        std::vector<vo_keypoint> kp(md);
        HIPC(c, hipMemcpy(kp.data(), S.sb->kp + (size_t)(2 * frame) * K, sizeof(vo_keypoint) * md, hipMemcpyDeviceToHost));
        for (int k = 0; k < md; ++k) { det[2 * k] = kp[k].x; det[2 * k + 1] = kp[k].y; }
    }
    return VO_OK;
}

int vo_get_landmarks(vo_ctx* c, double* out, int capacity, int* rows)
{
    if (!c) return VO_ERR_ARG;
    int r = (int)(c->landmarks.size() / 3);
    if (rows) *rows = r;
    if (out) memcpy(out, c->landmarks.data(), sizeof(double) * 3 * std::min(r, capacity));
    return r > capacity && out ? fail(c, VO_ERR_CAPACITY, "vo_get_landmarks: %d rows exceed capacity %d", r, capacity) : VO_OK;
}

int vo_set_landmark_frame(vo_ctx* c, int camera)
{
    if (!c || (camera != 0 && camera != 1)) return fail(c, VO_ERR_ARG, "vo_set_landmark_frame: mode must be 0 (world) or 1 (camera)");
    if (!c->pending.empty()) return fail(c, VO_ERR_STATE, "vo_set_landmark_frame: batches pending");
    c->lm_camera = camera;
    c->landmarks.clear();
    c->lm_n = 0;
    c->lm_frame_off.assign(1, 0);
    return VO_OK;
}

int vo_get_landmark_rows(vo_ctx* c, float* X, uint8_t* keep, int capacity, int* rows)
{
    if (!c || capacity < 0) return fail(c, VO_ERR_ARG, "vo_get_landmark_rows: bad arguments");
    if (!c->lm_camera) return fail(c, VO_ERR_STATE, "vo_get_landmark_rows: context keeps world rows (vo_set_landmark_frame(ctx, 1) first)");
    if (!c->pending.empty()) return fail(c, VO_ERR_STATE, "vo_get_landmark_rows: batches pending");
    if (c->lm_n > (size_t)INT_MAX)    // the device store is size_t; this API counts in int (vo_landmarks_world_dev: long)
        return fail(c, VO_ERR_CAPACITY, "vo_get_landmark_rows: %zu rows exceed INT_MAX (use vo_landmarks_world_dev)", c->lm_n);
    const int r = (int)c->lm_n;
    if (rows) *rows = r;
    const int m = std::min(r, capacity);
    if (m > 0 && (X || keep)) {
        hipSetDevice(c->device);
        HIPC(c, hipStreamSynchronize(c->stream));
        if (X) HIPC(c, hipMemcpy(X, c->d_lmX, sizeof(float) * 3 * m, hipMemcpyDeviceToHost));
        if (keep) HIPC(c, hipMemcpy(keep, c->d_lmkeep, m, hipMemcpyDeviceToHost));
    }
    return r > capacity && (X || keep) ? fail(c, VO_ERR_CAPACITY, "vo_get_landmark_rows: %d rows exceed capacity %d", r, capacity) : VO_OK;
}

int vo_landmarks_world_dev(vo_ctx* c, const double* poses, int n_frames, float* d_out, long capacity, long* rows)
{
    if (!c || n_frames < 0 || capacity < 0 || (n_frames > 0 && !poses))
        return fail(c, VO_ERR_ARG, "vo_landmarks_world_dev: bad arguments");
    if (!c->lm_camera) return fail(c, VO_ERR_STATE, "vo_landmarks_world_dev: context keeps world rows (vo_set_landmark_frame(ctx, 1) first)");
    if (!c->pending.empty()) return fail(c, VO_ERR_STATE, "vo_landmarks_world_dev: batches pending");
    const int nf = (int)c->lm_frame_off.size() - 1;
    if (n_frames != nf)
        return fail(c, VO_ERR_ARG, "vo_landmarks_world_dev: %d poses for %d collected frames", n_frames, nf);
    const long r = (long)c->lm_n;
    if (rows) *rows = r;
    if (r == 0) return VO_OK;
    if (!d_out) return VO_OK;
    if (r > capacity) return fail(c, VO_ERR_CAPACITY, "vo_landmarks_world_dev: %ld rows exceed capacity %ld", r, capacity);
    hipSetDevice(c->device);
    if (nf > c->lmw_cap) {
        hipFree(c->d_lmw_pose); hipFree(c->d_lmw_off);
        c->d_lmw_pose = nullptr; c->d_lmw_off = nullptr; c->lmw_cap = 0;
        const int cap = std::max(nf, 1024);
        HIPC(c, hipMalloc((void**)&c->d_lmw_pose, sizeof(double) * 16 * cap));
        HIPC(c, hipMalloc((void**)&c->d_lmw_off, sizeof(long long) * (cap + 1)));
        c->lmw_cap = cap;
    }
    HIPC(c, hipMemcpyAsync(c->d_lmw_pose, poses, sizeof(double) * 16 * nf, hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->d_lmw_off, c->lm_frame_off.data(), sizeof(long long) * (nf + 1), hipMemcpyHostToDevice,
                           c->stream));
    lm_world_launch(c->d_lmw_pose, c->d_lmw_off, nf, c->d_lmX, c->d_lmkeep, d_out, c->stream);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(c, VO_ERR_HIP, "launch: %s", hipGetErrorString(e));
    // d_out is read by the caller's streams (torch, RCCL) next: complete before returning
    HIPC(c, hipStreamSynchronize(c->stream));
    return VO_OK;
}

int vo_landmarks_to_world(const double pose[16], const float* X, const uint8_t* keep, int n, double* out)
{
    if (!pose || n < 0 || (n > 0 && (!X || !keep || !out))) return VO_ERR_ARG;
    for (int m = 0; m < n; ++m) {
        if (keep[m]) lm_world(pose, X + (size_t)m * 3, out + (size_t)m * 3);
        else out[3 * m] = out[3 * m + 1] = out[3 * m + 2] = 0.0;
    }
    return VO_OK;
}

int vo_chain_poses(const double* rel, const int32_t* status, int n, const double* pose0, double* out)
{
    if (n < 0 || (n > 0 && (!rel || !out))) return VO_ERR_ARG;
    double pose[16];
    memcpy(pose, pose0 ? pose0 : I4, sizeof(pose));
    for (int f = 0; f < n; ++f) {
        if (!status || status[f] == VO_OK) mat4_mul(pose, rel + (size_t)16 * f, pose);
        memcpy(out + (size_t)16 * f, pose, sizeof(pose));
    }
    return VO_OK;
}

int vo_landmarks_to_world_frames(const double* poses, const int32_t* rows_per_frame, int n_frames, const float* X,
                                 const uint8_t* keep, long n_rows, double* out)
{
    if (n_frames < 0 || n_rows < 0 || (n_frames > 0 && (!poses || !rows_per_frame))) return VO_ERR_ARG;
    long r = 0;
    for (int f = 0; f < n_frames; ++f) {
        const long k = rows_per_frame[f];
        if (k < 0 || r + k > n_rows) return VO_ERR_ARG;
        int rc = vo_landmarks_to_world(poses + (size_t)16 * f, X + 3 * r, keep + r, (int)k, out + 3 * r);
        if (rc) return rc;
        r += k;
    }
    return r == n_rows ? VO_OK : VO_ERR_ARG;
}

int vo_reset(vo_ctx* c)
{
    if (!c) return VO_ERR_ARG;
    hipSetDevice(c->device);
    // drops any pending asynchronous batches: wait for this context's streams only
    HIPC(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < vo_ctx::MAX_SUB; ++k) HIPC(c, hipStreamSynchronize(c->sub[k]));
    HIPC(c, hipStreamSynchronize(c->copy_stream));
    c->pending.clear();
    c->next_step_set = 0;
    c->next_slot = 0;
    for (void* p : c->lm_retired) hipFree(p);
    c->lm_retired.clear();
    c->last_step_set = -1;
    c->have_features = false;
    c->frame_index = 0;
    memcpy(c->pose, I4, sizeof(I4));
    c->landmarks.clear();
    c->lm_n = 0;
    c->lm_frame_off.assign(1, 0);
    HIPC(c, hipMemset(c->d_pair_n + c->max_batch, 0, sizeof(int)));
    HIPC(c, hipMemset(c->aux.pair_n + c->max_batch, 0, sizeof(int)));
    return VO_OK;
}

int vo_set_frame_index(vo_ctx* c, long frame_index)
{
    if (!c || frame_index < 0) return VO_ERR_ARG;
    c->frame_index = frame_index;
    return VO_OK;
}

// Standalone calls use frame slot 0 and the carry slots: they invalidate the
// loop state of vo_step (call vo_reset before stepping again).
static int upload_desc(vo_ctx* c, int slot, const uint8_t* d, int n)
{
    const int K = c->sb.kp_cap;
    if (n) HIPC(c, hipMemcpyAsync(c->sb.desc + (size_t)slot * K * VO_DESC_LEN, d, (size_t)n * VO_DESC_LEN, hipMemcpyHostToDevice, c->stream));
    desc_meta_launch(c->sb.desc + (size_t)slot * K * VO_DESC_LEN, c->sb.meta + (size_t)slot * K, n, c->stream);
    HIPC(c, hipMemcpyAsync(c->sb.n_kp + slot, &n, sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));   // &n is a stack value
    return VO_OK;
}

int vo_track(vo_ctx* c, const uint8_t* old_l, const uint8_t* old_r, int n_old, const uint8_t* cur_l, int n_cl,
             const uint8_t* cur_r, int n_cr, uint32_t* idx_out, int capacity, int* K_out)
{
    if (!c || n_old < 0 || n_cl < 0 || n_cr < 0) return fail(c, VO_ERR_ARG, "vo_track: bad arguments");
    const int K = c->sb.kp_cap, M = c->max_batch;
    if (n_old > K || n_cl > K || n_cr > K) return fail(c, VO_ERR_CAPACITY, "vo_track: more rows than max_keypoints");
    BEGIN_CALL(c);
    c->have_features = false;
    c->last_set = 0;                                   // set 0's descriptor slots are overwritten
    int rc;
    if ((rc = upload_desc(c, 2 * M, old_l, n_old))) return rc;
    if ((rc = upload_desc(c, 2 * M + 1, old_r, n_old))) return rc;
    if ((rc = upload_desc(c, 0, cur_l, n_cl))) return rc;
    if ((rc = upload_desc(c, 1, cur_r, n_cr))) return rc;
    std::vector<int> iota(std::max(n_old, 1));
    for (int k = 0; k < n_old; ++k) iota[k] = k;
    if (n_old) {
        HIPC(c, hipMemcpy(c->d_pair_i + (size_t)M * K, iota.data(), sizeof(int) * n_old, hipMemcpyHostToDevice));
        HIPC(c, hipMemcpy(c->d_pair_j + (size_t)M * K, iota.data(), sizeof(int) * n_old, hipMemcpyHostToDevice));
    }
    HIPC(c, hipMemcpy(c->d_pair_n + M, &n_old, sizeof(int), hipMemcpyHostToDevice));
    StepArgs a = step_args(c, 1);
    track_enqueue(c->gb, c->mb, c->d_jobs + job_track(c, 0, 0), a, c->mp, c->stream);
    int n = 0;
    HIPC(c, hipMemcpyAsync(&n, c->gb.list_n + 3, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    rc = finish(c);
    if (rc) return rc;
    if (K_out) *K_out = n;
    const int m = std::min(n, capacity);
    if (m > 0 && idx_out) {
        std::vector<int> ol(m), cl(m), cr(m);
        HIPC(c, hipMemcpy(ol.data(), track_list(c->gb, 0, TL_OLF), sizeof(int) * m, hipMemcpyDeviceToHost));
        HIPC(c, hipMemcpy(cl.data(), track_list(c->gb, 0, TL_CLF), sizeof(int) * m, hipMemcpyDeviceToHost));
        HIPC(c, hipMemcpy(cr.data(), track_list(c->gb, 0, TL_CRF), sizeof(int) * m, hipMemcpyDeviceToHost));
        for (int k = 0; k < m; ++k) {
            idx_out[3 * k] = (uint32_t)ol[k] + 1;
            idx_out[3 * k + 1] = (uint32_t)cl[k] + 1;
            idx_out[3 * k + 2] = (uint32_t)cr[k] + 1;
        }
    }
    if (n > capacity) return fail(c, VO_ERR_CAPACITY, "vo_track: %d rows exceed capacity %d", n, capacity);
    return VO_OK;
}

int vo_triangulate(vo_ctx* c, const float* x1, const float* x2, int n, const double P1[12], const double P2[12], double* X)
{
    if (!c || n < 0 || (n && (!x1 || !x2 || !X)) || !P1 || !P2) return fail(c, VO_ERR_ARG, "vo_triangulate: bad arguments");
    BEGIN_CALL(c);
    const vo_calib cal = calib_of(P1, P2, nullptr);
    const int K = c->sb.kp_cap;
    std::vector<float> q((size_t)std::min(n, K) * 4 + 4);
    for (int b = 0; b < n; b += K) {
        const int m = std::min(K, n - b);
        for (int k = 0; k < m; ++k) {
            q[4 * k] = x1[2 * (b + k)]; q[4 * k + 1] = x1[2 * (b + k) + 1];
            q[4 * k + 2] = x2[2 * (b + k)]; q[4 * k + 3] = x2[2 * (b + k) + 1];
        }
        HIPC(c, hipMemcpyAsync(c->gb.oldpos, q.data(), sizeof(float) * 4 * m, hipMemcpyHostToDevice, c->stream));
        triangulate_launch(c->gb.oldpos, m, cal, c->gb.world, c->stream);
        HIPC(c, hipMemcpyAsync(X + 3 * (size_t)b, c->gb.world, sizeof(double) * 3 * m, hipMemcpyDeviceToHost, c->stream));
        int rc = finish(c);
        if (rc) return rc;
        g_prof = c->prof.on ? &c->prof : nullptr;
    }
    g_prof = nullptr;
    return VO_OK;
}

int vo_estworldpose(vo_ctx* c, const double* img, const double* world, int n, const double K9[9],
                    const vo_ransac_params* params, uint32_t frame_key, double T[16], uint8_t* inliers, int* n_inliers)
{
    if (!c || n < 0 || (n && (!img || !world)) || !K9 || !T) return fail(c, VO_ERR_ARG, "vo_estworldpose: bad arguments");
    if (n > c->sb.kp_cap) return fail(c, VO_ERR_CAPACITY, "vo_estworldpose: %d points exceed max_keypoints", n);
    const vo_ransac_params rp = params ? *params : c->rp;
    if (rp.max_num_trials > c->gb.n_hyp)
        return fail(c, VO_ERR_ARG, "vo_estworldpose: MaxNumTrials %d exceeds the context's %d hypothesis slots (vo_create ransac.max_num_trials)",
                    rp.max_num_trials, c->gb.n_hyp);
    if (n_inliers) *n_inliers = 0;
    if (n < 4) return fail(c, VO_ERR_TOO_FEW_POINTS, "estworldpose: need at least 4 points, got %d", n);
    BEGIN_CALL(c);
    c->have_features = false;
    HIPC(c, hipMemcpyAsync(c->gb.imgpt, img, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->gb.world, world, sizeof(double) * 3 * n, hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->d_fn, &n, sizeof(int), hipMemcpyHostToDevice, c->stream));
    estworldpose_launch(c->gb, c->gb.imgpt, c->gb.world, c->d_fn, K9, rp, frame_key, c->stream);
    FrameGeom g;
    HIPC(c, hipMemcpyAsync(&g, c->gb.fg, sizeof(g), hipMemcpyDeviceToHost, c->stream));
    if (inliers) HIPC(c, hipMemcpyAsync(inliers, c->gb.inliers, n, hipMemcpyDeviceToHost, c->stream));
    int rc = finish(c);
    if (rc) return rc;
    memcpy(T, g.T, sizeof(g.T));
    if (n_inliers) *n_inliers = g.n_inliers;
    if (g.status == VO_ERR_NO_CONSENSUS) return fail(c, g.status, "estworldpose: no consensus (MSAC found no model with >= 4 inliers)");
    if (g.status != VO_OK) return fail(c, g.status, "estworldpose failed (%d)", g.status);
    return VO_OK;
}

int vo_landmarks(vo_ctx* c, const float* l_pos, const float* r_pos, int S, const float* old_l, const float* old_r, int Kn,
                 const double pose[16], double* out, int capacity, int* rows_out)
{
    if (!c || S < 0 || Kn < 0 || !pose || (S && (!l_pos || !r_pos)) || (Kn && (!old_l || !old_r)))
        return fail(c, VO_ERR_ARG, "vo_landmarks: bad arguments");
    if (!c->has_calib) return fail(c, VO_ERR_STATE, "vo_landmarks: no calibration");
    const int K = c->sb.kp_cap;
    if (S > K || Kn > K) return fail(c, VO_ERR_CAPACITY, "vo_landmarks: more rows than max_keypoints");
    BEGIN_CALL(c);
    c->have_features = false;
    std::vector<float> sp((size_t)S * 4 + 4), op((size_t)Kn * 4 + 4);
    for (int j = 0; j < S; ++j) { sp[4 * j] = l_pos[2 * j]; sp[4 * j + 1] = l_pos[2 * j + 1]; sp[4 * j + 2] = r_pos[2 * j]; sp[4 * j + 3] = r_pos[2 * j + 1]; }
    for (int k = 0; k < Kn; ++k) { op[4 * k] = old_l[2 * k]; op[4 * k + 1] = old_l[2 * k + 1]; op[4 * k + 2] = old_r[2 * k]; op[4 * k + 3] = old_r[2 * k + 1]; }
    int cnt[2] = {S, Kn};
    HIPC(c, hipMemcpyAsync(c->gb.spos, sp.data(), sizeof(float) * 4 * S, hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->gb.oldpos, op.data(), sizeof(float) * 4 * Kn, hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->gb.s_n, &cnt[0], sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->d_fn, &cnt[1], sizeof(int), hipMemcpyHostToDevice, c->stream));
    landmarks_launch(c->gb, c->d_fn, c->calib, c->stream);
    int rows = 0;
    HIPC(c, hipMemcpyAsync(&rows, c->gb.lm_rows, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    int rc = finish(c);
    if (rc) return rc;
    std::vector<float> X((size_t)rows * 3);
    std::vector<uint8_t> keep(rows);
    HIPC(c, hipMemcpy(X.data(), c->gb.lm_X, sizeof(float) * 3 * rows, hipMemcpyDeviceToHost));
    HIPC(c, hipMemcpy(keep.data(), c->gb.lm_keep, rows, hipMemcpyDeviceToHost));
    if (rows_out) *rows_out = rows;
    if (out) {
        for (int m = 0; m < rows && m < capacity; ++m) {
            out[3 * m] = out[3 * m + 1] = out[3 * m + 2] = 0.0;
            if (keep[m]) lm_world(pose, &X[(size_t)m * 3], out + 3 * m);
        }
    }
    if (rows > capacity) return fail(c, VO_ERR_CAPACITY, "vo_landmarks: %d rows exceed capacity %d", rows, capacity);
    return VO_OK;
}

}  // extern "C"

#if VO_EXPERIMENTAL
// ---------------------------------------------------------------------------
// Test build only (libvo_exp.so, make exp): selects the experimental kernels that the product
// library does not contain -- the fused octave (octave.hip) and the eager MSAC kernels -- so
// their parity tests can run them against the default path.  Process-wide; read at enqueue.
// ---------------------------------------------------------------------------
namespace vo {
int g_exp_fused_octave = 0, g_exp_msac_eager = 0;
}
extern "C" int vo_exp_set(int fused_octave, int msac_eager)
{
    vo::g_exp_fused_octave = fused_octave ? 1 : 0;
    vo::g_exp_msac_eager = msac_eager ? 1 : 0;
    return VO_OK;
}
#endif
