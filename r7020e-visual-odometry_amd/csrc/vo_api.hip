// vo_api.hip — the C-ABI of libvo (include/vo.h): context, staging and the
// orchestration of the per-frame pipeline on one HIP stream.
#include "vo_internal.h"
#include "vo_geom.h"
#include <cstdio>
#include <cstring>
#include <cstdarg>
#include <string>
#include <vector>
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
    Pyramid py;
    Pyramid* d_py = nullptr;
    SiftBuffers sb;                  // 2*max_batch + 2 image slots (last 2 = carried frame)
    MatchBuffers mb;
    MatchJob* d_jobs = nullptr;      // job tables (see JOB_* offsets)
    int* d_pair_i = nullptr;         // stereo pairs per frame slot [slots][kp_cap]
    int* d_pair_j = nullptr;
    int* d_pair_n = nullptr;         // [slots]
    uint8_t* d_img = nullptr;        // image staging [2*max_batch][rows*cols]
    // vo_match staging
    uint8_t* d_fd[2] = {nullptr, nullptr};
    DescMeta* d_fm[2] = {nullptr, nullptr};
    int* d_fn = nullptr;             // [2]
    int* d_mi = nullptr; int* d_mj = nullptr; int* d_mn = nullptr;
    GeomBuffers gb;
    std::string err;
    Profiler prof;
    int last_B = 0;
    // loop state (vo_step)
    long frame_index = 0;
    bool have_features = false;
    double pose[16];
    std::vector<double> landmarks;
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
    p->max_num_trials = 2048; p->confidence = 99.0; p->max_reprojection_error = 1.0; p->seed = 0x5EED;
}

const char* vo_last_error(const vo_ctx* c) { return c ? c->err.c_str() : g_create_err.c_str(); }

void* vo_stream(vo_ctx* c) { return c ? (void*)c->stream : nullptr; }

// job table layout: [0, B) stereo; [B, B + 4*B) tracking steps; last: vo_match
static int job_stereo(const vo_ctx*, int f) { return f; }
static int job_track(const vo_ctx* c, int step, int f) { return c->max_batch + step * c->max_batch + f; }
static int job_single(const vo_ctx* c) { return 5 * c->max_batch; }

static void destroy_buffers(vo_ctx* c)
{
    sift_free(c->sb);
    match_free(c->mb);
    geom_free(c->gb);
    hipFree(c->d_py); hipFree(c->d_jobs); hipFree(c->d_pair_i); hipFree(c->d_pair_j); hipFree(c->d_pair_n);
    hipFree(c->d_img); hipFree(c->d_fd[0]); hipFree(c->d_fd[1]); hipFree(c->d_fm[0]); hipFree(c->d_fm[1]);
    hipFree(c->d_fn); hipFree(c->d_mi); hipFree(c->d_mj); hipFree(c->d_mn);
}

vo_ctx* vo_create(int device, int rows, int cols, int max_batch, const vo_calib* calib, const vo_sift_params* sift,
                  const vo_match_params* match, const vo_ransac_params* ransac)
{
    if (rows < 16 || cols < 16 || rows > 2048 || cols > 2048 || max_batch < 1 || max_batch > 64) {
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
    if (c->sp.n_octave_layers < 1 || c->sp.n_octave_layers > 5 || c->sp.max_keypoints < 16) {
        fail(nullptr, VO_ERR_ARG, "vo_create: bad sift params");
        delete c;
        return nullptr;
    }
    auto bail = [&](const char* what, hipError_t e) -> vo_ctx* {
        fail(nullptr, VO_ERR_HIP, "vo_create: %s: %s", what, hipGetErrorString(e));
        destroy_buffers(c);
        if (c->stream) hipStreamDestroy(c->stream);
        delete c;
        return nullptr;
    };
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return bail("stream", e);
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
    }
    if ((e = hipMalloc((void**)&c->d_fn, sizeof(int) * 2)) != hipSuccess) return bail("staging", e);
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
    return c;
}

void vo_destroy(vo_ctx* c)
{
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    destroy_buffers(c);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
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

int vo_kernel_times(vo_ctx* c, const char** names, double* ms, int* calls, int capacity, int* n)
{
    if (!c) return VO_ERR_ARG;
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
    if (e != hipSuccess) return fail(c, VO_ERR_HIP, "stream sync: %s", hipGetErrorString(e));
    e = hipGetLastError();
    if (e != hipSuccess) return fail(c, VO_ERR_HIP, "launch: %s", hipGetErrorString(e));
    if (c->prof.on) c->prof.collect();
    g_prof = nullptr;
    return VO_OK;
}

static void begin_call(vo_ctx* c)
{
    hipSetDevice(c->device);
    g_prof = c->prof.on ? &c->prof : nullptr;
}

int vo_sift(vo_ctx* c, const uint8_t* img, int rows, int cols, int ld, vo_keypoint* kps, uint8_t* desc, int capacity,
            int* n_out)
{
    if (!c || !img || rows != c->rows || cols != c->cols || ld < cols) return fail(c, VO_ERR_ARG, "vo_sift: bad arguments");
    begin_call(c);
    HIPC(c, hipMemcpy2DAsync(c->d_img, cols, img, ld, cols, rows, hipMemcpyHostToDevice, c->stream));
    ImageSrc src{c->d_img, c->d_img, (size_t)rows * cols, cols, 0};
    sift_enqueue(c->py, c->sb, src, 1, c->sp, c->stream, c->d_py);
    int n = 0;
    HIPC(c, hipMemcpyAsync(&n, c->sb.n_kp, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    int rc = finish(c);
    if (rc) return rc;
    if (n_out) *n_out = n;
    int m = std::min(std::min(n, c->sb.kp_cap), capacity);
    if (m > 0) {
        if (kps) HIPC(c, hipMemcpy(kps, c->sb.kp, sizeof(vo_keypoint) * m, hipMemcpyDeviceToHost));
        if (desc) HIPC(c, hipMemcpy(desc, c->sb.desc, (size_t)m * VO_DESC_LEN, hipMemcpyDeviceToHost));
    }
    if (n > c->sb.kp_cap) return fail(c, VO_ERR_CAPACITY, "vo_sift: %d keypoints exceed max_keypoints %d", n, c->sb.kp_cap);
    if (n > capacity) return fail(c, VO_ERR_CAPACITY, "vo_sift: %d keypoints exceed capacity %d", n, capacity);
    return VO_OK;
}

int vo_match(vo_ctx* c, const uint8_t* F1, int n1, const uint8_t* F2, int n2, uint32_t* pairs, int capacity, int* n_pairs)
{
    if (!c || n1 < 0 || n2 < 0 || (n1 && !F1) || (n2 && !F2)) return fail(c, VO_ERR_ARG, "vo_match: bad arguments");
    if (n1 > c->sb.kp_cap || n2 > c->sb.kp_cap) return fail(c, VO_ERR_CAPACITY, "vo_match: more rows than max_keypoints");
    begin_call(c);
    int nn[2] = {n1, n2};
    if (n1) HIPC(c, hipMemcpyAsync(c->d_fd[0], F1, (size_t)n1 * VO_DESC_LEN, hipMemcpyHostToDevice, c->stream));
    if (n2) HIPC(c, hipMemcpyAsync(c->d_fd[1], F2, (size_t)n2 * VO_DESC_LEN, hipMemcpyHostToDevice, c->stream));
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
    if (P > capacity) return fail(c, VO_ERR_CAPACITY, "vo_match: %d pairs exceed capacity %d", P, capacity);
    return VO_OK;
}

// SIFT + stereo match on B frames already in device memory.
static int enqueue_sift_stereo(vo_ctx* c, const uint8_t* d_l, const uint8_t* d_r, int B)
{
    ImageSrc src{d_l, d_r, (size_t)c->rows * c->cols, c->cols, 0};
    sift_enqueue(c->py, c->sb, src, 2 * B, c->sp, c->stream, c->d_py);
    match_launch(c->mb, c->d_jobs + job_stereo(c, 0), B, c->mp, c->stream);
    return VO_OK;
}

int vo_sift_match_batch_dev(vo_ctx* c, const uint8_t* d_lefts, const uint8_t* d_rights, int B, vo_pair_stats* stats)
{
    if (!c || !d_lefts || !d_rights || B < 1 || B > c->max_batch) return fail(c, VO_ERR_ARG, "vo_sift_match_batch_dev: bad arguments");
    begin_call(c);
    enqueue_sift_stereo(c, d_lefts, d_rights, B);
    c->last_B = B;
    if (!stats && !c->prof.on) {
        g_prof = nullptr;
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return fail(c, VO_ERR_HIP, "launch: %s", hipGetErrorString(e));
        return VO_OK;
    }
    std::vector<int> nk(2 * B), np(B);
    HIPC(c, hipMemcpyAsync(nk.data(), c->sb.n_kp, sizeof(int) * 2 * B, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemcpyAsync(np.data(), c->d_pair_n, sizeof(int) * B, hipMemcpyDeviceToHost, c->stream));
    int rc = finish(c);
    if (rc) return rc;
    if (stats) {
        for (int f = 0; f < B; ++f) {
            stats[f].n_left = nk[2 * f]; stats[f].n_right = nk[2 * f + 1]; stats[f].n_stereo = np[f];
            stats[f].flags = (nk[2 * f] > c->sb.kp_cap || nk[2 * f + 1] > c->sb.kp_cap) ? 1 : 0;
        }
    }
    return VO_OK;
}

int vo_fetch_keypoints(vo_ctx* c, int image, vo_keypoint* kps, uint8_t* desc, int capacity, int* n)
{
    if (!c || image < 0 || image >= c->sb.n_img) return fail(c, VO_ERR_ARG, "vo_fetch_keypoints: bad image");
    hipSetDevice(c->device);
    HIPC(c, hipStreamSynchronize(c->stream));
    int cnt = 0;
    HIPC(c, hipMemcpy(&cnt, c->sb.n_kp + image, sizeof(int), hipMemcpyDeviceToHost));
    if (n) *n = cnt;
    int m = std::min(std::min(cnt, c->sb.kp_cap), capacity);
    if (m > 0) {
        if (kps) HIPC(c, hipMemcpy(kps, c->sb.kp + (size_t)image * c->sb.kp_cap, sizeof(vo_keypoint) * m, hipMemcpyDeviceToHost));
        if (desc) HIPC(c, hipMemcpy(desc, c->sb.desc + (size_t)image * c->sb.kp_cap * VO_DESC_LEN, (size_t)m * VO_DESC_LEN, hipMemcpyDeviceToHost));
    }
    return VO_OK;
}

int vo_fetch_stereo_pairs(vo_ctx* c, int frame, uint32_t* pairs, int capacity, int* n)
{
    if (!c || frame < 0 || frame >= c->max_batch) return fail(c, VO_ERR_ARG, "vo_fetch_stereo_pairs: bad frame");
    hipSetDevice(c->device);
    HIPC(c, hipStreamSynchronize(c->stream));
    int P = 0;
    HIPC(c, hipMemcpy(&P, c->d_pair_n + frame, sizeof(int), hipMemcpyDeviceToHost));
    if (n) *n = P;
    int m = std::min(P, capacity);
    if (m > 0 && pairs) {
        std::vector<int> ii(m), jj(m);
        HIPC(c, hipMemcpy(ii.data(), c->d_pair_i + (size_t)frame * c->sb.kp_cap, sizeof(int) * m, hipMemcpyDeviceToHost));
        HIPC(c, hipMemcpy(jj.data(), c->d_pair_j + (size_t)frame * c->sb.kp_cap, sizeof(int) * m, hipMemcpyDeviceToHost));
        for (int k = 0; k < m; ++k) { pairs[2 * k] = (uint32_t)ii[k] + 1; pairs[2 * k + 1] = (uint32_t)jj[k] + 1; }
    }
    return VO_OK;
}

}  // extern "C"

// ---- stage-2 entry points (tracking / geometry / loop) --------------------
extern "C" {
int vo_track(vo_ctx* c, const uint8_t*, const uint8_t*, int, const uint8_t*, int, const uint8_t*, int, uint32_t*, int, int*)
{ return fail(c, VO_ERR_STATE, "vo_track: not built yet"); }
int vo_triangulate(vo_ctx* c, const float*, const float*, int, const double*, const double*, double*)
{ return fail(c, VO_ERR_STATE, "vo_triangulate: not built yet"); }
int vo_estworldpose(vo_ctx* c, const double*, const double*, int, const double*, const vo_ransac_params*, uint32_t, double*,
                    uint8_t*, int*)
{ return fail(c, VO_ERR_STATE, "vo_estworldpose: not built yet"); }
int vo_landmarks(vo_ctx* c, const float*, const float*, int, const float*, const float*, int, const double*, double*, int, int*)
{ return fail(c, VO_ERR_STATE, "vo_landmarks: not built yet"); }
int vo_step(vo_ctx* c, const uint8_t*, const uint8_t*, int, vo_step_out*) { return fail(c, VO_ERR_STATE, "vo_step: not built yet"); }
int vo_step_batch(vo_ctx* c, const uint8_t*, const uint8_t*, int, int, vo_step_out*) { return fail(c, VO_ERR_STATE, "not built yet"); }
int vo_step_batch_dev(vo_ctx* c, const uint8_t*, const uint8_t*, int, vo_step_out*) { return fail(c, VO_ERR_STATE, "not built yet"); }
int vo_get_landmarks(vo_ctx* c, double*, int, int*) { return fail(c, VO_ERR_STATE, "not built yet"); }
int vo_reset(vo_ctx* c) { return fail(c, VO_ERR_STATE, "not built yet"); }
}
