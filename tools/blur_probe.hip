// blur_probe.hip — isolates where the level blur's time goes (instrumentation, not libvo).
// Times k_blur_stream<r, TAG> on 64 octave-0 planes (2484 x 750, pitch 2560) for the
// production variant and the probe variants (no row pass / no column pass / neither /
// cached stores), so the HBM, VALU and LDS shares can be separated.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -I csrc tools/blur_probe.hip
#include "../r7020e-visual-odometry_amd/csrc/sift.hip"
#include <cstdio>

using namespace vo;

// the profiler hooks sift.hip's host code references (unused here)
namespace vo {
Profiler* g_prof = nullptr;
void Profiler::begin(const char*, hipStream_t) {}
void Profiler::end(hipStream_t) {}
void Profiler::collect() {}
void Profiler::reset_totals() {}
Profiler::~Profiler() {}
}

// reference streaming pattern: each wave copies its 256-column strip of a band row by
// row (P rows of loads in flight, non-temporal 16-B stores) -- the practical floor for
// 1 plane in + 1 plane out in this access order
template <int P>
__global__ __launch_bounds__(64) void k_copy_strip(const float* __restrict__ a, float* __restrict__ b, int pitch, int R,
                                                   size_t plane, int n_strips, int n_bands, int TH)
{
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = bid % n_strips, tb = bid / n_strips, band = tb % n_bands, img = tb / n_bands;
    const int x0 = strip * 256, y0 = min(band * TH, R - TH);
    const int xl = x0 + 4 * (int)threadIdx.x;
    const float* ap = a + img * plane;
    float* bp = b + img * plane;
    f4 pf[P];
#pragma unroll
    for (int u = 0; u < P; ++u) pf[u] = *reinterpret_cast<const f4*>(ap + (size_t)(y0 + u) * pitch + xl);
    for (int k0 = 0; k0 < TH; k0 += P) {
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int k = k0 + u;
            const f4 v = pf[u];
            pf[u] = *reinterpret_cast<const f4*>(ap + (size_t)(y0 + min(k + P, TH - 1)) * pitch + xl);
            __builtin_nontemporal_store(v * 2.0f, reinterpret_cast<f4*>(bp + (size_t)(y0 + k) * pitch + xl));
        }
    }
}

template <int RAD, int TAG, int CPL = 4>
static float run(const float* src, float* dst, size_t plane, int pitch, int R, int C, int n_img, int TH, const Kern& K)
{
    const int n_strips = (C + 64 * CPL - 1) / (64 * CPL), n_bands = (R + TH - 1) / TH;
    const int blocks = n_strips * n_bands * n_img;
    ImageSrc isrc{};
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int w = 0; w < 2; ++w)
        hipLaunchKernelGGL((k_blur_stream<RAD, TAG, CPL>), dim3(blocks), dim3(64), 0, 0, src, plane, plane, pitch, R, C, dst, K,
                           n_strips, n_bands, TH, isrc, 0, 0);
    hipEventRecord(a);
    const int it = 10;
    for (int i = 0; i < it; ++i)
        hipLaunchKernelGGL((k_blur_stream<RAD, TAG, CPL>), dim3(blocks), dim3(64), 0, 0, src, plane, plane, pitch, R, C, dst, K,
                           n_strips, n_bands, TH, isrc, 0, 0);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return 1000.0f * ms / it;
}

template <int RAD>
static void probe(const float* src, float* dst, size_t plane, int pitch, int R, int C, int n)
{
    Kern K{};
    K.r = RAD;
    for (int j = 0; j <= RAD; ++j) K.k[j] = 1.0f / (2 * RAD + 1);
    const double mb = 8.0 * (double)R * C * n / 1e6;     // algorithmic: 4 B in + 4 B out per px
    const int TH = getenv("TH") ? atoi(getenv("TH")) : 48;
    float t0 = run<RAD, 0>(src, dst, plane, pitch, R, C, n, TH, K);
    float t8 = run<RAD, 8>(src, dst, plane, pitch, R, C, n, TH, K);
    float t16 = run<RAD, 16>(src, dst, plane, pitch, R, C, n, TH, K);
    float t24 = run<RAD, 24>(src, dst, plane, pitch, R, C, n, TH, K);
    float t2 = run<RAD, 2>(src, dst, plane, pitch, R, C, n, TH, K);
    float t56 = run<RAD, 56>(src, dst, plane, pitch, R, C, n, TH, K);
    float t120 = run<RAD, 120>(src, dst, plane, pitch, R, C, n, TH, K);
    float c0 = run<RAD, 0, 2>(src, dst, plane, pitch, R, C, n, TH, K);
    float c24 = run<RAD, 24, 2>(src, dst, plane, pitch, R, C, n, TH, K);
    float c56 = run<RAD, 56, 2>(src, dst, plane, pitch, R, C, n, TH, K);
    printf("r=%2d  full %6.1f us (%5.0f GB/s) | no-row %6.1f | no-col %6.1f | neither %6.1f | cached %6.1f | "
           "no compute+no LDS %6.1f | +no halo %6.1f\n", RAD, t0, mb / t0 * 1e3, t8, t16, t24, t2, t56, t120);
    printf("      CPL=2 full %6.1f us (%5.0f GB/s) | neither %6.1f | no compute+no LDS %6.1f\n", c0, mb / c0 * 1e3, c24, c56);
}

static void copy_ref(const float* src, float* dst, size_t plane, int pitch, int R, int C, int n)
{
    const int TH = 48, n_strips = (C + 255) / 256, n_bands = (R + TH - 1) / TH;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int w = 0; w < 2; ++w)
        hipLaunchKernelGGL(k_copy_strip<4>, dim3(n_strips * n_bands * n), dim3(64), 0, 0, src, dst, pitch, R, plane, n_strips, n_bands, TH);
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i)
        hipLaunchKernelGGL(k_copy_strip<4>, dim3(n_strips * n_bands * n), dim3(64), 0, 0, src, dst, pitch, R, plane, n_strips, n_bands, TH);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double us = 100.0 * ms, mb = 8.0 * (double)R * C * n / 1e6;
    printf("copy-strip reference (1 in + 1 out, TH=48, P=4): %6.1f us (%5.0f GB/s algorithmic)\n", us, mb / us * 1e3);
}

int main()
{
    const int R = getenv("ROWS") ? atoi(getenv("ROWS")) : 750, C = getenv("COLS") ? atoi(getenv("COLS")) : 2484, n = 64;
    const int pitch = getenv("PITCH") ? atoi(getenv("PITCH")) : (C + 255) / 256 * 256;
    printf("pitch %d\n", pitch);
    const size_t plane = (size_t)R * pitch;
    float *src, *dst;
    hipMalloc(&src, sizeof(float) * plane * n);
    hipMalloc(&dst, sizeof(float) * plane * n);
    hipMemset(src, 0, sizeof(float) * plane * n);
    printf("%d x %d, %d images\n", R, C, n);
    copy_ref(src, dst, plane, pitch, R, C, n);
    probe<5>(src, dst, plane, pitch, R, C, n);
    probe<8>(src, dst, plane, pitch, R, C, n);
    probe<13>(src, dst, plane, pitch, R, C, n);
    return 0;
}
