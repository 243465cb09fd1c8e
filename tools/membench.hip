// membench.hip — HBM access-pattern probe for the level-blur design (not part of libvo).
// Each pattern reads one fp32 plane and writes two (the G_i / D_{i-1} traffic of one
// blur level), 32 images of 2496 x 750 floats.  Prints GB/s per pattern.
//   linear : each wave streams contiguous 1-KB chunks, grid-stride
//   strip  : each wave owns a 256-column strip of a TH-row band and walks its rows
//            (the k_blur_stream order), P rows of loads in flight
// Build: hipcc --offload-arch=gfx950 -O3 -o membench membench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_linear(const f4* __restrict__ a, f4* __restrict__ b, f4* __restrict__ c, size_t n4)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        f4 v = a[i];
        b[i] = v * 2.0f;
        c[i] = v - 1.0f;
    }
}

template <int P, int NT, int LDSKB>
__global__ __launch_bounds__(64) void k_strip(const float* __restrict__ a, float* __restrict__ b, float* __restrict__ c,
                                              int pitch, int R, int C, size_t plane, int n_strips, int n_bands, int TH)
{
    __shared__ float occ_limit[LDSKB * 256 + 1];           // caps waves/CU at 160/LDSKB
    if (threadIdx.x == 1000) occ_limit[TH] = 0.0f;
    if (LDSKB && threadIdx.x == 999) a = (const float*)&occ_limit[0];
    const int bid = blockIdx.x;
    const int strip = bid % n_strips, tb = bid / n_strips, band = tb % n_bands, img = tb / n_bands;
    const int x0 = strip * 256, y0 = min(band * TH, R - TH);
    const int xl = min(x0 + 4 * (int)threadIdx.x, C - 4);
    const float* ap = a + img * plane;
    float* bp = b + img * plane;
    float* cp = c + img * plane;
    f4 pf[P];
#pragma unroll
    for (int u = 0; u < P; ++u) pf[u] = *reinterpret_cast<const f4*>(ap + (size_t)(y0 + u) * pitch + xl);
    for (int k0 = 0; k0 < TH; k0 += P) {
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int k = k0 + u;
            const f4 v = pf[u];
            pf[u] = *reinterpret_cast<const f4*>(ap + (size_t)(y0 + min(k + P, TH - 1)) * pitch + xl);
            if (NT) {
                __builtin_nontemporal_store(v * 2.0f, reinterpret_cast<f4*>(bp + (size_t)(y0 + k) * pitch + xl));
                __builtin_nontemporal_store(v - 1.0f, reinterpret_cast<f4*>(cp + (size_t)(y0 + k) * pitch + xl));
            } else {
                *reinterpret_cast<f4*>(bp + (size_t)(y0 + k) * pitch + xl) = v * 2.0f;
                *reinterpret_cast<f4*>(cp + (size_t)(y0 + k) * pitch + xl) = v - 1.0f;
            }
        }
    }
}

// read-only and write-only references
__global__ __launch_bounds__(256) void k_read(const f4* __restrict__ a, f4* __restrict__ out, size_t n4)
{
    f4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) acc += a[i];
    if (acc.x == 1234.5f) out[0] = acc;
}
__global__ __launch_bounds__(256) void k_write(f4* __restrict__ b, size_t n4)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        b[i] = f4{1.0f, 2.0f, 3.0f, (float)i};
}

int main()
{
    const int R = 750, C = 2484, pitch = 2496, NI = 32;
    const size_t plane = (size_t)R * pitch, n = plane * NI, n4 = n / 4;
    float *a, *b, *c;
    hipMalloc(&a, n * 4); hipMalloc(&b, n * 4); hipMalloc(&c, n * 4);
    hipMemset(a, 0, n * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(e0);
        const int it = 10;
        for (int i = 0; i < it; ++i) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s %8.1f us  %7.0f GB/s\n", name, 1000.0 * ms / it, bytes / (ms / it * 1e-3) / 1e9);
    };
    const double b3 = 3.0 * n * 4;
    for (int g : {1024, 2048, 4096, 8192})
        timeit((std::string("linear grid=") + std::to_string(g)).c_str(), b3,
               [&] { k_linear<<<g, 256>>>((const f4*)a, (f4*)b, (f4*)c, n4); });
    timeit("read", 1.0 * n * 4, [&] { k_read<<<4096, 256>>>((const f4*)a, (f4*)b, n4); });
    timeit("write", 1.0 * n * 4, [&] { k_write<<<4096, 256>>>((f4*)b, n4); });
    const int n_strips = (C + 255) / 256;
    for (int TH : {48, 96, 192}) {
        const int n_bands = (R + TH - 1) / TH, blocks = n_strips * n_bands * NI;
        char nm[64];
        snprintf(nm, sizeof nm, "strip TH=%d P=4", TH);
        timeit(nm, b3, [&] { k_strip<4, 0, 0><<<blocks, 64>>>(a, b, c, pitch, R, C, plane, n_strips, n_bands, TH); });
        snprintf(nm, sizeof nm, "strip TH=%d P=8", TH);
        timeit(nm, b3, [&] { k_strip<8, 0, 0><<<blocks, 64>>>(a, b, c, pitch, R, C, plane, n_strips, n_bands, TH); });
        snprintf(nm, sizeof nm, "strip TH=%d P=8 nt", TH);
        timeit(nm, b3, [&] { k_strip<8, 1, 0><<<blocks, 64>>>(a, b, c, pitch, R, C, plane, n_strips, n_bands, TH); });
    }
    {
        const int TH = 48, n_bands = (R + TH - 1) / TH, blocks = n_strips * n_bands * NI;
        timeit("strip P=4 nt 32w/CU", b3, [&] { k_strip<4, 1, 5><<<blocks, 64>>>(a, b, c, pitch, R, C, plane, n_strips, n_bands, TH); });
        timeit("strip P=4 nt 16w/CU", b3, [&] { k_strip<4, 1, 10><<<blocks, 64>>>(a, b, c, pitch, R, C, plane, n_strips, n_bands, TH); });
        timeit("strip P=4 nt 12w/CU", b3, [&] { k_strip<4, 1, 13><<<blocks, 64>>>(a, b, c, pitch, R, C, plane, n_strips, n_bands, TH); });
        timeit("strip P=4 nt 8w/CU", b3, [&] { k_strip<4, 1, 20><<<blocks, 64>>>(a, b, c, pitch, R, C, plane, n_strips, n_bands, TH); });
        timeit("strip P=8 nt 8w/CU", b3, [&] { k_strip<8, 1, 20><<<blocks, 64>>>(a, b, c, pitch, R, C, plane, n_strips, n_bands, TH); });
        timeit("strip P=4 st 12w/CU", b3, [&] { k_strip<4, 0, 13><<<blocks, 64>>>(a, b, c, pitch, R, C, plane, n_strips, n_bands, TH); });
        timeit("strip P=4 st 8w/CU", b3, [&] { k_strip<4, 0, 20><<<blocks, 64>>>(a, b, c, pitch, R, C, plane, n_strips, n_bands, TH); });
    }
    return 0;
}
