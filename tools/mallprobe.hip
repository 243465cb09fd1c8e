// mallprobe.hip — Infinity Cache (MALL) probe for the scale-space design (not part of libvo).
// For a buffer of S MB: kernel W writes it (plain 16-B stores), kernel R then streams it
// back (16-B loads, sum into one word per wave).  Reports R's GB/s for S from 16 MB to
// 1 GB: below ~256 MB the re-read should be served by the Infinity Cache.
//   Build: hipcc --offload-arch=gfx950 -O3 -o tools/mallprobe tools/mallprobe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_write(f4* __restrict__ a, size_t n4, float v)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        a[i] = f4{v, v + 1.0f, v + 2.0f, (float)i};
}

__global__ __launch_bounds__(256) void k_read(const f4* __restrict__ a, size_t n4, float* __restrict__ out)
{
    f4 s = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    const float t = s.x + s.y + s.z + s.w;
    if (t == 1234.5f) out[blockIdx.x] = t;          // never true; keeps the loads
}

int main()
{
    const size_t maxb = (size_t)1 << 30;
    f4* a;
    float* o;
    hipMalloc(&a, maxb);
    hipMalloc(&o, 1 << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const size_t sizes_mb[] = {16, 32, 64, 128, 192, 256, 384, 512, 1024};
    for (size_t mb : sizes_mb) {
        const size_t n4 = mb * (1 << 20) / 16;
        float best_r = 1e30f, best_w = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(e0);
            k_write<<<4096, 256>>>(a, n4, (float)rep);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float tw;
            hipEventElapsedTime(&tw, e0, e1);
            hipEventRecord(e0);
            k_read<<<4096, 256>>>(a, n4, o);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float tr;
            hipEventElapsedTime(&tr, e0, e1);
            if (tr < best_r) best_r = tr;
            if (tw < best_w) best_w = tw;
        }
        printf("S=%5zu MB  write %7.1f GB/s  read-after-write %7.1f GB/s\n", mb, mb * 1.048576e-3 / (best_w * 1e-3),
               mb * 1.048576e-3 / (best_r * 1e-3));
    }
    return 0;
}
