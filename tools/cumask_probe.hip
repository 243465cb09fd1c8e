// cumask_probe.hip -- does hipExtStreamCreateWithCUMask restrict a stream's kernels to the
// masked CUs on this stack?  A VALU-bound kernel of 4096 one-wave blocks, timed on an
// unmasked stream and on streams masked to 1/4 and 1/64 of the CUs.
// Build: hipcc --offload-arch=gfx950 -O3 tools/cumask_probe.hip -o tools/cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(64) void k_spin(float* out, int iters)
{
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    for (int i = 0; i < iters; ++i) a = __builtin_fmaf(a, b, 1e-7f);
    if (a == 12345.0f) out[blockIdx.x] = a;
}

static float run(hipStream_t s, float* out)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_spin, dim3(4096), dim3(64), 0, s, out, 20000);
    (void)hipEventRecord(e0, s);
    hipLaunchKernelGGL(k_spin, dim3(4096), dim3(64), 0, s, out, 20000);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main()
{
    int n_cu = 0;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    (void)hipMalloc(&out, 4096 * sizeof(float));
    hipStream_t s0;
    (void)hipStreamCreate(&s0);
    printf("CUs %d  unmasked %.3f ms\n", n_cu, run(s0, out));
    for (int div : {4, 64}) {
        std::vector<uint32_t> m((n_cu + 31) / 32, 0u);
        for (int i = 0; i < n_cu; ++i)
            if (i % div == 0) m[i / 32] |= 1u << (i % 32);
        hipStream_t s;
        hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data());
        printf("mask 1/%d (%s): %.3f ms\n", div, hipGetErrorString(e), e == hipSuccess ? run(s, out) : -1.0f);
    }
    return 0;
}
