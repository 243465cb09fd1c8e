// mallprobe.hip — what HBM rate the scale-space traffic can expect on MI355X (not part of libvo).
//
// Round-2 version had one 16-B load per lane in flight (a serial accumulator), so it measured
// its own memory-level parallelism.  This version keeps U independent 16-B loads in flight per
// lane (unrolled, separate accumulators), at a grid of `waves_per_cu` x 256 CUs, and measures
// for buffers well beyond the 256 MB Infinity Cache:
//   write       : plain 16-B stores (U per lane per iteration)
//   read (RAW)  : re-read of the buffer the write kernel just produced (read-after-write)
//   copy        : read buffer A (freshly written) and write buffer B — the level blur's
//                 G_{i-1} -> G_i traffic shape (one read stream + one write stream)
// Each figure is the best of 5 repetitions, bytes / kernel time (HIP events).
//   Build: hipcc --offload-arch=gfx950 -O3 -o tools/mallprobe tools/mallprobe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void k_write(f4* __restrict__ a, size_t n4, float v)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) a[i + u * stride] = f4{v, v + 1.0f, v + 2.0f, (float)u};
    }
    for (; i < n4; i += stride) a[i] = f4{v, v, v, v};
}

template <int U>
__global__ __launch_bounds__(256) void k_read(const f4* __restrict__ a, size_t n4, float* __restrict__ out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    f4 s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) s[u] = f4{0, 0, 0, 0};
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        f4 t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = a[i + u * stride];          // U loads issued back to back
#pragma unroll
        for (int u = 0; u < U; ++u) s[u] += t[u];
    }
    for (; i < n4; i += stride) s[0] += a[i];
    f4 z = s[0];
#pragma unroll
    for (int u = 1; u < U; ++u) z += s[u];
    const float t = z.x + z.y + z.z + z.w;
    if (t == 1234.5f) out[blockIdx.x] = t;          // never true; keeps the loads
}

template <int U>
__global__ __launch_bounds__(256) void k_copy(const f4* __restrict__ a, f4* __restrict__ b, size_t n4)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        f4 t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = a[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) b[i + u * stride] = t[u] * 1.0001f;
    }
    for (; i < n4; i += stride) b[i] = a[i];
}

// blocked: workgroup b sweeps its own contiguous chunk of n4 / gridDim.x vectors (a DRAM-page
// friendlier order than the grid stride); U loads in flight per lane
template <int U>
__global__ __launch_bounds__(256) void k_copy_blk(const f4* __restrict__ a, f4* __restrict__ b, size_t n4)
{
    const size_t chunk = (n4 + gridDim.x - 1) / gridDim.x;
    const size_t lo = blockIdx.x * chunk, hi = lo + chunk < n4 ? lo + chunk : n4;
    size_t i = lo + threadIdx.x;
    for (; i + (U - 1) * 256 < hi; i += U * 256) {
        f4 t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = a[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) b[i + u * 256] = t[u] * 1.0001f;
    }
    for (; i < hi; i += 256) b[i] = a[i];
}

template <int U>
__global__ __launch_bounds__(256) void k_read_blk(const f4* __restrict__ a, size_t n4, float* __restrict__ out)
{
    const size_t chunk = (n4 + gridDim.x - 1) / gridDim.x;
    const size_t lo = blockIdx.x * chunk, hi = lo + chunk < n4 ? lo + chunk : n4;
    size_t i = lo + threadIdx.x;
    f4 s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) s[u] = f4{0, 0, 0, 0};
    for (; i + (U - 1) * 256 < hi; i += U * 256) {
        f4 t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = a[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) s[u] += t[u];
    }
    for (; i < hi; i += 256) s[0] += a[i];
    f4 z = s[0];
#pragma unroll
    for (int u = 1; u < U; ++u) z += s[u];
    const float t = z.x + z.y + z.z + z.w;
    if (t == 1234.5f) out[blockIdx.x] = t;
}

static float timed(hipEvent_t e0, hipEvent_t e1, void (*launch)(void*), void* arg)
{
    hipEventRecord(e0);
    launch(arg);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t;
    hipEventElapsedTime(&t, e0, e1);
    return t;
}

struct Args { f4* a; f4* b; float* o; size_t n4; int grid; int u; float v; };

template <int U> static void lw(void* p) { Args* A = (Args*)p; k_write<U><<<A->grid, 256>>>(A->a, A->n4, A->v); }
template <int U> static void lr(void* p) { Args* A = (Args*)p; k_read<U><<<A->grid, 256>>>(A->a, A->n4, A->o); }
template <int U> static void lc(void* p) { Args* A = (Args*)p; k_copy<U><<<A->grid, 256>>>(A->a, A->b, A->n4); }

template <int U> static void lcb(void* p) { Args* A = (Args*)p; k_copy_blk<U><<<A->grid, 256>>>(A->a, A->b, A->n4); }
template <int U> static void lrb(void* p) { Args* A = (Args*)p; k_read_blk<U><<<A->grid, 256>>>(A->a, A->n4, A->o); }

typedef void (*Fn)(void*);
static Fn pick(int kind, int u)
{
    if (kind == 0) return u == 1 ? lw<1> : u == 4 ? lw<4> : lw<8>;
    if (kind == 1) return u == 1 ? lr<1> : u == 4 ? lr<4> : lr<8>;
    return u == 1 ? lc<1> : u == 4 ? lc<4> : lc<8>;
}

int main()
{
    const size_t maxb = (size_t)2 << 30;                   // 2 GiB per buffer
    f4 *a, *b;
    float* o;
    if (hipMalloc(&a, maxb) != hipSuccess || hipMalloc(&b, maxb) != hipSuccess || hipMalloc(&o, 1 << 22) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int dev = 0, n_cu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    printf("CUs %d; figures are GB/s (1e9 B/s), best of 5; copy counts read + write bytes\n", n_cu);
    const size_t sizes_mb[] = {64, 256, 512, 1024, 2048};
    const int units[] = {1, 4, 8};
    const int waves_per_cu[] = {8, 16, 32};                 // 256-thread blocks = 4 waves each
    for (size_t mb : sizes_mb) {
        for (int u : units) {
            for (int w : waves_per_cu) {
                Args A{a, b, o, mb * (1 << 20) / 16, n_cu * w / 4, u, 0.0f};
                float best[3] = {1e30f, 1e30f, 1e30f};
                for (int rep = 0; rep < 5; ++rep) {
                    A.v = (float)rep;
                    float tw = timed(e0, e1, pick(0, u), &A);                 // write a
                    float tr = timed(e0, e1, pick(1, u), &A);                 // read a (just written)
                    timed(e0, e1, pick(0, u), &A);                            // write a again
                    float tc = timed(e0, e1, pick(2, u), &A);                 // copy a -> b
                    if (tw < best[0]) best[0] = tw;
                    if (tr < best[1]) best[1] = tr;
                    if (tc < best[2]) best[2] = tc;
                }
                const double gb = mb * 1.048576e-3;
                printf("S=%5zu MB  U=%d  waves/CU=%2d  write %7.1f  read-after-write %7.1f  copy %7.1f\n", mb, u, w,
                       gb / (best[0] * 1e-3), gb / (best[1] * 1e-3), 2 * gb / (best[2] * 1e-3));
                fflush(stdout);
            }
        }
    }
    printf("blocked (each workgroup sweeps one contiguous chunk):\n");
    for (size_t mb : {(size_t)1024, (size_t)2048}) {
        for (int w : {4, 8, 16}) {
            for (int blocks_per : {1, 4}) {                   // workgroups per 4-wave slot set
                Args A{a, b, o, mb * (1 << 20) / 16, n_cu * w / 4 * blocks_per, 4, 0.0f};
                float br = 1e30f, bc = 1e30f;
                for (int rep = 0; rep < 5; ++rep) {
                    timed(e0, e1, pick(0, 4), &A);
                    float tr = timed(e0, e1, lrb<4>, &A);
                    timed(e0, e1, pick(0, 4), &A);
                    float tc = timed(e0, e1, lcb<4>, &A);
                    if (tr < br) br = tr;
                    if (tc < bc) bc = tc;
                }
                const double gb = mb * 1.048576e-3;
                printf("S=%5zu MB  U=4  waves/CU=%2d  grid x%d  read-after-write %7.1f  copy %7.1f\n", mb, w, blocks_per,
                       gb / (br * 1e-3), 2 * gb / (bc * 1e-3));
                fflush(stdout);
            }
        }
    }
    return 0;
}
