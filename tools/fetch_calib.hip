// fetch_calib.hip — calibrates rocprofv3 FETCH_SIZE for the access shapes of libvo's feature
// kernels (not part of libvo).  The microarchitecture guide calibrates FETCH_SIZE only for wide
// coalesced streaming reads (it reports exactly half their bytes on gfx950) and leaves other
// widths uncalibrated; k_orient / k_desc / k_refine read 4-B values from small windows.  Each
// kernel below reads a KNOWN number of distinct 128-B lines once, so FETCH_SIZE per dispatch
// (rocprofv3 --pmc FETCH_SIZE) divided by that figure is the factor to apply to those kernels.
//   k_stream16 : 16 B per lane, coalesced, the whole 1 GiB buffer           lines = 1 GiB / 128
//   k_stream4  : 4 B per lane, coalesced, the whole buffer                   lines = 1 GiB / 128
//   k_win32a   : one wave per 32 x 32-float window, rows 128-B aligned        lines = 32 per window
//   k_win32u   : the same windows shifted by 16 floats (each row on 2 lines)  lines = 64 per window
//   k_win24    : one wave per 24 x 24-float window at an arbitrary 4-B offset (k_orient's shape):
//                lines counted on the host from the offsets
// One cell of 64 rows x 256 floats per window, so no line is shared between windows.
//   Build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
static const int PITCH = 8192;                 // floats per row (32 KiB)
static const int ROWS = 32768;                 // 1 GiB plane
static const int CELL_R = 64, CELL_C = 256;    // one window per cell
static const int CELLS_X = PITCH / CELL_C, CELLS_Y = ROWS / CELL_R;
static const int NWIN = CELLS_X * CELLS_Y;     // 16384 windows

__global__ __launch_bounds__(256) void k_stream16(const f4* __restrict__ a, size_t n4, float* __restrict__ out)
{
    f4 s = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s.x + s.y + s.z + s.w == 12345.0f) out[0] = s.x;
}

__global__ __launch_bounds__(256) void k_stream4(const float* __restrict__ a, size_t n, float* __restrict__ out)
{
    float s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.0f) out[0] = s;
}

__device__ __forceinline__ uint32_t hash(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// one wave per window; lane l reads column l % W of two rows per iteration
template <int W>
__global__ __launch_bounds__(64) void k_win(const float* __restrict__ a, int shift, int random_off, float* __restrict__ out)
{
    const int w = blockIdx.x, lane = threadIdx.x;
    const int cx = w % CELLS_X, cy = w / CELLS_X;
    int off = shift;
    if (random_off) off = hash(w) % (CELL_C - W);        // any 4-B offset within the cell
    const float* base = a + (size_t)(cy * CELL_R) * PITCH + cx * CELL_C + off;
    float s = 0;
    const int per = 64 / 32;                              // rows per iteration (lanes 32..63 idle for W = 24)
    for (int r = lane / 32; r < W; r += per)
        if (lane % 32 < W) s += base[(size_t)r * PITCH + lane % 32];
    if (s == 12345.0f) out[0] = s;
}

static long lines_win24()
{
    long n = 0;
    for (int w = 0; w < NWIN; ++w) {
        uint32_t x = (uint32_t)w;
        x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
        const int off = x % (CELL_C - 24);
        const long first = off / 32, last = (off + 23) / 32;     // 32 floats per 128-B line; cells are line aligned
        n += 24 * (last - first + 1);
    }
    return n;
}

int main()
{
    const size_t n = (size_t)PITCH * ROWS;
    float* a = nullptr;
    float* out = nullptr;
    if (hipMalloc(&a, n * 4) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(a, 0, n * 4);
    hipDeviceSynchronize();
    auto run = [&](const char* name, auto launch, double lines) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-11s lines %12.0f  line_bytes %14.0f  %.3f ms\n", name, lines, lines * 128.0, ms);
    };
    for (int rep = 0; rep < 2; ++rep) {
        run("k_stream16", [&] { hipLaunchKernelGGL(k_stream16, dim3(4096), dim3(256), 0, 0, (const f4*)a, n / 4, out); }, n * 4 / 128.0);
        run("k_stream4", [&] { hipLaunchKernelGGL(k_stream4, dim3(4096), dim3(256), 0, 0, a, n, out); }, n * 4 / 128.0);
        run("k_win32a", [&] { hipLaunchKernelGGL(k_win<32>, dim3(NWIN), dim3(64), 0, 0, a, 0, 0, out); }, 32.0 * NWIN);
        run("k_win32u", [&] { hipLaunchKernelGGL(k_win<32>, dim3(NWIN), dim3(64), 0, 0, a, 16, 0, out); }, 64.0 * NWIN);
        run("k_win24", [&] { hipLaunchKernelGGL(k_win<24>, dim3(NWIN), dim3(64), 0, 0, a, 0, 1, out); }, (double)lines_win24());
    }
    if (hipDeviceSynchronize() != hipSuccess) { printf("error\n"); return 1; }
    printf("done\n");
    return 0;
}
