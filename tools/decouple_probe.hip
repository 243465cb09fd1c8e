// decouple_probe.hip — does sharing one in-order vmcnt between a streaming kernel's row loads and
// its row stores cost bandwidth?  (instrumentation, not libvo)
// The level blur's memory pattern without its arithmetic: 64 planes of 750 rows x 2560 floats
// (492 MB in, 492 MB out, beyond the 256 MB MALL), one 256-column strip x 128-row band per unit:
//   coupled<P>   one wave per unit loads row k+P while it stores row k (loads and stores in one
//                vmcnt queue: waiting for a load also waits for every store issued before it)
//   decoupled<D> two waves per unit: a loader wave keeps D blocks of 4 rows of loads in flight and
//                writes landed rows into an LDS ring; a storer wave reads the ring and stores, and
//                never waits on vmcnt (one barrier per block of 4 rows)
//   loads only / stores only: the halves alone
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/decouple_probe.hip -o tools/decouple_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int PITCH = 2560, R = 750, NIMG = 64, TH = 128, NS = 10;   // 10 strips of 256 columns
constexpr int NB = (R + TH - 1) / TH;
constexpr size_t PLANE = (size_t)PITCH * R;

__device__ inline void unit(int bid, int& x0, int& y0, int& img)
{
    const int strip = bid % NS, tb = bid / NS;
    x0 = strip * 256; y0 = (tb % NB) * TH; img = tb / NB;
}

template <int P>
__global__ __launch_bounds__(64) void k_coupled(const float* __restrict__ a, float* __restrict__ b)
{
    int x0, y0, img;
    unit(blockIdx.x, x0, y0, img);
    const int th = min(TH, R - y0), xl = x0 + 4 * threadIdx.x;
    const float* ap = a + img * PLANE + xl;
    float* bp = b + img * PLANE + xl;
    f4 pf[P];
#pragma unroll
    for (int u = 0; u < P; ++u) pf[u] = *reinterpret_cast<const f4*>(ap + (size_t)(y0 + u) * PITCH);
    for (int k0 = 0; k0 < th; k0 += P) {
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int k = k0 + u;
            const f4 v = pf[u];
            pf[u] = *reinterpret_cast<const f4*>(ap + (size_t)(y0 + min(k + P, th - 1)) * PITCH);
            if (k < th) __builtin_nontemporal_store(v * 2.0f, reinterpret_cast<f4*>(bp + (size_t)(y0 + k) * PITCH));
        }
    }
}

// D blocks of 4 rows in flight in the loader's registers; ring of 2 blocks in LDS
template <int D>
__global__ __launch_bounds__(128) void k_decoupled(const float* __restrict__ a, float* __restrict__ b)
{
    __shared__ f4 ring[2][4][64];
    int x0, y0, img;
    unit(blockIdx.x, x0, y0, img);
    const int th = min(TH, R - y0), nblk = (th + 3) / 4;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int xl = x0 + 4 * lane;
    const float* ap = a + img * PLANE + xl;
    float* bp = b + img * PLANE + xl;
    f4 pf[D + 1][4];
    auto load = [&](int blk, f4 (&s)[4]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) s[u] = *reinterpret_cast<const f4*>(ap + (size_t)(y0 + min(4 * blk + u, th - 1)) * PITCH);
    };
    // wave-uniform roles in two separate loops (no per-block branches, so the compiler's waitcnt
    // pass keeps exact counts); one s_barrier per block in both
    if (w == 0) {
#pragma unroll
        for (int d = 0; d < D; ++d) load(d, pf[d]);
#pragma unroll
        for (int u = 0; u < 4; ++u) ring[0][u][lane] = pf[0][u];   // block 0 (waits for it)
        load(D, pf[0]);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_s_barrier();
        for (int t = 0; t < nblk; t += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                // block t+d+1 is in set (d+1)%D: stage it into the ring slot the storer does not
                // read this block, then refill the set with block t+d+1+D (clamped: re-reads)
                const int blk = t + d;
#pragma unroll
                for (int u = 0; u < 4; ++u) ring[(blk + 1) & 1][u][lane] = pf[(d + 1) % D][u];
                load(min(blk + 1 + D, nblk - 1), pf[(d + 1) % D]);
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_s_barrier();
            }
        }
    } else {
        __builtin_amdgcn_s_barrier();
        for (int t = 0; t < nblk; t += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int blk = t + d;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = min(4 * blk + u, th - 1);       // past the band: row th-1 again
                    const f4 v = ring[blk & 1][u][lane];
                    __builtin_nontemporal_store(v * 2.0f, reinterpret_cast<f4*>(bp + (size_t)(y0 + k) * PITCH));
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_s_barrier();
            }
        }
    }
}

// the blur-shaped comparison: W dependent packed FMAs per row vector (about the level blur's
// per-row VALU), occupancy capped by dynamic LDS at the blur's 2 waves per SIMD.
//   coupledW: one wave per unit, P = 4 rows ahead, stores in the same vmcnt queue
//   dec3W:    1 loader wave + 3 compute waves per workgroup (3 bands of one strip), the loader
//             keeping 2 blocks of 4 rows per band in flight in registers, an LDS ring of 2
//             blocks per band; compute waves never wait on vmcnt
template <int W>
__device__ __forceinline__ f4 work(f4 v)
{
    f4 a = v;
#pragma unroll
    for (int i = 0; i < W; ++i) a = a * 0.999f + v;
    return a;
}

template <int W>
__global__ __launch_bounds__(64) void k_coupledW(const float* __restrict__ a, float* __restrict__ b)
{
    extern __shared__ float pad[];
    int x0, y0, img;
    unit(blockIdx.x, x0, y0, img);
    const int th = min(TH, R - y0), xl = x0 + 4 * threadIdx.x;
    const float* ap = a + img * PLANE + xl;
    float* bp = b + img * PLANE + xl;
    constexpr int P = 4;
    f4 pf[P];
#pragma unroll
    for (int u = 0; u < P; ++u) pf[u] = *reinterpret_cast<const f4*>(ap + (size_t)(y0 + u) * PITCH);
    for (int k0 = 0; k0 < th; k0 += P) {
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int k = min(k0 + u, th - 1);
            const f4 v = pf[u];
            pf[u] = *reinterpret_cast<const f4*>(ap + (size_t)(y0 + min(k0 + u + P, th - 1)) * PITCH);
            __builtin_nontemporal_store(work<W>(v), reinterpret_cast<f4*>(bp + (size_t)(y0 + k) * PITCH));
        }
    }
    if (threadIdx.x == 1000) pad[0] = 0;
}

constexpr int NBG = (NB + 2) / 3;   // band groups of 3
template <int W>
__global__ __launch_bounds__(256) void k_dec3W(const float* __restrict__ a, float* __restrict__ b)
{
    __shared__ f4 ring[3][2][4][64];                      // band, block parity, row, lane
    extern __shared__ float pad[];
    const int bid = blockIdx.x;
    const int strip = bid % NS, tb = bid / NS, bg = tb % NBG, img = tb / NBG;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int x0 = strip * 256, xl = x0 + 4 * lane;
    constexpr int nblk = TH / 4;                          // every band runs TH rows (clamped re-reads past R)
    if (w == 0) {
        const float* ap[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) ap[c] = a + img * PLANE + xl;
        auto rowp = [&](int c, int k) {
            const int y = min((3 * bg + c) * TH + k, R - 1);
            return reinterpret_cast<const f4*>(a + img * PLANE + (size_t)y * PITCH + xl);
        };
        f4 s0[3][4], s1[3][4];
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int u = 0; u < 4; ++u) s0[c][u] = *rowp(c, u);
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int u = 0; u < 4; ++u) s1[c][u] = *rowp(c, 4 + u);
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int u = 0; u < 4; ++u) ring[c][0][u][lane] = s0[c][u];
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_s_barrier();
        for (int t = 0; t < nblk; t += 2) {
            // even block t: s1 holds block t+1 -> ring parity 1; refill s0 with block t+2
#pragma unroll
            for (int c = 0; c < 3; ++c)
#pragma unroll
                for (int u = 0; u < 4; ++u) ring[c][1][u][lane] = s1[c][u];
#pragma unroll
            for (int c = 0; c < 3; ++c)
#pragma unroll
                for (int u = 0; u < 4; ++u) s0[c][u] = *rowp(c, min(4 * (t + 2) + u, TH - 1));
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_s_barrier();
#pragma unroll
            for (int c = 0; c < 3; ++c)
#pragma unroll
                for (int u = 0; u < 4; ++u) ring[c][0][u][lane] = s0[c][u];
#pragma unroll
            for (int c = 0; c < 3; ++c)
#pragma unroll
                for (int u = 0; u < 4; ++u) s1[c][u] = *rowp(c, min(4 * (t + 3) + u, TH - 1));
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_s_barrier();
        }
    } else {
        const int c = w - 1, band = 3 * bg + c;
        float* bp = b + img * PLANE + xl;
        __builtin_amdgcn_s_barrier();
        for (int t = 0; t < nblk; ++t) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int y = min(band * TH + 4 * t + u, R - 1);
                const f4 v = ring[c][t & 1][u][lane];
                __builtin_nontemporal_store(work<W>(v), reinterpret_cast<f4*>(bp + (size_t)y * PITCH));
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_s_barrier();
        }
    }
    if (threadIdx.x == 1000) pad[0] = 0;
}

__global__ __launch_bounds__(64) void k_loads(const float* __restrict__ a, float* __restrict__ b)
{
    int x0, y0, img;
    unit(blockIdx.x, x0, y0, img);
    const int th = min(TH, R - y0), xl = x0 + 4 * threadIdx.x;
    const float* ap = a + img * PLANE + xl;
    f4 acc = {0, 0, 0, 0};
    for (int k0 = 0; k0 < th; k0 += 8) {
        f4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f4*>(ap + (size_t)(y0 + min(k0 + u, th - 1)) * PITCH);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    if (acc.x == 12345.0f) b[0] = acc.y;
}

__global__ __launch_bounds__(64) void k_stores(const float* __restrict__ a, float* __restrict__ b)
{
    int x0, y0, img;
    unit(blockIdx.x, x0, y0, img);
    const int th = min(TH, R - y0), xl = x0 + 4 * threadIdx.x;
    float* bp = b + img * PLANE + xl;
    const f4 v = {1.0f, 2.0f, 3.0f, (float)xl};
    for (int k = 0; k < th; ++k) __builtin_nontemporal_store(v, reinterpret_cast<f4*>(bp + (size_t)(y0 + k) * PITCH));
}

template <typename F>
static float timeit(F launch, int reps = 5)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    launch(); launch();
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[reps / 2];
}

int main()
{
    float *a, *b;
    const size_t bytes = PLANE * NIMG * sizeof(float);
    hipMalloc(&a, bytes); hipMalloc(&b, bytes);
    hipMemset(a, 0, bytes); hipMemset(b, 0, bytes);
    const int units = NS * NB * NIMG;
    const double alg = 2.0 * (double)NIMG * R * 2560 * 4;          // read + write bytes
    auto rep = [&](const char* n, float ms, double by) { printf("%-22s %8.3f ms  %6.2f TB/s\n", n, ms, by / (ms * 1e-3) / 1e12); };
    rep("coupled P=4", timeit([&] { hipLaunchKernelGGL(k_coupled<4>, dim3(units), dim3(64), 0, 0, a, b); }), alg);
    rep("coupled P=8", timeit([&] { hipLaunchKernelGGL(k_coupled<8>, dim3(units), dim3(64), 0, 0, a, b); }), alg);
    rep("decoupled D=2", timeit([&] { hipLaunchKernelGGL(k_decoupled<2>, dim3(units), dim3(128), 0, 0, a, b); }), alg);
    rep("decoupled D=3", timeit([&] { hipLaunchKernelGGL(k_decoupled<3>, dim3(units), dim3(128), 0, 0, a, b); }), alg);
    rep("decoupled D=4", timeit([&] { hipLaunchKernelGGL(k_decoupled<4>, dim3(units), dim3(128), 0, 0, a, b); }), alg);
    // blur-shaped: 2 blur waves per SIMD (8 per CU): coupled one-wave units with 20 KB of LDS
    // each; decoupled 4-wave workgroups with 40 KB (2 per CU: 6 compute + 2 loader waves)
    const int units3 = NS * NBG * NIMG;
    const double alg3 = 2.0 * (double)NIMG * NBG * 3 * TH * 2560 * 4;
    rep("coupledW8 occ2", timeit([&] { hipLaunchKernelGGL(k_coupledW<8>, dim3(units), dim3(64), 20480, 0, a, b); }), alg);
    rep("dec3W8 occ2", timeit([&] { hipLaunchKernelGGL(k_dec3W<8>, dim3(units3), dim3(256), 40960 - 24576, 0, a, b); }), alg3);
    rep("coupledW32 occ2", timeit([&] { hipLaunchKernelGGL(k_coupledW<32>, dim3(units), dim3(64), 20480, 0, a, b); }), alg);
    rep("dec3W32 occ2", timeit([&] { hipLaunchKernelGGL(k_dec3W<32>, dim3(units3), dim3(256), 40960 - 24576, 0, a, b); }), alg3);
    rep("loads only", timeit([&] { hipLaunchKernelGGL(k_loads, dim3(units), dim3(64), 0, 0, a, b); }), alg / 2);
    rep("stores only", timeit([&] { hipLaunchKernelGGL(k_stores, dim3(units), dim3(64), 0, 0, a, b); }), alg / 2);
    // correctness of the copies: b = 2 a
    std::vector<float> ha(PITCH * 8), hb(PITCH * 8);
    hipMemset(a, 0, bytes);
    std::vector<float> src(PLANE);
    for (size_t i = 0; i < PLANE; ++i) src[i] = (float)(i % 977);
    hipMemcpy(a + 5 * PLANE, src.data(), PLANE * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_decoupled<3>, dim3(units), dim3(128), 0, 0, a, b);
    std::vector<float> dst(PLANE);
    hipMemcpy(dst.data(), b + 5 * PLANE, PLANE * 4, hipMemcpyDeviceToHost);
    long bad = 0;
    for (int y = 0; y < R; ++y)
        for (int x = 0; x < NS * 256; ++x) bad += dst[(size_t)y * PITCH + x] != 2.0f * src[(size_t)y * PITCH + x];
    printf("decoupled copy mismatches: %ld\n", bad);
    hipFree(a); hipFree(b);
    return bad ? 1 : 0;
}
