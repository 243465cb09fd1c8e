// match.hip — matchFeatures (VO.m:87,283,293,311,323) on gfx950.
//
// SIFT descriptors are u8-valued (0..255).  The SSD of unit-normalised rows
// (matchFeatures' Metric SSD on normalised features) is computed from the
// EXACT integer dot product:  ssd = 2 - 2 * ((float)dot * inv|a|) * inv|b|
// (DESIGN.md §3.3).  The dot products run on the i8 matrix cores:
// v_mfma_i32_32x32x32_i8 on (a - 128) x (b - 128), corrected by the row sums
//   dot(a,b) = dot(a',b') + 128 (sum a + sum b) - 2^21,
// so the result is exact and order-free; MFMA throughput is 8x the v_dot4
// VALU path.  The top-2 search is fused into the MFMA epilogue: each lane keeps
// (best, idx, second) for its 16 accumulator rows, halves merge by xor
// shuffles with a (value, index) total order, chunks of F2 merge in
// k_match_final, which also applies MatchThreshold / MaxRatio and compacts the
// pairs in ascending F1 order with a block prefix sum.
#include "vo_internal.h"

namespace vo {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// (b,i,s) <- merge with (b2,i2,s2): lexicographic min on (value, index), and
// the second smallest value of the union multiset.  Associative & commutative.
__device__ __forceinline__ void top2_merge(float& b, int& i, float& s, float b2, int i2, float s2)
{
    const float ns = fminf(fminf(s, s2), fmaxf(b, b2));
    if (b2 < b || (b2 == b && i2 < i)) { b = b2; i = i2; }
    s = ns;
}

__device__ __forceinline__ int job_rows(const int* p, int cap)
{
    int n = *p;
    return n < 0 ? 0 : (n > cap ? cap : n);
}

__device__ __forceinline__ v4i load_frag(const uint8_t* row, int off)
{
    v4i v = *reinterpret_cast<const v4i*>(row + off);
    v ^= (v4i){(int)0x80808080, (int)0x80808080, (int)0x80808080, (int)0x80808080};
    return v;
}

// One wave per (job, 32-row F1 tile, CHUNK-column F2 chunk).  Block = 4 waves.
__global__ __launch_bounds__(256) void k_match_partial(const MatchJob* __restrict__ jobs, int n_jobs,
                                                       MatchTop2* __restrict__ partial, int row_cap, int n_chunks_cap)
{
    const int lane = threadIdx.x & 63, h = lane >> 5, l31 = lane & 31;
    const long wave0 = (long)blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = (long)gridDim.x * 4;
    // total tasks
    long total = 0;
    for (int j = 0; j < n_jobs; ++j) {
        const int n1 = job_rows(jobs[j].n1, row_cap), n2 = job_rows(jobs[j].n2, row_cap);
        total += (long)((n1 + 31) / 32) * ((n2 + VO_MATCH_CHUNK - 1) / VO_MATCH_CHUNK);
    }
    for (long t = wave0; t < total; t += nwaves) {
        // locate job
        int jb = 0, n1 = 0, n2 = 0, nch = 0;
        long acc = 0, rel = 0;
        for (int j = 0; j < n_jobs; ++j) {
            n1 = job_rows(jobs[j].n1, row_cap);
            n2 = job_rows(jobs[j].n2, row_cap);
            nch = (n2 + VO_MATCH_CHUNK - 1) / VO_MATCH_CHUNK;
            const long nt = (long)((n1 + 31) / 32) * nch;
            if (t < acc + nt) { jb = j; rel = t - acc; break; }
            acc += nt;
        }
        const MatchJob J = jobs[jb];
        const int tile = (int)(rel / nch), chunk = (int)(rel - (long)tile * nch);
        const int i0 = tile * 32, j0 = chunk * VO_MATCH_CHUNK;
        const int j1 = min(j0 + VO_MATCH_CHUNK, n2);
        // A fragments: F1 row i0 + l31, bytes [32kk + 16h, +16)
        v4i a[4];
        {
            const int ia = i0 + l31;
            if (ia < n1) {
                const int ra = J.idx1 ? J.idx1[ia] : ia;
                const uint8_t* row = J.d1 + (size_t)ra * VO_DESC_LEN;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) a[kk] = load_frag(row, 32 * kk + 16 * h);
            } else {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) a[kk] = (v4i){0, 0, 0, 0};
            }
        }
        // per-accumulator-row metadata
        int sa[16];
        float ina[16];
        float best[16], second[16];
        int bidx[16];
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = i0 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
            if (row < n1) {
                const int ra = J.idx1 ? J.idx1[row] : row;
                const DescMeta m = J.m1[ra];
                sa[reg] = m.sum; ina[reg] = m.inv_norm;
            } else { sa[reg] = 0; ina[reg] = 0.0f; }
            best[reg] = INFINITY; second[reg] = INFINITY; bidx[reg] = -1;
        }
        for (int jt = j0; jt < j1; jt += 32) {
            const int jc = jt + l31;
            const bool cv = jc < j1;
            v4i b[4];
            int sb = 0;
            float inb = 0.0f;
            if (cv) {
                const int rb = J.idx2 ? J.idx2[jc] : jc;
                const uint8_t* row = J.d2 + (size_t)rb * VO_DESC_LEN;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) b[kk] = load_frag(row, 32 * kk + 16 * h);
                const DescMeta m = J.m2[rb];
                sb = m.sum; inb = m.inv_norm;
            } else {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) b[kk] = (v4i){0, 0, 0, 0};
            }
            v16i accv = (v16i){0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) accv = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[kk], b[kk], accv, 0, 0, 0);
            if (cv) {
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    const int dot = accv[reg] + 128 * (sa[reg] + sb) - 2097152;
                    const float c = ((float)dot * ina[reg]) * inb;
                    const float sv = 2.0f - 2.0f * c;
                    if (sv < best[reg]) { second[reg] = best[reg]; best[reg] = sv; bidx[reg] = jc; }
                    else if (sv < second[reg]) second[reg] = sv;
                }
            }
        }
        // merge the 32 lanes of each half (same accumulator rows, different columns)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
#pragma unroll
            for (int off = 16; off >= 1; off >>= 1) {
                const float b2 = __shfl_xor(best[reg], off);
                const int i2 = __shfl_xor(bidx[reg], off);
                const float s2 = __shfl_xor(second[reg], off);
                top2_merge(best[reg], bidx[reg], second[reg], b2, i2, s2);
            }
        }
        if (l31 < 16) {
            // lane l31 of half h writes accumulator row `l31` (select by unrolled compare)
            float bb = INFINITY, ss = INFINITY;
            int ii = -1;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg)
                if (reg == l31) { bb = best[reg]; ii = bidx[reg]; ss = second[reg]; }
            const int row = i0 + (l31 & 3) + 8 * (l31 >> 2) + 4 * h;
            if (row < n1) {
                MatchTop2 m;
                m.best = bb; m.idx = ii; m.second = ss; m.pad = 0;
                partial[((size_t)jb * n_chunks_cap + chunk) * row_cap + row] = m;
            }
        }
    }
}

__device__ __forceinline__ uint32_t block_exscan_1024_m(uint32_t v, uint32_t* sh, uint32_t* total)
{
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    if (wid == 0) {
        uint32_t s = lane < 16 ? sh[lane] : 0;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            uint32_t y = __shfl_up(s, o);
            if (lane >= o) s += y;
        }
        if (lane < 16) sh[16 + lane] = s;
    }
    __syncthreads();
    uint32_t before = wid ? sh[16 + wid - 1] : 0;
    *total = sh[16 + 15];
    __syncthreads();
    return before + x - v;
}

// One block (1024 threads) per job: merge chunks, accept, compact.
__global__ __launch_bounds__(1024) void k_match_final(const MatchJob* __restrict__ jobs, const MatchTop2* __restrict__ partial,
                                                      int row_cap, int n_chunks_cap, float T, float max_ratio)
{
    __shared__ uint32_t sh[32];
    const int jb = blockIdx.x, tid = threadIdx.x;
    const MatchJob J = jobs[jb];
    const int n1 = job_rows(J.n1, row_cap), n2 = job_rows(J.n2, row_cap);
    const int nch = (n2 + VO_MATCH_CHUNK - 1) / VO_MATCH_CHUNK;
    const int chunk = (n1 + 1023) / 1024;
    const int a = tid * chunk, e = min(a + chunk, n1);
    const MatchTop2* P = partial + (size_t)jb * n_chunks_cap * row_cap;
    // pass 1: count accepted rows in my range
    uint32_t cnt = 0;
    for (int r = a; r < e; ++r) {
        float b = INFINITY, s = INFINITY;
        int i = -1;
        for (int c = 0; c < nch; ++c) {
            const MatchTop2 m = P[(size_t)c * row_cap + r];
            top2_merge(b, i, s, m.best, m.idx, m.second);
        }
        const bool ok = i >= 0 && b <= T && (b / s) <= max_ratio;
        cnt += ok;
    }
    uint32_t total;
    uint32_t base = block_exscan_1024_m(cnt, sh, &total);
    for (int r = a; r < e; ++r) {
        float b = INFINITY, s = INFINITY;
        int i = -1;
        for (int c = 0; c < nch; ++c) {
            const MatchTop2 m = P[(size_t)c * row_cap + r];
            top2_merge(b, i, s, m.best, m.idx, m.second);
        }
        const bool ok = i >= 0 && b <= T && (b / s) <= max_ratio;
        if (ok) {
            if (base < (uint32_t)J.cap) { J.out_i[base] = r; J.out_j[base] = i; }
            base++;
        }
    }
    if (tid == 0) *J.out_n = (int)(total < (uint32_t)J.cap ? total : (uint32_t)J.cap);
}

// Descriptor metadata for externally supplied descriptors (vo_match on host data).
__global__ void k_desc_meta(const uint8_t* __restrict__ desc, DescMeta* __restrict__ meta, int n)
{
    const int lane = threadIdx.x & 63;
    for (long t = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < n; t += (long)gridDim.x * (blockDim.x >> 6)) {
        const uint8_t* d = desc + t * VO_DESC_LEN;
        int v0 = d[lane], v1 = d[lane + 64];
        int sum = v0 + v1, sq = v0 * v0 + v1 * v1;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) { sum += __shfl_xor(sum, off); sq += __shfl_xor(sq, off); }
        if (lane == 0) { DescMeta m; m.sum = sum; m.inv_norm = sq > 0 ? 1.0f / sqrtf((float)sq) : 0.0f; meta[t] = m; }
    }
}

hipError_t match_alloc(MatchBuffers& b, int max_jobs, int row_cap)
{
    b.max_jobs = max_jobs;
    b.row_cap = row_cap;
    b.n_chunks = (row_cap + VO_MATCH_CHUNK - 1) / VO_MATCH_CHUNK;
    hipError_t e = hipMalloc((void**)&b.jobs, sizeof(MatchJob) * max_jobs);
    if (e != hipSuccess) return e;
    return hipMalloc((void**)&b.partial, sizeof(MatchTop2) * (size_t)max_jobs * b.n_chunks * row_cap);
}

void match_free(MatchBuffers& b)
{
    hipFree(b.jobs);
    hipFree(b.partial);
    b = MatchBuffers();
}

MatchBuffers match_view(const MatchBuffers& b, int k0)
{
    MatchBuffers v = b;
    v.jobs = b.jobs ? b.jobs + k0 : nullptr;
    v.partial = b.partial + (size_t)k0 * b.n_chunks * b.row_cap;
    v.max_jobs = b.max_jobs - k0;
    return v;
}

void match_launch(const MatchBuffers& b, const MatchJob* d_jobs, int n_jobs, const vo_match_params& p, hipStream_t s)
{
    if (n_jobs <= 0) return;
    VO_LAUNCH(k_match_partial, dim3(2048), dim3(256), 0, s, d_jobs, n_jobs, b.partial, b.row_cap, b.n_chunks);
    VO_LAUNCH(k_match_final, dim3(n_jobs), dim3(1024), 0, s, d_jobs, (const MatchTop2*)b.partial, b.row_cap, b.n_chunks,
              p.match_threshold * 0.04f, p.max_ratio);
}

void desc_meta_launch(const uint8_t* desc, DescMeta* meta, int n, hipStream_t s)
{
    if (n <= 0) return;
    int blocks = (n + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    VO_LAUNCH(k_desc_meta, dim3(blocks), dim3(256), 0, s, desc, meta, n);
}

}  // namespace vo
