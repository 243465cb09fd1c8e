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
// k_match_merge (one thread per F1 row), which also applies MatchThreshold /
// MaxRatio; k_match_compact writes the pairs in ascending F1 order with a block
// prefix sum.
#include "vo_internal.h"

namespace vo {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// Ranking in the cosine domain.  The spec's SSD is sv = 2 - 2c with
// c = ((float)dot * inv|a|) * inv|b|; sv is a non-increasing function of c, so the
// k-th largest c maps to the k-th smallest sv, and for c >= 0.5 (sv <= 1, Sterbenz:
// 2 - 2c is exact) it is strictly decreasing.  Every accepted match has
// sv <= 0.04, so the argmax-c set equals the argmin-sv set there and the tie rule
// (lowest F2 index) picks the same column; the second-best SSD is recovered as
// 2 - 2 * (second-largest c).  Rows whose best sv > 1 may pick another index among
// sv ties but are rejected by the threshold either way.
// (b,i,s) <- merge with (b2,i2,s2): lexicographic max on (value, -index), and the
// second largest value of the union multiset.  Associative & commutative.
__device__ __forceinline__ void top2c_merge(float& b, int& i, float& s, float b2, int i2, float s2)
{
    const float ns = fmaxf(fmaxf(s, s2), fminf(b, b2));
    if (b2 > b || (b2 == b && i2 < i)) { b = b2; i = i2; }
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
// The F2 side is software-pipelined: the index of tile t+2 and the fragments +
// metadata of tile t+1 are in flight while tile t runs its 4 MFMAs and epilogue.
// Epilogue per accumulator element: dot = acc + 128 sa - 2^21 + 128 sb (one add3),
// c = ((float)dot * inv|a|) * inv|b|, then a branch-free top-2 on c.
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
        // per-accumulator-row constants
        int rk[16];
        float ina[16];
        float best[16], second[16];
        int bidx[16];
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = i0 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
            int sa = 0;
            ina[reg] = 0.0f;
            if (row < n1) {
                const int ra = J.idx1 ? J.idx1[row] : row;
                const DescMeta m = J.m1[ra];
                sa = m.sum; ina[reg] = m.inv_norm;
            }
            rk[reg] = 128 * sa - 2097152;
            best[reg] = -INFINITY; second[reg] = -INFINITY; bidx[reg] = -1;
        }
        // F2 pipeline: column jc of tile jt -> descriptor row (clamped into the chunk; the
        // epilogue masks columns >= j1)
        auto col_row = [&](int jt) {
            const int jc = min(jt + l31, j1 - 1);
            return J.idx2 ? J.idx2[jc] : jc;
        };
        v4i bn[4];
        int ckn, rb_next = col_row(j0 + 32 < j1 ? j0 + 32 : j0);
        float inbn;
        {
            const int rb = col_row(j0);
            const uint8_t* row = J.d2 + (size_t)rb * VO_DESC_LEN;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) bn[kk] = load_frag(row, 32 * kk + 16 * h);
            const DescMeta m = J.m2[rb];
            ckn = 128 * m.sum; inbn = m.inv_norm;
        }
        for (int jt = j0; jt < j1; jt += 32) {
            v4i b[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) b[kk] = bn[kk];
            const int ck = ckn;
            const float inb = inbn;
            if (jt + 32 < j1) {                           // issue tile jt+32, and the index of jt+64
                const uint8_t* row = J.d2 + (size_t)rb_next * VO_DESC_LEN;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) bn[kk] = load_frag(row, 32 * kk + 16 * h);
                const DescMeta m = J.m2[rb_next];
                ckn = 128 * m.sum; inbn = m.inv_norm;
                if (jt + 64 < j1) rb_next = col_row(jt + 64);
            }
            v16i accv = (v16i){0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) accv = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[kk], b[kk], accv, 0, 0, 0);
            const int jc = jt + l31;
            // ragged last tile: masked columns get c = -inf (never ranked)
            const float cmask = jc < j1 ? 0.0f : -INFINITY;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const float f = (float)(accv[reg] + rk[reg] + ck);
                const float c = (f * ina[reg]) * inb + cmask;
                const bool gt = c > best[reg];
                second[reg] = fmaxf(second[reg], fminf(c, best[reg]));
                best[reg] = fmaxf(best[reg], c);
                bidx[reg] = gt ? jc : bidx[reg];
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
                top2c_merge(best[reg], bidx[reg], second[reg], b2, i2, s2);
            }
        }
        if (l31 < 16) {
            // lane l31 of half h writes accumulator row `l31` (select by unrolled compare)
            float bb = -INFINITY, ss = -INFINITY;
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

// One thread per (job, F1 row): merge the F2 chunks, back to SSD, MatchThreshold and
// MaxRatio.  res = accepted F2 index or -1.
__global__ __launch_bounds__(256) void k_match_merge(const MatchJob* __restrict__ jobs, const MatchTop2* __restrict__ partial,
                                                     int* __restrict__ res, int row_cap, int n_chunks_cap, float T, float max_ratio)
{
    const int jb = blockIdx.y, r = blockIdx.x * 256 + threadIdx.x;
    const int n1 = job_rows(jobs[jb].n1, row_cap), n2 = job_rows(jobs[jb].n2, row_cap);
    if (r >= n1) return;
    const int nch = (n2 + VO_MATCH_CHUNK - 1) / VO_MATCH_CHUNK;
    const MatchTop2* P = partial + (size_t)jb * n_chunks_cap * row_cap + r;
    float b = -INFINITY, s = -INFINITY;
    int i = -1;
    for (int c = 0; c < nch; ++c) {
        const MatchTop2 m = P[(size_t)c * row_cap];
        top2c_merge(b, i, s, m.best, m.idx, m.second);
    }
    const float bs = 2.0f - 2.0f * b, ss = 2.0f - 2.0f * s;      // SSD of best / second best
    const bool ok = i >= 0 && bs <= T && (bs / ss) <= max_ratio;
    res[(size_t)jb * row_cap + r] = ok ? i : -1;
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

// One block (1024 threads) per job: compact the accepted rows in ascending F1 order.
__global__ __launch_bounds__(1024) void k_match_compact(const MatchJob* __restrict__ jobs, const int* __restrict__ res, int row_cap)
{
    __shared__ uint32_t sh[32];
    const int jb = blockIdx.x, tid = threadIdx.x;
    const MatchJob J = jobs[jb];
    const int n1 = job_rows(J.n1, row_cap);
    const int chunk = (n1 + 1023) / 1024;
    const int a = tid * chunk, e = min(a + chunk, n1);
    const int* R = res + (size_t)jb * row_cap;
    uint32_t cnt = 0;
    for (int r = a; r < e; ++r) cnt += R[r] >= 0;
    uint32_t total;
    uint32_t base = block_exscan_1024_m(cnt, sh, &total);
    for (int r = a; r < e; ++r) {
        const int i = R[r];
        if (i >= 0) {
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
    if ((e = hipMalloc((void**)&b.res, sizeof(int) * (size_t)max_jobs * row_cap)) != hipSuccess) return e;
    return hipMalloc((void**)&b.partial, sizeof(MatchTop2) * (size_t)max_jobs * b.n_chunks * row_cap);
}

void match_free(MatchBuffers& b)
{
    hipFree(b.jobs);
    hipFree(b.partial);
    hipFree(b.res);
    b = MatchBuffers();
}

MatchBuffers match_view(const MatchBuffers& b, int k0)
{
    MatchBuffers v = b;
    v.jobs = b.jobs ? b.jobs + k0 : nullptr;
    v.partial = b.partial + (size_t)k0 * b.n_chunks * b.row_cap;
    v.res = b.res + (size_t)k0 * b.row_cap;
    v.max_jobs = b.max_jobs - k0;
    return v;
}

void match_launch(const MatchBuffers& b, const MatchJob* d_jobs, int n_jobs, const vo_match_params& p, hipStream_t s)
{
    if (n_jobs <= 0) return;
    VO_LAUNCH(k_match_partial, dim3(2048), dim3(256), 0, s, d_jobs, n_jobs, b.partial, b.row_cap, b.n_chunks);
    VO_LAUNCH(k_match_merge, dim3((b.row_cap + 255) / 256, n_jobs), dim3(256), 0, s, d_jobs, (const MatchTop2*)b.partial,
              b.res, b.row_cap, b.n_chunks, p.match_threshold * 0.04f, p.max_ratio);
    VO_LAUNCH(k_match_compact, dim3(n_jobs), dim3(1024), 0, s, d_jobs, (const int*)b.res, b.row_cap);
}

void desc_meta_launch(const uint8_t* desc, DescMeta* meta, int n, hipStream_t s)
{
    if (n <= 0) return;
    int blocks = (n + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    VO_LAUNCH(k_desc_meta, dim3(blocks), dim3(256), 0, s, desc, meta, n);
}

}  // namespace vo
