// match.hip — matchFeatures (VO.m:87,283,293,311,323) on gfx950.
//
// SIFT descriptors are u8-valued (0..255).  The SSD of unit-normalised rows
// (matchFeatures' Metric SSD on normalised features) is computed from the
// EXACT integer dot product:  ssd = 2 - 2 * ((float)dot * inv|a|) * inv|b|
// (DESIGN.md §3.3).  The dot products run on the i8 matrix cores:
// v_mfma_i32_32x32x32_i8 on (a - 128) x (b - 128), corrected by the row sums
//   dot(a,b) = dot(a',b') + 128 (sum a + sum b) - 2^21,
// so the result is exact and order-free; MFMA throughput is 8x the v_dot4
// VALU path.  The top-2 search is fused into the MFMA epilogue: the tile is computed
// transposed (F2 columns x F1 rows), so each lane keeps (best, idx, second) for ONE F1
// row over the F2 columns it holds, the two half-waves that share a row merge with a
// (value, index) total order, and the F2 chunks merge in k_match_finish (one workgroup
// per job), which also applies MatchThreshold / MaxRatio and writes the pairs in
// ascending F1 order (k_match_merge + k_match_compact with VO_MATCH_FINISH=0).
#include "vo_internal.h"
#include "vo_geom.h"

namespace vo {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float vo_f2 __attribute__((ext_vector_type(2)));
typedef float vo_f4 __attribute__((ext_vector_type(4)));

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

// Pointers read from the job table are generic to the compiler, so loads through them became
// flat loads, which count in both vmcnt and lgkmcnt and can only be waited for with vmcnt(0) /
// lgkmcnt(0): every LDS wait of the tile loop also waited for the next tile's prefetch.  Every
// job pointer addresses global memory (hipMalloc), so its loads and stores go through the
// global address space.
template <class T>
__device__ __forceinline__ T gld(const T* p)
{
    return *(const __attribute__((address_space(1))) T*)p;
}
template <class T>
__device__ __forceinline__ void gst(T* p, T v)
{
    *(__attribute__((address_space(1))) T*)p = v;
}

__device__ __forceinline__ DescMeta gld_meta(const DescMeta* p)
{
    typedef int i2_t __attribute__((ext_vector_type(2)));
    const i2_t v = gld(reinterpret_cast<const i2_t*>(p));       // {sum, inv_norm bits}
    DescMeta m;
    m.sum = v.x;
    m.inv_norm = __int_as_float(v.y);
    return m;
}

__device__ __forceinline__ int job_rows(const int* p, int cap)
{
    int n = gld(p);
    return n < 0 ? 0 : (n > cap ? cap : n);
}

__device__ __forceinline__ v4i load_frag(const uint8_t* row, int off)
{
    v4i v = gld(reinterpret_cast<const v4i*>(row + off));
    v ^= (v4i){(int)0x80808080, (int)0x80808080, (int)0x80808080, (int)0x80808080};
    return v;
}

// One workgroup (4 waves) per (job, 128-row F1 block, CHUNK-column F2 chunk); wave w owns
// F1 rows [128 blk + 32 w, +32).  The F2 side is shared: each 32-column tile (4 KB of
// descriptors + metadata) is loaded once per workgroup, one 16-B load per thread, staged
// through a double-buffered LDS tile, and read by every wave as the MFMA A operand (the
// wave's F1 rows are the B operand, in registers): D = F2 tile x F1 rows, so lane l holds F1
// row l & 31 and 16 of the tile's columns.  Tile t+1 is written to LDS and tile t+2 is in
// flight from HBM/L2 while tile t runs its 4 MFMAs and epilogue.  Epilogue per accumulator
// element: dot = acc + 128 sa - 2^21 + 128 sb (one add3), c = ((float)dot * inv|a|) * inv|b|
// (packed muls, two columns at once); then one exact pre-test per tile -- the max of the
// lane's 16 values against its second best -- before the in-order top-2 update, which the wave
// skips when no lane passes.  (The untransposed tile -- D = F1 x F2, 16 rows' top-2 state per
// lane, 154 VGPRs, one wave vote per element -- measured 23 % slower isolated and cost the full
// path 3 %: its 3 waves per SIMD held register file the level blurs needed, r06_w.)
#define MP_ROWS 128
#define MP_LDS_ROW 144
#define VO_MP_MAX_JOBS 256        // jobs per launch (one per thread of the task-table prologue)
#ifndef VO_MP_BLOCKS
#define VO_MP_BLOCKS 5            // workgroups per CU the register budget of k_match_partial<1> is sized for (92 VGPRs)
#endif
#define MP_NBUF 2
#ifndef VO_MP_BSEARCH
// 1: binary search of a task's job in the task table (8 dependent LDS reads); 0: the linear scan
// (up to 255).  k_match_partial 0.623 against 0.667 / 0.679 ms isolated per 256-frame step
// (profiles/r06_r_ab_match_task.txt)
#define VO_MP_BSEARCH 1
#endif
// NB: 32-row F1 sub-blocks per wave (MP_ROWS * NB rows per workgroup); NB = 2 runs two
// independent MFMA chains per tile on the same F2 fragments (half the LDS reads per MFMA)
template <int NB>
__global__ __launch_bounds__(256, NB == 1 ? VO_MP_BLOCKS : 2) void k_match_partial(const MatchJob* __restrict__ jobs, int n_jobs,
                                                       MatchTop2* __restrict__ partial, int row_cap, int n_chunks_cap)
{
    constexpr int ROWS = MP_ROWS * NB;
    // F2 tile rows padded to 144 B (36 dwords): the 32 lanes of a half read 16 B at row l31,
    // so a 128-B stride would put them all on the same banks
    __shared__ __attribute__((aligned(16))) uint8_t bt[MP_NBUF][32 * MP_LDS_ROW];
    __shared__ __attribute__((aligned(16))) int bck[MP_NBUF][32];
    __shared__ __attribute__((aligned(16))) float binb[MP_NBUF][32];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, l31 = lane & 31;
    const int lr = tid >> 3, lseg = tid & 7;              // loader: row lr of the tile, bytes [16 lseg, +16)
    // task table: job j owns tasks [tstart[j], tstart[j+1]); job sizes are read on device
    // (counts of earlier kernels), one thread per job, then a block prefix sum
    __shared__ int tstart[VO_MP_MAX_JOBS + 1], jn1[VO_MP_MAX_JOBS], jnch[VO_MP_MAX_JOBS];
    __shared__ int wsum[4];
    {
        int my = 0;
        if (tid < n_jobs) {
            const int n1 = job_rows(jobs[tid].n1, row_cap), n2 = job_rows(jobs[tid].n2, row_cap);
            const int nch = (n2 + VO_MATCH_CHUNK - 1) / VO_MATCH_CHUNK;
            jn1[tid] = n1; jnch[tid] = nch;
            my = ((n1 + ROWS - 1) / ROWS) * nch;
        }
        int inc = my;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) { const int y = __shfl_up(inc, o); if (lane >= o) inc += y; }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        int before = 0;
        for (int w = 0; w < wave; ++w) before += wsum[w];
        if (tid < n_jobs) tstart[tid] = before + inc - my;
        if (tid == 255) tstart[min(n_jobs, VO_MP_MAX_JOBS)] = before + inc;
        __syncthreads();
    }
    const int total = tstart[n_jobs];
    // (an XCD-contiguous task order -- one job's row blocks, which read the same F2 tiles, on one
    // XCD's L2 -- measured slower: 0.825 against 0.667 ms isolated, profiles/r06_r_ab_match_task.txt)
    for (int t = blockIdx.x; t < total; t += gridDim.x) {       // workgroup-uniform
        int jb = 0;
#if VO_MP_BSEARCH
        // last job whose first task <= t (tstart is nondecreasing; empty jobs repeat a value)
        for (int step = VO_MP_MAX_JOBS / 2; step >= 1; step >>= 1)
            if (jb + step < n_jobs && tstart[jb + step] <= t) jb += step;
#else
        while (jb + 1 < n_jobs && tstart[jb + 1] <= t) ++jb;
#endif
        const int n1 = jn1[jb], nch = jnch[jb];
        const int n2 = job_rows(jobs[jb].n2, row_cap);
        const long rel = t - tstart[jb];
        const MatchJob J = jobs[jb];
        const int blk = (int)(rel / nch), chunk = (int)(rel - (long)blk * nch);
        const int i0 = blk * ROWS + 32 * NB * wave, j0 = chunk * VO_MATCH_CHUNK;
        const int j1 = min(j0 + VO_MATCH_CHUNK, n2);
        // F1 fragments (the MFMA B operand) of sub-block sb: row i0 + 32 sb + l31, bytes
        // [32kk + 16h, +16); the lane's row's sum term and inverse norm; its running top-2 over
        // the F2 columns this lane sees (both halves hold the row)
        v4i a[NB][4];
        int rk1[NB];
        float ina1[NB], best1[NB], second1[NB];
        int bidx1[NB];
#pragma unroll
        for (int sb = 0; sb < NB; ++sb) {
            const int ia = i0 + 32 * sb + l31;
            rk1[sb] = -2097152;
            ina1[sb] = 0.0f;
            if (ia < n1) {
                const int ra = J.idx1 ? gld(J.idx1 + ia) : ia;
                const uint8_t* row = J.d1 + (size_t)ra * VO_DESC_LEN;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) a[sb][kk] = load_frag(row, 32 * kk + 16 * h);
                const DescMeta m = gld_meta(J.m1 + ra);
                rk1[sb] = 128 * m.sum - 2097152;
                ina1[sb] = m.inv_norm;
            } else {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) a[sb][kk] = (v4i){0, 0, 0, 0};
            }
            best1[sb] = -INFINITY; second1[sb] = -INFINITY; bidx1[sb] = -1;
        }
        // loader: column jt + lr (clamped into the chunk; the epilogue masks columns >= j1)
        v4i gv;
        DescMeta gm;
        auto gload = [&](int jt) {
            const int jc = min(jt + lr, j1 - 1);
            const int rb = J.idx2 ? gld(J.idx2 + jc) : jc;
            gv = gld(reinterpret_cast<const v4i*>(J.d2 + (size_t)rb * VO_DESC_LEN + 16 * lseg));
            if (lseg == 0) gm = gld_meta(J.m2 + rb);
        };
        auto lstore = [&](int buf) {                       // stored as b - 128 (the MFMA operand)
            *reinterpret_cast<v4i*>(&bt[buf][lr * MP_LDS_ROW + 16 * lseg]) =
                gv ^ (v4i){(int)0x80808080, (int)0x80808080, (int)0x80808080, (int)0x80808080};
            if (lseg == 0) { bck[buf][lr] = 128 * gm.sum; binb[buf][lr] = gm.inv_norm; }
        };
        // the tile's MFMAs: D = F2 tile (A operand, from LDS) x F1 rows (B operand, registers):
        // lane l holds F1 row i0 + 32 sb + l31 and F2 columns jt + (reg & 3) + 8 (reg >> 2) + 4 h,
        // reg = 0..15 -- ascending in reg, so the lane meets its columns in ascending order
        auto tile_mfma = [&](int bi, v16i (&accv)[NB]) {
            v4i b[4];
            const uint8_t* brow = &bt[bi][l31 * MP_LDS_ROW + 16 * h];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) b[kk] = *reinterpret_cast<const v4i*>(brow + 32 * kk);
#pragma unroll
            for (int sb = 0; sb < NB; ++sb) accv[sb] = (v16i){0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int sb = 0; sb < NB; ++sb) accv[sb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(b[kk], a[sb][kk], accv[sb], 0, 0, 0);
        };
        auto tile_epilogue = [&](int bi, int jt, const v16i (&accv)[NB]) {
#pragma unroll
            for (int sb = 0; sb < NB; ++sb) {
                float cv[16];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    // the column metadata of regs 4q .. 4q+3: tile columns 8q + 4h .. +3 (one
                    // broadcast 16-B read each)
                    const v4i ck4 = *reinterpret_cast<const v4i*>(&bck[bi][8 * q + 4 * h]);
                    const vo_f4 ib4 = *reinterpret_cast<const vo_f4*>(&binb[bi][8 * q + 4 * h]);
#pragma unroll
                    for (int i = 0; i < 4; i += 2) {
                        // c = ((float)dot * inv|a|) * inv|b|, two columns at once as packed f32 muls
                        const vo_f2 fp = vo_f2{(float)(accv[sb][4 * q + i] + rk1[sb] + ck4[i]),
                                               (float)(accv[sb][4 * q + i + 1] + rk1[sb] + ck4[i + 1])};
                        const vo_f2 cp = (fp * vo_f2{ina1[sb], ina1[sb]}) * vo_f2{ib4[i], ib4[i + 1]};
                        cv[4 * q + i] = cp.x;
                        cv[4 * q + i + 1] = cp.y;
                    }
                }
                if (jt + 32 > j1) {                        // wave-uniform: the ragged last tile
#pragma unroll
                    for (int reg = 0; reg < 16; ++reg)
                        cv[reg] = jt + (reg & 3) + 8 * (reg >> 2) + 4 * h < j1 ? cv[reg] : -INFINITY;
                }
                // exact pre-test: a tile whose 16 values are all <= the lane's second best changes
                // nothing (the update below leaves best / second / index as they are for c <= second).
                // (An integer pre-test before the float conversion -- the tile's dots against
                // floor(second / inv|a| / max inv|b| (1 - 2^-16)) -- was bit-exact but 27 % slower:
                // the bound with the tile's largest inv|b| rarely clears a whole wave, so it only
                // added work, profiles/r06_zd_ab_match_ibound.txt)
                float m = fmaxf(fmaxf(fmaxf(cv[0], cv[1]), fmaxf(cv[2], cv[3])), fmaxf(fmaxf(cv[4], cv[5]), fmaxf(cv[6], cv[7])));
                m = fmaxf(m, fmaxf(fmaxf(fmaxf(cv[8], cv[9]), fmaxf(cv[10], cv[11])), fmaxf(fmaxf(cv[12], cv[13]), fmaxf(cv[14], cv[15]))));
                if (__builtin_amdgcn_ballot_w64(m > second1[sb])) {
#pragma unroll
                    for (int reg = 0; reg < 16; ++reg) {
                        const float c = cv[reg];
                        const bool g1 = c > best1[sb], g2 = c > second1[sb];
                        second1[sb] = g1 ? best1[sb] : (g2 ? c : second1[sb]);
                        best1[sb] = g1 ? c : best1[sb];
                        bidx1[sb] = g1 ? jt + (reg & 3) + 8 * (reg >> 2) + 4 * h : bidx1[sb];
                    }
                }
            }
        };
        // (a three-tile pipeline -- tile t+1's MFMAs issued before tile t's epilogue, 116 VGPRs at 4
        // waves per SIMD -- measured slower: 0.453 against 0.420 ms isolated, the 1080p block 0.121
        // against 0.129 of i8 peak, profiles/r06_za_ab_match_pipe_grid.txt)
        gload(j0);
        __syncthreads();                                   // previous task's readers are done with bt
        lstore(0);
        if (j0 + 32 < j1) gload(j0 + 32);
        int buf = 0;
        for (int jt = j0; jt < j1; jt += 32, buf ^= 1) {
            __syncthreads();                               // tile jt visible; tile jt-32's buffer free
            if (jt + 32 < j1) {
                lstore(buf ^ 1);                           // tile jt+32 (loaded one iteration ago)
                if (jt + 64 < j1) gload(jt + 64);
            }
            v16i accv[NB];
            tile_mfma(buf, accv);
            tile_epilogue(buf, jt, accv);
        }
#pragma unroll
        for (int sb = 0; sb < NB; ++sb) {
            const float ob = __shfl_xor(best1[sb], 32), os = __shfl_xor(second1[sb], 32);
            const int oi = __shfl_xor(bidx1[sb], 32);
            top2c_merge(best1[sb], bidx1[sb], second1[sb], ob, oi, os);
            const int row = i0 + 32 * sb + l31;
            if (h == 0 && row < n1) {
                MatchTop2 mt;
                mt.best = best1[sb]; mt.idx = bidx1[sb]; mt.second = second1[sb]; mt.pad = 0;
                partial[((size_t)jb * n_chunks_cap + chunk) * row_cap + row] = mt;
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
            if (base < (uint32_t)J.cap) { gst(J.out_i + base, r); gst(J.out_j + base, i); }
            base++;
        }
    }
    if (tid == 0) gst(J.out_n, (int)(total < (uint32_t)J.cap ? total : (uint32_t)J.cap));
}

// One 256-thread workgroup per job: k_match_merge + k_match_compact (+ k_compose) in one
// launch.  Rows go in tiles of 256 in ascending F1 order (coalesced partial reads): thread t
// merges row 256 k + t over the F2 chunks and applies MatchThreshold / MaxRatio; the tile's
// accepted rows are placed by a block prefix sum after the running count, so the pairs come
// out in ascending F1 order exactly as k_match_compact writes them.  With `compose` (a
// tracking step of find_remaining_points), the workgroup then applies that step's index
// composition to its frame's lists (k_compose, VO.m:287-333) -- so a tracking step is two
// launches (partial, finish) instead of four.
__global__ __launch_bounds__(256) void k_match_finish(const MatchJob* __restrict__ jobs, const MatchTop2* __restrict__ partial,
                                                      int row_cap, int n_chunks_cap, float T, float max_ratio,
                                                      MatchCompose cp, int with_compose)
{
    __shared__ uint32_t wsum[4];
    const int jb = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const MatchJob J = jobs[jb];
    const int n1 = job_rows(J.n1, row_cap), n2 = job_rows(J.n2, row_cap);
    const int nch = (n2 + VO_MATCH_CHUNK - 1) / VO_MATCH_CHUNK;
    const MatchTop2* P = partial + (size_t)jb * n_chunks_cap * row_cap;
    uint32_t base = 0;
    for (int r0 = 0; r0 < n1; r0 += 256) {                       // block-uniform
        const int r = r0 + tid;
        int acc = -1;
        if (r < n1) {
            float b = -INFINITY, s = -INFINITY;
            int i = -1;
            for (int c = 0; c < nch; ++c) {
                const MatchTop2 m = P[(size_t)c * row_cap + r];
                top2c_merge(b, i, s, m.best, m.idx, m.second);
            }
            const float bs = 2.0f - 2.0f * b, ss = 2.0f - 2.0f * s;      // SSD of best / second best
            acc = (i >= 0 && bs <= T && (bs / ss) <= max_ratio) ? i : -1;
        }
        const unsigned long long bal = __builtin_amdgcn_ballot_w64(acc >= 0);
        if (lane == 0) wsum[wid] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t before = base;
        for (int w = 0; w < wid; ++w) before += wsum[w];
        const uint32_t pos = before + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        if (acc >= 0 && pos < (uint32_t)J.cap) { gst(J.out_i + pos, r); gst(J.out_j + pos, acc); }
        base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();                                          // wsum reused by the next tile
    }
    const int n_out = (int)(base < (uint32_t)J.cap ? base : (uint32_t)J.cap);
    if (tid == 0) gst(J.out_n, n_out);
    if (!with_compose) return;
    __syncthreads();                                              // the pairs are visible to the block
    // k_compose of tracking step cp.step for frame f = jb
    const int f = cp.f0 + jb, K = cp.kp_cap, M = cp.M, st = cp.step;
    int* L = cp.lists + (size_t)f * TL_COUNT * K;
    const int pp = f ? f - 1 : M;
    const int n = min(n_out, K);
    for (int k = tid; k < n; k += 256) {
        const int i = gld(J.out_i + k), j = gld(J.out_j + k);
        if (st == 0) {
            L[TL_OL1 * K + k] = cp.pair_i[(size_t)pp * K + j];
            L[TL_OR1 * K + k] = cp.pair_j[(size_t)pp * K + j];
            L[TL_CL * K + k] = i;
        } else if (st == 1) {
            L[TL_OL2 * K + k] = L[TL_OL1 * K + j];
            L[TL_OR2 * K + k] = L[TL_OR1 * K + j];
            L[TL_CR * K + k] = i;
        } else if (st == 2) {
            L[TL_CL2 * K + k] = L[TL_CL * K + i];
            L[TL_CR2 * K + k] = L[TL_CR * K + j];
        } else {
            L[TL_OLF * K + k] = L[TL_OL2 * K + j];
            L[TL_ORF * K + k] = L[TL_OR2 * K + j];
            L[TL_CLF * K + k] = L[TL_CL2 * K + i];
            L[TL_CRF * K + k] = L[TL_CR2 * K + i];
        }
    }
    if (tid == 0) cp.list_n[4 * f + st] = n;
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

#ifndef VO_MATCH_FINISH
#define VO_MATCH_FINISH 1         // 0: k_match_merge + k_match_compact (+ k_compose) as separate launches
#endif
void match_launch(const MatchBuffers& b, const MatchJob* d_jobs, int n_jobs, const vo_match_params& p, hipStream_t s,
                  const MatchCompose* compose)
{
    if (n_jobs <= 0) return;
    if (n_jobs > VO_MP_MAX_JOBS) {                       // the task table holds VO_MP_MAX_JOBS jobs
        MatchCompose rest;
        if (compose) {                                   // frames VO_MP_MAX_JOBS.. of a tracking step
            rest = *compose;
            rest.f0 += VO_MP_MAX_JOBS;
        }
        match_launch(b, d_jobs, VO_MP_MAX_JOBS, p, s, compose);
        match_launch(match_view(b, VO_MP_MAX_JOBS), d_jobs + VO_MP_MAX_JOBS, n_jobs - VO_MP_MAX_JOBS, p, s,
                     compose ? &rest : nullptr);
        return;
    }
#ifndef VO_TRACK_GRID
#define VO_TRACK_GRID 256         // k_match_partial workgroups for the tracking steps (stereo: 2048); 256 measured +1 % on the
                                  // full path over 2048 (fewer resident beside the SIFT streams), 64 / 128 / 512 / 8192 not
                                  // (profiles/r06_lm_ab_track_grid.txt)
#endif
#ifndef VO_STEREO_GRID
#define VO_STEREO_GRID 2048
#endif
    // (two F1 sub-blocks per wave for the stereo matches, k_match_partial<2> at 165 VGPRs: configs[1]
    // -1 %, the 1080p block 0.123 against 0.128 of i8 peak, profiles/r06_y_ab_match_nb2_chunk.txt)
    VO_LAUNCH_NAMED("k_match_partial", k_match_partial<1>, dim3(compose ? VO_TRACK_GRID : VO_STEREO_GRID), dim3(256), 0, s,
                    d_jobs, n_jobs, b.partial, b.row_cap, b.n_chunks);
    if (VO_MATCH_FINISH) {
        MatchCompose cp{};
        if (compose) cp = *compose;
        VO_LAUNCH(k_match_finish, dim3(n_jobs), dim3(256), 0, s, d_jobs, (const MatchTop2*)b.partial, b.row_cap, b.n_chunks,
                  p.match_threshold * 0.04f, p.max_ratio, cp, compose ? 1 : 0);
        return;
    }
    VO_LAUNCH(k_match_merge, dim3((b.row_cap + 255) / 256, n_jobs), dim3(256), 0, s, d_jobs, (const MatchTop2*)b.partial,
              b.res, b.row_cap, b.n_chunks, p.match_threshold * 0.04f, p.max_ratio);
    VO_LAUNCH(k_match_compact, dim3(n_jobs), dim3(1024), 0, s, d_jobs, (const int*)b.res, b.row_cap);
}

void match_launch(const MatchBuffers& b, const MatchJob* d_jobs, int n_jobs, const vo_match_params& p, hipStream_t s)
{
    match_launch(b, d_jobs, n_jobs, p, s, nullptr);
}

// single-precision descriptor matrix (MATLAB's extractFeatures output: n x 128 single, integer
// values 0..255) -> packed u8 rows.  col_major: element (i, k) at F[i + k * ld] (MATLAB's own
// layout, so a MEX gateway passes mxGetSingles() without a copy); else F[i * ld + k].  One
// thread per element, the row index fastest for column-major input (coalesced reads).  A value
// that is not an integer in [0, 255] raises *bad.
__global__ __launch_bounds__(256) void k_pack_f32_desc(const float* __restrict__ F, int n, int ld, int col_major,
                                                       uint8_t* __restrict__ out, int* __restrict__ bad)
{
    const long total = (long)n * VO_DESC_LEN;
    for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
        int i, k;
        float v;
        if (col_major) { i = (int)(t % n); k = (int)(t / n); v = F[(size_t)k * ld + i]; }
        else { i = (int)(t / VO_DESC_LEN); k = (int)(t % VO_DESC_LEN); v = F[(size_t)i * ld + k]; }
        const bool ok = v >= 0.0f && v <= 255.0f && v == rintf(v);
        out[(size_t)i * VO_DESC_LEN + k] = ok ? (uint8_t)v : 0;
        if (!ok) *bad = 1;
    }
}

void pack_f32_desc_launch(const float* F, int n, int ld, int col_major, uint8_t* out, int* bad, hipStream_t s)
{
    if (n <= 0) return;
    long total = (long)n * VO_DESC_LEN;
    int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    VO_LAUNCH(k_pack_f32_desc, dim3(blocks), dim3(256), 0, s, F, n, ld, col_major, out, bad);
}

// ---------------------------------------------------------------------------
// matchFeatures on general single-precision features (vo_match_f32 when the rows are not
// u8-valued SIFT descriptors).  Spec, restated by the oracle's oracle_match_f32 (vo_ref.c):
//   a_k = f_k / nrm (0 if nrm == 0), nrm = sqrtf(fmaf chain of f_k^2 over k = 0..127);
//   ssd(i, j) = fmaf chain of (a_k - b_k)^2 over k = 0..127;
//   best / second = smallest / second smallest ssd of row i (multiset; ties -> lowest j);
//   accept best <= 0.04 * MatchThreshold and best / second <= MaxRatio (the u8 path's rule).
// k_f32_norm: one thread per row; F2 rows are written transposed ([128][n2]) so k_match_f32's
// lanes (one F2 column each) read them coalesced.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_f32_norm(const float* __restrict__ F, int n, int ld, int col_major, int transpose,
                                                  float* __restrict__ out)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    auto at = [&](int k) { return col_major ? F[(size_t)k * ld + i] : F[(size_t)i * ld + k]; };
    float n2 = 0.0f;
    for (int k = 0; k < VO_DESC_LEN; ++k) { const float v = at(k); n2 = fmaf(v, v, n2); }
    const float nrm = sqrtf(n2);
    for (int k = 0; k < VO_DESC_LEN; ++k) {
        const float v = nrm > 0.0f ? at(k) / nrm : 0.0f;
        out[transpose ? (size_t)k * n + i : (size_t)i * VO_DESC_LEN + k] = v;
    }
}

// one wave per F1 row (grid-stride): the row in LDS (broadcast reads), lane l scores columns
// l, l + 64, ... with the sequential fmaf chain, keeps its own top-2, and the wave merges the
// 64 top-2s with the order-free (value, index) rule; res[i] = accepted column or -1
__global__ __launch_bounds__(64) void k_match_f32(const float* __restrict__ A, int n1, const float* __restrict__ BT, int n2,
                                                  float T, float max_ratio, int* __restrict__ res)
{
    __shared__ float a[VO_DESC_LEN];
    const int lane = threadIdx.x;
    for (int i = blockIdx.x; i < n1; i += gridDim.x) {
        a[lane] = A[(size_t)i * VO_DESC_LEN + lane];
        a[lane + 64] = A[(size_t)i * VO_DESC_LEN + lane + 64];
        __syncthreads();
        float best = INFINITY, second = INFINITY;
        int bidx = -1;
        for (int j = lane; j < n2; j += 64) {
            float ssd = 0.0f;
            for (int k = 0; k < VO_DESC_LEN; ++k) {
                const float d = a[k] - BT[(size_t)k * n2 + j];
                ssd = fmaf(d, d, ssd);
            }
            if (ssd < best) { second = best; best = ssd; bidx = j; }
            else if (ssd < second) second = ssd;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const float b2 = __shfl_xor(best, off), s2 = __shfl_xor(second, off);
            const int i2 = __shfl_xor(bidx, off);
            const float ns = fminf(fminf(second, s2), fmaxf(best, b2));
            if (i2 >= 0 && (bidx < 0 || b2 < best || (b2 == best && i2 < bidx))) { best = b2; bidx = i2; }
            second = ns;
        }
        if (lane == 0) res[i] = (bidx >= 0 && best <= T && best / second <= max_ratio) ? bidx : -1;
        __syncthreads();
    }
}

void match_f32_launch(const float* F1, int n1, int ld1, const float* F2, int n2, int ld2, int col_major, float* A, float* BT,
                      int* res, const vo_match_params& p, hipStream_t s)
{
    if (n1 <= 0) return;
    VO_LAUNCH(k_f32_norm, dim3((n1 + 255) / 256), dim3(256), 0, s, F1, n1, ld1, col_major, 0, A);
    if (n2 > 0) VO_LAUNCH(k_f32_norm, dim3((n2 + 255) / 256), dim3(256), 0, s, F2, n2, ld2, col_major, 1, BT);
    VO_LAUNCH(k_match_f32, dim3(std::min(n1, 8192)), dim3(64), 0, s, A, n1, BT, n2, p.match_threshold * 0.04f, p.max_ratio,
              res);
}

void desc_meta_launch(const uint8_t* desc, DescMeta* meta, int n, hipStream_t s)
{
    if (n <= 0) return;
    int blocks = (n + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    VO_LAUNCH(k_desc_meta, dim3(blocks), dim3(256), 0, s, desc, meta, n);
}

}  // namespace vo
