// octave.hip — one octave's Gaussian levels 1..5, its extremum test and the next octave's base
// in a single pass (k_octave): detectSIFTFeatures' scale space + DoG extrema, VO.m:79-80.
//
// The per-level path (sift.hip: k_blur_stream per level, k_ext_stream, k_down) moves every
// octave pixel through HBM ~16 times: each level blur reads G_{i-1} and writes G_i (8 B per
// pixel and level), the extremum test re-reads all six levels (24 B), k_down re-reads G_3.
// Here one workgroup streams a vertical strip of the octave top to bottom and keeps the
// cascade on chip:
//   * 5 level waves, one per Gaussian level i = 1..5 (radius r_i), each over a 256-column
//     window (64 lanes x 4 columns) with its vertical ring of row-pass results in registers
//     (the k_blur_stream scheme).  Level 1 streams G_0 from HBM; level i >= 2 takes G_{i-1}
//     rows from an LDS history written by level i-1.  Each level writes its owned columns of
//     G_i to HBM (the feature stages read them), G_i rows to its LDS history, and
//     D_{i-1} = G_i - G_{i-1} rows to a DoG history; level 3 also writes the next octave's
//     base (G_3 decimated by 2).
//   * 1 extremum wave: per row, D_0..D_4 rows from the DoG histories, horizontal 3-max/min
//     (4 columns per lane, outer neighbours by DPP), a 3-row register window, the 26-neighbour
//     test of layers 1..3, words OR-ed into the mask in k_ext_stream's (even, odd) layout.
// Waves run decoupled, synchronised by per-history counters in LDS (rows emitted, rows
// released): a level emits row y only into a free slot, a consumer reads row q only once it
// has been emitted.  HBM traffic per octave pixel: G_0 read ~1.5x (window overlap) + G_1..G_5
// written once = ~26 B, against ~66 B for the per-level kernels.
//
// Strips: the window covers columns [X, X + 256); level i is exact on a range that shrinks by
// r_i each side, so after r_1 + ... + r_5 = 42 (+2 for the 4-column alignment) the strip owns
// 168 columns [X + 44, X + 212), with one column each side for the extremum test.  Image edges:
// reflect-101 on columns at read time (the consumer reads the reflected column of the
// producer's row), on rows through the reflected input sequence (as k_blur_stream).
// Per-output arithmetic equals the oracle's blur exactly: acc = k0 * s0; acc = fmaf(kj, s[-j] +
// s[+j], acc) for the row pass, then the same for the column pass -- bit-identical planes.
#include "vo_internal.h"
#include <cstring>
#include <cstdio>
#include <type_traits>
#include <utility>

namespace vo {

namespace {

typedef float of_f2 __attribute__((ext_vector_type(2)));
typedef float of_f4 __attribute__((ext_vector_type(4)));

constexpr int OF_W = 256;                    // window columns
constexpr int OF_H = 44;                     // window columns left of the owned range
constexpr int OF_S = 168;                    // owned columns per strip
constexpr int OF_G = 16;                     // guard floats each side of a G history row
constexpr int OF_RW = OF_W + 2 * OF_G;       // G history row (floats)
constexpr int OF_DL = 10, OF_DN = 44;        // DoG rows keep lanes [10, 54): columns [X+40, X+216)
constexpr int OF_DW = 4 * OF_DN;
constexpr int OF_OL = 11, OF_ON = 42;        // owned lanes [11, 53)
constexpr int OF_P = 4;                      // ring block of the LDS-fed levels
constexpr int OF_P1 = 8;                     // ring block (= prefetch depth) of level 1 (HBM-fed)
constexpr int OF_WAVES = 8;                  // 5 level waves + 3 extremum waves (one per layer)
constexpr int OF_DSLACK = 12;                // DoG history rows beyond the minimum (decoupling)

// LDS counters
enum : int { C_PROD = 0,        // + i (1..5): rows of G_i emitted (and D_{i-1})
             C_REL = 7,         // + i (1..4): rows of G_i released by level i+1
             C_EXT = 12,        // + l - 1 (l = 1..3): DoG rows released by the extremum wave of layer l
             C_N = 16 };
static_assert(C_PROD + 5 < C_REL + 1 && C_REL + 4 < C_EXT && C_EXT + 2 < C_N, "LDS counter slots overlap");

constexpr int of_rh(int r) { return (r + 3) / 4 * 4; }

template <int R1, int R2, int R3, int R4, int R5>
struct OfCfg {
    static constexpr int r(int i) { return i == 1 ? R1 : i == 2 ? R2 : i == 3 ? R3 : i == 4 ? R4 : R5; }
    // G_i history depth (i = 1..4): the consumer (level i+1, radius r, block P) holds at most
    // r + P rows; +1 of slack
    static constexpr int dg(int i) { return r(i + 1) + OF_P + 1; }
    // rows of G_i beyond row t that the extremum test of layer l needs to load row t
    // (D_{l+1} row t = G_{l+2} row t <- G_{l+1} row t + r(l+2) <- ...):
    // lead(l, l+2) = 0, lead(l, i) = lead(l, i+1) + r(i+1)
    static constexpr int lead(int l, int i)
    {
        int v = 0;
        for (int j = i + 1; j <= l + 2; ++j) v += r(j);
        return v;
    }
    // D_m history depth (m = 0..4, written with G_{m+1}; read by the layers l with |l - m| <= 1):
    // the rows a consumer has not loaded yet, max over its consumers, + slack
    static constexpr int dd(int m)
    {
        int v = 1;
        for (int l = 1; l <= 3; ++l)
            if (l - 1 <= m && m <= l + 1 && lead(l, m + 1) + 1 > v) v = lead(l, m + 1) + 1;
        return v + OF_DSLACK;
    }
    static constexpr int g_off(int i)                   // G_i history (i = 1..4; 5 = end of them)
    {
        int v = 0;
        for (int j = 1; j < i; ++j) v += dg(j) * OF_RW;
        return v;
    }
    static constexpr int d_off(int m)                   // D_m history (m = 0..4; 5 = end of them)
    {
        int v = g_off(5);
        for (int j = 0; j < m; ++j) v += dd(j) * OF_DW;
        return v;
    }
    static constexpr int lds_floats() { return d_off(5) + C_N; }
    static constexpr int ctr_off = d_off(5);
    static_assert(lds_floats() * 4 <= 160 * 1024, "k_octave LDS exceeds the CU's 160 KB");
};

__device__ __forceinline__ int of_load(const int* p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// wave-uniform spin until *p >= v.  Bounded: a wait that outlives ~2^24 polls (about a second,
// orders of magnitude beyond any legitimate wait) gives up, so a scheduling bug can only corrupt
// the result, never hang the device
__device__ __forceinline__ void of_wait(const int* p, int v)
{
    for (int it = 0; of_load(p) < v && it < (1 << 24); ++it) __builtin_amdgcn_s_sleep(1);
}
// the same with a wave-private cache of the counter: no LDS access while the last value seen
// already satisfies the request (producers usually run ahead)
#ifdef OF_STATS
// diagnostic build: per-wave cycles spent in each kind of wait (k_octave stats, octave 0)
// [wave][kind]: kind 0 input wait, 1 G-slot wait, 2 DoG-slot wait, 3 whole role
__device__ unsigned long long of_stat[8 * 4];
#define OF_STAT_BEGIN const long long t0_ = clock64();
#define OF_STAT_END(k) if ((threadIdx.x & 63) == 0) atomicAdd(&of_stat[(threadIdx.x >> 6) * 4 + (k)], (unsigned long long)(clock64() - t0_));
#else
#define OF_STAT_BEGIN
#define OF_STAT_END(k)
#endif
__device__ __forceinline__ void of_wait_c(const int* p, int v, int& seen, int kind = 0)
{
    if (seen >= v) return;
    OF_STAT_BEGIN
    for (int it = 0; it < (1 << 24); ++it) {
        seen = of_load(p);
        if (seen >= v) break;
        __builtin_amdgcn_s_sleep(1);
    }
    (void)kind;
    OF_STAT_END(kind)
}
// reflect-101 for |overshoot| < n (one fold; every caller's range is well inside that)
__device__ __forceinline__ int of_refl(int p, int n) { return p < 0 ? -p : p >= n ? 2 * n - 2 - p : p; }
// publish *p = v after this wave's earlier LDS writes
__device__ __forceinline__ void of_publish(int* p, int v)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

enum : int { OF_SHL1 = 0x130, OF_SHR1 = 0x138 };
template <int CTRL>
__device__ __forceinline__ float of_dpp(float old, float src)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ unsigned long long of_spread32(uint32_t x)
{
    unsigned long long v = x;
    v = (v | v << 16) & 0x0000FFFF0000FFFFull;
    v = (v | v << 8) & 0x00FF00FF00FF00FFull;
    v = (v | v << 4) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | v << 2) & 0x3333333333333333ull;
    v = (v | v << 1) & 0x5555555555555555ull;
    return v;
}

template <typename F, int... I>
__device__ __forceinline__ void of_for_impl(F&& f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void of_for(F&& f) { of_for_impl(f, std::make_integer_sequence<int, N>{}); }

}  // namespace

// the workgroup's dynamic LDS (histories + counters), visible to the role functions by name so
// they address it as LDS (the roles are separate functions: each has its own register budget)
extern __shared__ __attribute__((aligned(16))) float of_lds[];

// ---------------------------------------------------------------------------------------------
// One level wave: Gaussian level LV (radius RAD) of one strip.
// ---------------------------------------------------------------------------------------------
template <class CFG, int LV, bool EDGE>
__device__ __forceinline__ void of_level(const float* __restrict__ g0, float* __restrict__ gout,
                                                   float* __restrict__ nbase, const float* __restrict__ taps, int R, int C,
                                                   int pitch, int Rn, int Cn, int pitchn, int X)
{
    float* const lds = of_lds;
    int* const ctr = reinterpret_cast<int*>(of_lds + CFG::ctr_off);
    constexpr int RAD = CFG::r(LV);
    constexpr int P = LV == 1 ? OF_P1 : OF_P;
    constexpr int RH = of_rh(RAD);
    constexpr int NQ = 1 + 2 * RH / 4;
    constexpr int NW = 4 * NQ;
    constexpr int NR = 2 * RAD + P;
    constexpr int F = (2 * RAD + P - 1) / P * P;          // ring-fill steps (no output)
    constexpr int E = F - 2 * RAD;                        // extra reflected rows above row 0
    const int lane = threadIdx.x & 63;
    const int TH = (R + P - 1) / P * P;
    const int xl = X + 4 * lane;                          // this lane's first column
    float k[RAD + 1];
#pragma unroll
    for (int j = 0; j <= RAD; ++j) k[j] = taps[LV * 16 + j];
    constexpr int DGI = LV <= 4 ? CFG::dg(LV) : 1, DGP = LV >= 2 ? CFG::dg(LV - 1) : 1, DDP = CFG::dd(LV - 1);
    constexpr int GOFF = LV <= 4 ? CFG::g_off(LV) : 0, GOFFP = LV >= 2 ? CFG::g_off(LV - 1) : 0, DOFF = CFG::d_off(LV - 1);
    float* ghist = lds + GOFF;                            // this level's G history (LV <= 4)
    const float* gin = lds + GOFFP;                       // the previous level's (LV >= 2)
    float* dhist = lds + DOFF;
    const bool dlane = lane >= OF_DL && lane < OF_DL + OF_DN;
    const bool own = lane >= OF_OL && lane < OF_OL + OF_ON && xl < C;
    int cm[4];                                            // level 1, edge strips: reflected columns
#pragma unroll
    for (int i = 0; i < 4; ++i) cm[i] = of_refl(xl + i, C);
    int seen_in = 0, seen_rel = 0, seen_ext[3] = {0, 0, 0};   // cached counters (see of_wait_c)

    of_f4 pf[LV == 1 ? P : 1];                            // level 1: prefetched G_0 rows
    of_f4 graw[LV == 1 ? NR : 1];                         // level 1: the ring's G_0 rows as read (for D_0)
    of_f2 H[NR][2];

    auto load_g0 = [&](int kk) -> of_f4 {
        const int y = of_refl(kk - RAD - E, R);
        const float* rp = g0 + (size_t)y * pitch;
        if constexpr (!EDGE) return *reinterpret_cast<const of_f4*>(rp + xl);
        return of_f4{rp[cm[0]], rp[cm[1]], rp[cm[2]], rp[cm[3]]};
    };
    if constexpr (LV == 1) {
        of_for<P>([&](auto uc) { pf[decltype(uc)::value] = load_g0(decltype(uc)::value); });
    }

    auto block = [&](int kk0) {
        of_for<P>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            const int kk = kk0 + u;
            float w[NW];
            if constexpr (LV == 1) {
                const of_f4 vm = pf[u];
                graw[2 * RAD + u] = vm;
                // unconditional (clamped) prefetch: a conditional VMEM load makes the compiler's
                // waitcnt tracking fall back to vmcnt(0) at every block, serialising the stream
                pf[u] = load_g0(min(kk + P, F + TH - 1));
                // neighbours by whole-wave DPP shifts (the outer lanes get values they never use)
#pragma unroll
                for (int i = 0; i < NW; ++i) w[i] = 0.0f;
                float Lf[4], Rt[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) w[RH + c] = Lf[c] = Rt[c] = vm[c];
#pragma unroll
                for (int s = 1; s <= RH / 4; ++s) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        if (c >= s * 4 - RAD) {
                            Lf[c] = of_dpp<OF_SHR1>(Lf[c], Lf[c]);
                            w[RH - s * 4 + c] = Lf[c];
                        }
                        if (3 - c >= s * 4 - RAD) {
                            Rt[c] = of_dpp<OF_SHL1>(Rt[c], Rt[c]);
                            w[RH + s * 4 + c] = Rt[c];
                        }
                    }
                }
            } else {
                const int q = of_refl(kk - RAD - E, R);
                of_wait_c(ctr + C_PROD + LV - 1, q + 1, seen_in);
                const float* rp = gin + (q % DGP) * OF_RW + OF_G;
                if constexpr (!EDGE) {
#pragma unroll
                    for (int t = 0; t < NQ; ++t) {
                        const of_f4 v = *reinterpret_cast<const of_f4*>(rp + 4 * lane - RH + 4 * t);
#pragma unroll
                        for (int c = 0; c < 4; ++c) w[4 * t + c] = v[c];
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < NW; ++i) {
                        int col = xl - RH + i;
                        col = of_refl(col, C);
                        w[i] = rp[col - X];
                    }
                }
            }
            // row pass on column pairs (x, x+1), x = RH + 2c: packed v_pk_fma (IEEE per element)
            of_f2 Ev[NW / 2], Ov[NW / 2 - 1];
#pragma unroll
            for (int m = 0; m < NW / 2; ++m) Ev[m] = of_f2{w[2 * m], w[2 * m + 1]};
#pragma unroll
            for (int m = 0; m < NW / 2 - 1; ++m) Ov[m] = __builtin_shufflevector(Ev[m], Ev[m + 1], 1, 2);
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int x = RH + 2 * c;
                of_f2 acc = of_f2{k[0], k[0]} * Ev[x / 2];
#pragma unroll
                for (int j = 1; j <= RAD; ++j) {
                    const of_f2 lo = (j & 1) ? Ov[(x - j - 1) / 2] : Ev[(x - j) / 2];
                    const of_f2 hi = (j & 1) ? Ov[(x + j - 1) / 2] : Ev[(x + j) / 2];
                    acc = __builtin_elementwise_fma(of_f2{k[j], k[j]}, lo + hi, acc);
                }
                H[2 * RAD + u][c] = acc;
            }
            const int y = kk - F;
            if (y >= 0 && y < R) {
                of_f4 g;
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    of_f2 acc = of_f2{k[0], k[0]} * H[u + RAD][c];
#pragma unroll
                    for (int j = 1; j <= RAD; ++j)
                        acc = __builtin_elementwise_fma(of_f2{k[j], k[j]}, H[u + RAD - j][c] + H[u + RAD + j][c], acc);
                    g[2 * c] = acc.x;
                    g[2 * c + 1] = acc.y;
                }
                // free slots: G_LV row y - dg released by level LV+1, D rows by the extremum wave
                if constexpr (LV <= 4) of_wait_c(ctr + C_REL + LV, y - DGI + 1, seen_rel, 1);
                // DoG slot of row y: every extremum wave reading D_{LV-1} (layers LV-2 .. LV)
                // has loaded row y - DDP
#pragma unroll
                for (int l = 1; l <= 3; ++l)
                    if (l - 1 <= LV - 1 && LV - 1 <= l + 1) of_wait_c(ctr + C_EXT + l - 1, y - DDP + 1, seen_ext[l - 1], 2);
                // D_{LV-1}(y) = G_LV(y) - G_{LV-1}(y) on the DoG lanes
                if (dlane) {
                    of_f4 gp = of_f4{0.0f, 0.0f, 0.0f, 0.0f};
                    if constexpr (LV == 1) {
                        gp = graw[u + RAD];                       // G_0 row y, kept from its read (no reload)
                    } else {
                        gp = *reinterpret_cast<const of_f4*>(gin + (y % DGP) * OF_RW + OF_G + 4 * lane);
                    }
                    *reinterpret_cast<of_f4*>(dhist + (y % DDP) * OF_DW + 4 * (lane - OF_DL)) = g - gp;
                }
                if constexpr (LV <= 4)
                    *reinterpret_cast<of_f4*>(ghist + (y % DGI) * OF_RW + OF_G + 4 * lane) = g;
                if (own) __builtin_nontemporal_store(g, reinterpret_cast<of_f4*>(gout + (size_t)y * pitch + xl));
                if constexpr (LV == 3) {
                    // the next octave's base: G_3 decimated by 2 (even rows, even columns)
                    if (nbase && own && !(y & 1) && (y >> 1) < Rn && (xl >> 1) < Cn)
                        *reinterpret_cast<of_f2*>(nbase + (size_t)(y >> 1) * pitchn + (xl >> 1)) =
                            of_f2{g.x, g.z};
                }
                of_publish(ctr + C_PROD + LV, y + 1);
            }
        });
        if constexpr (LV >= 2) {
            // once per block: rows of G_{LV-1} no future step reads -- below the next output
            // row (its D) and below the next input rows (the reflected bottom rows reach down
            // to R - RAD - P)
            const int kn = kk0 + P;
            const int rel = kn >= F + TH ? R : max(0, min(kn - F, R - RAD - P));
            of_publish(ctr + C_REL + LV - 1, rel);
        }
#pragma unroll
        for (int q = 0; q < 2 * RAD; ++q) {
            H[q][0] = H[q + P][0];
            H[q][1] = H[q + P][1];
            if constexpr (LV == 1) graw[q] = graw[q + P];
        }
    };
#pragma unroll 1
    for (int kk0 = 0; kk0 < F + TH; kk0 += P) block(kk0);
}

// ---------------------------------------------------------------------------------------------
// An extremum wave: k_ext_stream's test of one layer on the DoG histories, 4 columns per lane.
// Layer LY reads D_{LY-1}, D_LY, D_{LY+1}; it loads row rho once G_{LY+2} row rho is emitted and
// releases it at once (its horizontal 3-max/min and centre stay in a 3-row register window).
// ---------------------------------------------------------------------------------------------
template <class CFG, int LY>
__device__ __forceinline__ void of_extrema(unsigned long long* __restrict__ mrow, int wb, int wr, float thr, int R, int C,
                                           int X, int own0)
{
    float* const lds = of_lds;
    int* const ctr = reinterpret_cast<int*>(of_lds + CFG::ctr_off);
    constexpr int DOFFS[3] = {CFG::d_off(LY - 1), CFG::d_off(LY), CFG::d_off(LY + 1)};
    constexpr int DDS[3] = {CFG::dd(LY - 1), CFG::dd(LY), CFG::dd(LY + 1)};
    constexpr int W = 3, B = VO_SIFT_BORDER;
    const int lane = threadIdx.x & 63;
    const int xl = X + 4 * lane;
    const bool dlane = lane >= OF_DL && lane < OF_DL + OF_DN;
    const int c_lo = max(own0, B), c_hi = min(own0 + OF_S, C - B);     // tested columns [c_lo, c_hi)
    bool inc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) inc[j] = xl + j >= c_lo && xl + j < c_hi;
    of_f4 hmx[W][3], hmn[W][3], dc[W];
    int seen = 0;

    // row rho of D_{LY-1}, D_LY, D_{LY+1} into window slot SL; then release it
    auto load = [&](int rho, auto sl_c) {
        constexpr int SL = decltype(sl_c)::value;
        of_wait_c(ctr + C_PROD + LY + 2, rho + 1, seen);    // G_{LY+2} row rho emitted -> D_{LY+1} row rho
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            of_f4 v = of_f4{0.0f, 0.0f, 0.0f, 0.0f};
            if (dlane) v = *reinterpret_cast<const of_f4*>(lds + DOFFS[m] + (rho % DDS[m]) * OF_DW + 4 * (lane - OF_DL));
            const float lf = of_dpp<OF_SHR1>(v.x, v.w), rt = of_dpp<OF_SHL1>(v.w, v.x);
            hmx[SL][m] = of_f4{fmaxf(fmaxf(lf, v.x), v.y), fmaxf(fmaxf(v.x, v.y), v.z), fmaxf(fmaxf(v.y, v.z), v.w),
                               fmaxf(fmaxf(v.z, v.w), rt)};
            hmn[SL][m] = of_f4{fminf(fminf(lf, v.x), v.y), fminf(fminf(v.x, v.y), v.z), fminf(fminf(v.y, v.z), v.w),
                               fminf(fminf(v.z, v.w), rt)};
            if (m == 1) dc[SL] = v;
        }
        of_publish(ctr + C_EXT + LY - 1, rho + 1);          // rows <= rho: read
    };
    // test row t (window slots A = t-1, M = t, Z = t+1)
    auto test = [&](int t, auto a_c, auto m_c, auto z_c) {
        constexpr int SA = decltype(a_c)::value, SM = decltype(m_c)::value, SZ = decltype(z_c)::value;
        unsigned long long bal[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float bmx = hmx[SA][0][j], bmn = hmn[SA][0][j];
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                bmx = fmaxf(fmaxf(fmaxf(bmx, hmx[SA][m][j]), hmx[SM][m][j]), hmx[SZ][m][j]);
                bmn = fminf(fminf(fminf(bmn, hmn[SA][m][j]), hmn[SM][m][j]), hmn[SZ][m][j]);
            }
            const float val = dc[SM][j];
            const bool e = ((val > thr) & (val >= bmx)) | ((val < -thr) & (val <= bmn));
            bal[j] = __ballot(e & inc[j]);
        }
        // words of the 128-column mask strips k overlapping [c_lo, c_hi): bit b of the even word
        // = column 128k + 2b = lane l0 + b/2, slot 2 (b & 1); odd words: slots 1, 3
        const size_t rowbase = (size_t)wb + (size_t)(t - B) * wr;
        for (int ks = c_lo / 128; ks <= (c_hi - 1) / 128; ++ks) {
            const int l0 = (128 * ks - X) / 4;
            uint32_t sv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                sv[j] = (uint32_t)(l0 >= 64 || l0 <= -32 ? 0ull : l0 >= 0 ? bal[j] >> l0 : bal[j] << (-l0));
            const unsigned long long ev = of_spread32(sv[0]) | of_spread32(sv[2]) << 1;
            const unsigned long long od = of_spread32(sv[1]) | of_spread32(sv[3]) << 1;
            if (lane == 0 && ev) atomicOr(mrow + rowbase + 2 * ks, ev);
            if (lane == 1 && od) atomicOr(mrow + rowbase + 2 * ks + 1, od);
        }
    };
    const int t_end = R - B;                           // tested rows [B, R - B)
    if (t_end > B && c_hi > c_lo) {
        load(B - 1, std::integral_constant<int, 0>{});
        load(B, std::integral_constant<int, 1>{});
#pragma unroll 1
        for (int t = B; t < t_end; t += W) {
            load(t + 1, std::integral_constant<int, 2>{});
            test(t, std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{});
            if (t + 1 >= t_end) break;
            load(t + 2, std::integral_constant<int, 0>{});
            test(t + 1, std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{}, std::integral_constant<int, 0>{});
            if (t + 2 >= t_end) break;
            load(t + 3, std::integral_constant<int, 1>{});
            test(t + 2, std::integral_constant<int, 2>{}, std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
        }
    }
    of_publish(ctr + C_EXT + LY - 1, 1 << 28);          // everything released
}

template <int R1, int R2, int R3, int R4, int R5>
__global__ __launch_bounds__(64 * OF_WAVES, 1) void k_octave(OctArgs a)
{
    using CFG = OfCfg<R1, R2, R3, R4, R5>;
    int* ctr = reinterpret_cast<int*>(of_lds + CFG::ctr_off);
    const int bid = blockIdx.x;                         // (image, strip)
    const int img = bid / a.n_strips, strip = bid - img * a.n_strips;
    // owned columns [own0, own0 + 168); the last strip is shifted left so its window keeps
    // enough valid columns right of the owned range (duplicate columns are written with
    // identical values, mask bits OR-ed twice)
    const int own0 = min(strip * OF_S, max(0, (a.C - OF_S + 3) & ~3));   // a multiple of 4: 16-B columns
    const int X = own0 - OF_H;
    const bool edge = X - OF_G < 0 || X + OF_W + OF_G > a.C;
    // every count starts at 0, except the extremum waves' releases: the test starts at row
    // BORDER, so DoG rows below BORDER - 1 are never read
    if (threadIdx.x < C_N)
        ctr[threadIdx.x] = threadIdx.x >= C_EXT && threadIdx.x < C_EXT + 3 ? VO_SIFT_BORDER - 1 : 0;
    __syncthreads();
    __builtin_amdgcn_s_setprio(2);                      // scale-space priority (as k_blur_stream)
    float* const ib = a.arena + img * a.istride;
    float* const nb = a.nbase ? a.nbase + img * a.istride : nullptr;
    // wave -> role; wave w runs on SIMD w % 4: each heavy level shares its SIMD with a light
    // wave (levels 5, 4, 3 with the extremum waves, levels 2 and 1 together).  The role is
    // wave-uniform (readfirstlane): a divergent branch would keep every role's registers live.
    const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#define OF_LEVEL_E(LV, E) of_level<CFG, LV, E>(ib + a.goff[0], ib + a.goff[LV], nb, &a.k[0][0], a.R, a.C, a.pitch, a.Rn, a.Cn, a.pitchn, X)
#define OF_LEVEL(LV) do { if (edge) OF_LEVEL_E(LV, true); else OF_LEVEL_E(LV, false); } while (0)
#define OF_EXT(LY) of_extrema<CFG, LY>(a.mask + (size_t)img * a.n_words, a.wb[LY - 1], a.wr, a.thr, a.R, a.C, X, own0)
    OF_STAT_BEGIN
    switch (role) {
    case 0: OF_LEVEL(5); break;
    case 1: OF_LEVEL(4); break;
    case 2: OF_LEVEL(3); break;
    case 3: OF_LEVEL(2); break;
    case 4: OF_EXT(1); break;
    case 5: OF_EXT(2); break;
    case 6: OF_EXT(3); break;
    default: OF_LEVEL(1); break;
    }
    OF_STAT_END(3)
#undef OF_EXT
#undef OF_LEVEL_E
#undef OF_LEVEL
}

// radii the kernel is instantiated for: SIFT defaults (3 layers, sigma 1.6, x2 upsample)
constexpr int OF_R[6] = {0, 5, 6, 8, 10, 13};
using OfDefault = OfCfg<5, 6, 8, 10, 13>;

bool octave_fused_ok(const Pyramid& py, int o)
{
    if (py.L != 3) return false;
    for (int i = 1; i <= 5; ++i)
        if (py.krad[i] != OF_R[i]) return false;
    const OctGeom& g = py.oct[o];
    return g.cols >= OF_W && g.rows >= 64;
}

void octave_fused_launch(const Pyramid& py, const Pyramid* d_py, const SiftBuffers& b, int o, int n_img, float thr,
                         hipStream_t s)
{
    const OctGeom& g = py.oct[o];
    OctArgs a;
    memset(&a, 0, sizeof(a));
    a.arena = b.arena;
    a.istride = py.istride;
    a.R = g.rows; a.C = g.cols; a.pitch = g.pitch;
    for (int i = 0; i < 6; ++i) a.goff[i] = g.g_off[i];
    if (o + 1 < py.n_oct) {
        const OctGeom& n = py.oct[o + 1];
        a.nbase = b.arena + n.g_off[0];
        a.Rn = n.rows; a.Cn = n.cols; a.pitchn = n.pitch;
    }
    a.mask = b.mask;
    a.n_words = py.n_words;
    for (int l = 0; l < 3; ++l) a.wb[l] = py.wbase[o * 3 + l];
    a.wr = py.wrow[o];
    a.thr = thr;
    for (int i = 1; i <= 5; ++i)
        for (int j = 0; j <= py.krad[i]; ++j) a.k[i][j] = py.kern[i][j];
    a.n_strips = (g.cols + OF_S - 1) / OF_S;
    const size_t lds = sizeof(float) * OfDefault::lds_floats();
    raise_lds_limit((const void*)k_octave<5, 6, 8, 10, 13>);
    static const char* const names[] = {"k_octave_o0", "k_octave_o1", "k_octave_o2", "k_octave_o3", "k_octave_o4",
                                        "k_octave_o5", "k_octave_o6", "k_octave_o7"};
    VO_LAUNCH_NAMED(names[o < 8 ? o : 7], (k_octave<5, 6, 8, 10, 13>), dim3(a.n_strips * n_img), dim3(64 * OF_WAVES), lds,
                    s, a);
#ifdef OF_STATS
    if (o == 0) {
        unsigned long long st[32];
        hipStreamSynchronize(s);
        hipMemcpyFromSymbol(st, HIP_SYMBOL(of_stat), sizeof(st));
        const char* role[8] = {"L5", "L4", "L3", "L2", "ext1", "ext2", "ext3", "L1"};
        const double n = (double)a.n_strips * n_img;
        fprintf(stderr, "k_octave o0 stats (mean cycles per workgroup): ");
        for (int w = 0; w < 8; ++w)
            fprintf(stderr, "%s total %.0f in %.0f gslot %.0f dslot %.0f | ", role[w], st[w * 4 + 3] / n, st[w * 4] / n,
                    st[w * 4 + 1] / n, st[w * 4 + 2] / n);
        fprintf(stderr, "\n");
        memset(st, 0, sizeof(st));
        hipMemcpyToSymbol(HIP_SYMBOL(of_stat), st, sizeof(st));
    }
#endif
}

}  // namespace vo
