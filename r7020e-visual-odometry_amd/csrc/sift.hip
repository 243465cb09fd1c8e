// sift.hip — detectSIFTFeatures + extractFeatures (VO.m:79-84) on gfx950.
//
// Pipeline per batch of n_img images:
//   k_blur_fused          one launch per scale level: row + column Gaussian
//                         passes through one LDS tile, writes G_i and the DoG
//                         D_{i-1} = G_i - G_{i-1} (octave 0: x2 upsample fused)
//   k_down                next octave base = G[o-1][L](2y, 2x)
//   k_ext_tile            26-neighbour extremum test on LDS tiles of all DoG
//                         levels, ballot -> 64-bit mask per 64 columns
//   k_seg_count/scan/emit deterministic compaction in (octave, layer, row,
//                         col) scan order (prefix sums, no atomic append)
//   k_refine_orient       one wave per candidate: Newton refinement (wave-
//                         uniform), orientation histogram (lanes stride the
//                         window, 2^-20 fixed-point LDS atomics), peaks by ballot
//   k_scan_cands/k_expand keypoint list in candidate order, then peak order
//   k_desc                one wave per keypoint: 4x4x8 trilinear histogram
//                         (fixed-point LDS atomics), norms as a wave tree
// Every float expression follows oracle/sift_ref.c operation for operation.
#include "vo_internal.h"
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <algorithm>
#include <utility>
#include <type_traits>
#include <mutex>

namespace vo {

// Level blur taps; nb (image 0's plane, same per-image stride as the output): the streaming blur of
// level L also stores the next octave's base, its output decimated by 2 (even rows, even columns)
struct Kern { float k[VO_SIFT_MAX_RADIUS + 1]; int r; float* nb; int nb_pitch, nb_rows, nb_cols; };

// ---------------------------------------------------------------------------
// geometry (host)
static int desc_radius_cap(const Pyramid& py, const vo_sift_params& p);

// ---------------------------------------------------------------------------
void build_pyramid_geometry(Pyramid& py, int rows, int cols, int n_img, const vo_sift_params& p)
{
    memset(&py, 0, sizeof(py));
    const int L = p.n_octave_layers;
    py.L = L;
    py.n_img = n_img;
    py.n_oct = vo_num_octaves(rows, cols, p.upsample);
    int R = p.upsample ? rows * 2 : rows, C = p.upsample ? cols * 2 : cols;
    size_t off = 0;
    size_t tmp_plane = 0;
    for (int o = 0; o < py.n_oct; ++o) {
        OctGeom& g = py.oct[o];
        if (o) { R /= 2; C /= 2; }
        g.rows = R; g.cols = C;
        g.dmax = (int)sqrt((double)C * C + (double)R * R);
        g.pitch = (C + 255) / 256 * 256;    // whole 256-column blur strips: masked-off lanes store into padding
        g.plane = (size_t)g.rows * g.pitch;
        for (int i = 0; i < L + 3; ++i) { g.g_off[i] = off; off += g.plane; }
        if (g.plane > tmp_plane) tmp_plane = g.plane;
    }
    py.istride = off;
    py.total = off * n_img;
    py.tmp_plane = tmp_plane;
    double sig[VO_SIFT_MAX_LAYERS];
    vo_level_sigmas(L, p.sigma, sig);
    py.krad[0] = vo_gauss_kernel(vo_base_sigma(p.sigma, p.upsample), py.kern[0], VO_SIFT_MAX_RADIUS + 1);
    for (int i = 1; i < L + 3; ++i) py.krad[i] = vo_gauss_kernel(sig[i], py.kern[i], VO_SIFT_MAX_RADIUS + 1);
    int w = 0, b = 0, t = 0;
    for (int o = 0; o < py.n_oct; ++o) {
        int ir = py.oct[o].rows - 2 * VO_SIFT_BORDER, ic = py.oct[o].cols - 2 * VO_SIFT_BORDER;
        if (ir < 0) ir = 0;
        if (ic < 0) ic = 0;
        // words of 64 absolute columns covering the interior [BORDER, cols - BORDER)
        // (an even count: the extremum test writes a strip's two words as a pair, see k_ext_stream)
        py.wrow[o] = ic > 0 ? ((py.oct[o].cols - VO_SIFT_BORDER - 1) / 64 + 2) / 2 * 2 : 0;
        for (int l = 0; l < L; ++l) { py.wbase[b++] = w; w += ir * py.wrow[o]; }
        py.ebase[o] = t;
        py.estrips[o] = py.wrow[o] / 2;
        t += py.estrips[o] * ((ir + VO_EXT_BAND - 1) / VO_EXT_BAND);
    }
    py.wbase[b] = w;
    py.n_words = w;
    py.ebase[py.n_oct] = t;
    py.n_units = t;
    py.n_seg = (w + VO_SEG_WORDS - 1) / VO_SEG_WORDS;
    py.dcap = desc_radius_cap(py, p);
}

SiftBuffers sift_view(const SiftBuffers& b, const Pyramid& py, int img0, int n)
{
    SiftBuffers v = b;
    v.arena = b.arena + (size_t)img0 * py.istride;
    v.tmp = b.tmp + (size_t)img0 * py.tmp_plane;
    v.mask = b.mask + (size_t)img0 * py.n_words;
    v.woff = b.woff + (size_t)img0 * py.n_seg;
    v.cand = b.cand + (size_t)img0 * b.cand_cap;
    v.n_cand = b.n_cand + img0;
    v.acc = b.acc + (size_t)img0 * b.cand_cap;
    v.n_acc = b.n_acc + img0;
    v.cout = b.cout + (size_t)img0 * b.cand_cap;
    v.koff = b.koff + (size_t)img0 * b.cand_cap;
    v.n_kp = b.n_kp + img0;
    v.kp = b.kp + (size_t)img0 * b.kp_cap;
    v.kpi = b.kpi + (size_t)img0 * b.kp_cap;
    v.desc = b.desc + (size_t)img0 * b.kp_cap * VO_DESC_LEN;
    v.meta = b.meta + (size_t)img0 * b.kp_cap;
    v.n_img = n;
    return v;
}

hipError_t sift_alloc(SiftBuffers& b, const Pyramid& py, int kp_cap, int cand_cap)
{
    const int n = py.n_img;
    b.n_img = n; b.kp_cap = kp_cap; b.cand_cap = cand_cap;
    hipError_t e;
#define VO_ALLOC(ptr, bytes) do { e = hipMalloc((void**)&(ptr), (bytes)); if (e != hipSuccess) return e; } while (0)
    VO_ALLOC(b.arena, sizeof(float) * py.total);
    VO_ALLOC(b.tmp, sizeof(float) * py.tmp_plane * n);
    VO_ALLOC(b.mask, sizeof(unsigned long long) * (size_t)py.n_words * n + 8);
    VO_ALLOC(b.woff, sizeof(uint32_t) * (size_t)py.n_seg * n + 8);
    VO_ALLOC(b.cand, sizeof(uint32_t) * (size_t)cand_cap * n);
    VO_ALLOC(b.n_cand, sizeof(int) * n);
    VO_ALLOC(b.acc, sizeof(int) * (size_t)cand_cap * n);
    VO_ALLOC(b.n_acc, sizeof(int) * n);
    VO_ALLOC(b.cout, sizeof(CandOut) * (size_t)cand_cap * n);
    VO_ALLOC(b.koff, sizeof(uint32_t) * (size_t)cand_cap * n);
    VO_ALLOC(b.n_kp, sizeof(int) * n);
    VO_ALLOC(b.kp, sizeof(vo_keypoint) * (size_t)kp_cap * n);
    VO_ALLOC(b.kpi, sizeof(KpInt) * (size_t)kp_cap * n);
    VO_ALLOC(b.desc, (size_t)VO_DESC_LEN * kp_cap * n);
    VO_ALLOC(b.meta, sizeof(DescMeta) * (size_t)kp_cap * n);
#undef VO_ALLOC
    return hipSuccess;
}

void sift_free(SiftBuffers& b)
{
    hipFree(b.arena); hipFree(b.tmp); hipFree(b.mask); hipFree(b.woff); hipFree(b.cand); hipFree(b.n_cand); hipFree(b.acc); hipFree(b.n_acc);
    hipFree(b.cout); hipFree(b.koff); hipFree(b.n_kp); hipFree(b.kp); hipFree(b.kpi); hipFree(b.desc); hipFree(b.meta);
    b = SiftBuffers();
}

// ---------------------------------------------------------------------------
// Gaussian pyramid
// ---------------------------------------------------------------------------
__device__ __forceinline__ float up_sample(const uint8_t* __restrict__ img, int ld, int rows, int cols, int y, int x)
{
    int ya = y >> 1, yb = (y & 1) ? (ya + 1 < rows ? ya + 1 : rows - 1) : (ya > 0 ? ya - 1 : 0);
    int xa = x >> 1, xb = (x & 1) ? (xa + 1 < cols ? xa + 1 : cols - 1) : (xa > 0 ? xa - 1 : 0);
    float ha = 0.75f * (float)img[ya * ld + xa] + 0.25f * (float)img[ya * ld + xb];
    float hb = 0.75f * (float)img[yb * ld + xa] + 0.25f * (float)img[yb * ld + xb];
    return 0.75f * ha + 0.25f * hb;
}

// Octave-0 source plane from the u8 image: the x2 upsample (UP) or a plain
// u8 -> float conversion, 4 columns per thread, non-temporal 16-B stores.
// Columns in [C, pitch) are padding and receive 0.
template <bool UP>
__global__ __launch_bounds__(256) void k_base_src(ImageSrc isrc, int in_rows, int in_cols, float* __restrict__ dst,
                                                  size_t plane, int pitch, int R, int C, int n_img)
{
    // grid: x = 4-column groups (256 per block), y = row, z = image
    const int y = blockIdx.y, img = blockIdx.z;
    const int x = 4 * (blockIdx.x * 256 + threadIdx.x);
    if (x >= pitch) return;
    const uint8_t* base8 = ((img & 1) ? isrc.right : isrc.left) + (size_t)(img >> 1) * isrc.frame_stride;
    float v[4];
    const int g2 = x >> 1;                               // UP: source columns g2-1 .. g2+2 feed outputs x .. x+3
    if (UP && g2 >= 1 && g2 + 5 < in_cols) {
        // the 4 source bytes of rows ya, yb from two aligned 32-bit words each (unaligned ld)
        const int ya = y >> 1, yb = (y & 1) ? (ya + 1 < in_rows ? ya + 1 : in_rows - 1) : (ya > 0 ? ya - 1 : 0);
        float s[2][4];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint8_t* a = base8 + (size_t)(q ? yb : ya) * isrc.ld + g2 - 1;
            const uintptr_t al = reinterpret_cast<uintptr_t>(a) & ~(uintptr_t)3;
            const uint32_t w0 = *reinterpret_cast<const uint32_t*>(al), w1 = *reinterpret_cast<const uint32_t*>(al + 4);
            const uint32_t b4 = __builtin_amdgcn_alignbyte(w1, w0, (uint32_t)(reinterpret_cast<uintptr_t>(a) & 3));
#pragma unroll
            for (int i = 0; i < 4; ++i) s[q][i] = (float)((b4 >> (8 * i)) & 0xff);
        }
        // s[.][0..3] = columns g2-1, g2, g2+1, g2+2 ; same expressions as up_sample
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int xa = 1 + (i >> 1), xb = (i & 1) ? xa + 1 : xa - 1;
            const float ha = 0.75f * s[0][xa] + 0.25f * s[0][xb];
            const float hb = 0.75f * s[1][xa] + 0.25f * s[1][xb];
            v[i] = x + i < C ? 0.75f * ha + 0.25f * hb : 0.0f;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            v[i] = x + i < C ? (UP ? up_sample(base8, isrc.ld, in_rows, in_cols, y, x + i) : (float)base8[y * isrc.ld + x + i])
                             : 0.0f;
    }
    typedef float f4_t __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(f4_t{v[0], v[1], v[2], v[3]}, reinterpret_cast<f4_t*>(dst + img * plane + (size_t)y * pitch + x));
}

// ---------------------------------------------------------------------------
// Fused separable blur of one scale level + DoG (one launch per level).
// A 64x64 output tile and its radius-r halo are staged once in LDS; the row
// pass writes a (64+2r) x 64 LDS image, the column pass writes G_i and
// D_{i-1} = G_i - G_{i-1} (G_{i-1} is the tile centre already in LDS).
// Register blocking: each thread produces 8 consecutive outputs along the
// filter direction from 8+2r values loaded once (LDS reads / output ~10
// instead of ~54).  RAD > 0 instantiates the radius (full unroll, static
// register indices); RAD == 0 is the generic runtime-radius path.
// MODE 0: float source plane (+DoG); 1: octave-0 base from the u8 image with
// the x2 upsample computed on the fly; 2: octave-0 base from u8, no upsample.
// Accumulation order per output = oracle_blur: acc = k0*s0;
// acc = fmaf(kj, s[-j] + s[+j], acc), j = 1..r (row pass, then column pass).
// ---------------------------------------------------------------------------
#define FT_W 64
#define FT_H 64
#define FT_V 8            // outputs per thread along the filter direction
#define FT_HW (FT_W + 4)  // row-pass LDS row stride: +4 floats breaks the 8-way b128 store conflict

__host__ __device__ constexpr int ft_iw(int r) { return (FT_W + 2 * r + 3) & ~3; }   // padded to 16 B
__host__ __device__ constexpr int ft_lds_floats(int r) { return (FT_H + 2 * r) * ft_iw(r) + (FT_H + 2 * r) * FT_HW; }

template <int RAD, int MODE>
__global__ __launch_bounds__(256) void k_blur_fused(const float* __restrict__ src, size_t plane, size_t dplane, int pitch, int R, int C,
                                                    float* __restrict__ g_out, float* __restrict__ d_out, Kern K,
                                                    ImageSrc isrc, int in_rows, int in_cols)
{
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int r = RAD > 0 ? RAD : K.r;
    const int IW = ft_iw(r), IH = FT_H + 2 * r;
    float* in = sm;
    float* hb = sm + IH * IW;
    const int img = blockIdx.z, x0 = blockIdx.x * FT_W, y0 = blockIdx.y * FT_H, tid = threadIdx.x;
    const uint8_t* base8 = nullptr;
    if (MODE != 0) base8 = ((img & 1) ? isrc.right : isrc.left) + (size_t)(img >> 1) * isrc.frame_stride;
    const float* srcp = src + img * plane;
    // ---- stage the input tile (reflect-101 only for tiles touching a border) ----
    const int LW = FT_W + 2 * r;
    const int ylo = y0 - r, xlo = x0 - r;
    const bool interior = ylo >= 0 && y0 + FT_H + r <= R && xlo >= 0 && x0 + FT_W + r <= C;
    const int lane = tid & 63, wv = tid >> 6;
    for (int rr = wv; rr < IH; rr += 4) {
        const int y = interior ? ylo + rr : vo_reflect101(ylo + rr, R);
        for (int cc = lane; cc < LW; cc += 64) {
            const int x = interior ? xlo + cc : vo_reflect101(xlo + cc, C);
            float v;
            if (MODE == 0) v = srcp[(size_t)y * pitch + x];
            else if (MODE == 1) v = up_sample(base8, isrc.ld, in_rows, in_cols, y, x);
            else v = (float)base8[y * isrc.ld + x];
            in[rr * IW + cc] = v;
        }
    }
    __syncthreads();
    // ---- row pass: IH rows x 64 columns, 8 consecutive columns per item ----
    for (int t = tid; t < IH * (FT_W / FT_V); t += 256) {
        const int rr = t >> 3, c0 = (t & 7) * FT_V;
        const float* s = in + rr * IW + c0;            // s[k] = input column c0 - r + k
        float out[FT_V];
        if constexpr (RAD > 0) {
            float v[FT_V + 2 * RAD];
#pragma unroll
            for (int k = 0; k < FT_V + 2 * RAD; ++k) v[k] = s[k];
#pragma unroll
            for (int i = 0; i < FT_V; ++i) {
                float acc = K.k[0] * v[i + RAD];
#pragma unroll
                for (int j = 1; j <= RAD; ++j) acc = fmaf(K.k[j], v[i + RAD - j] + v[i + RAD + j], acc);
                out[i] = acc;
            }
        } else {
            for (int i = 0; i < FT_V; ++i) {
                const float* q = s + i + r;
                float acc = K.k[0] * q[0];
                for (int j = 1; j <= r; ++j) acc = fmaf(K.k[j], q[-j] + q[j], acc);
                out[i] = acc;
            }
        }
#pragma unroll
        for (int i = 0; i < FT_V; ++i) hb[rr * FT_HW + c0 + i] = out[i];
    }
    __syncthreads();
    // ---- column pass: 64 columns x (64/8) row groups ----
    for (int t = tid; t < FT_W * (FT_H / FT_V); t += 256) {
        const int c = t & 63, y0l = (t >> 6) * FT_V;
        const int x = x0 + c;
        const float* s = hb + y0l * FT_HW + c;         // s[k*FT_HW] = row-pass row y0l - r + k (tile coords + r)
        float out[FT_V];
        if constexpr (RAD > 0) {
            float v[FT_V + 2 * RAD];
#pragma unroll
            for (int k = 0; k < FT_V + 2 * RAD; ++k) v[k] = s[k * FT_HW];
#pragma unroll
            for (int i = 0; i < FT_V; ++i) {
                float acc = K.k[0] * v[i + RAD];
#pragma unroll
                for (int j = 1; j <= RAD; ++j) acc = fmaf(K.k[j], v[i + RAD - j] + v[i + RAD + j], acc);
                out[i] = acc;
            }
        } else {
            for (int i = 0; i < FT_V; ++i) {
                const float* q = s + (i + r) * FT_HW;
                float acc = K.k[0] * q[0];
                for (int j = 1; j <= r; ++j) acc = fmaf(K.k[j], q[-j * FT_HW] + q[j * FT_HW], acc);
                out[i] = acc;
            }
        }
        if (x < C) {
#pragma unroll
            for (int i = 0; i < FT_V; ++i) {
                const int y = y0 + y0l + i;
                if (y < R) {
                    const size_t o = img * dplane + (size_t)y * pitch + x;
                    g_out[o] = out[i];
                    if (MODE == 0 && d_out) d_out[o] = out[i] - in[(y0l + i + r) * IW + c + r];
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Streaming level blur (MODE 0, compiled radius): one wave per (image, band of
// TH output rows, strip of 256 columns).  The wave walks the band's TH + 2r
// input rows top to bottom; each lane owns 4 consecutive columns.
//   - input rows are prefetched P rows ahead into registers (one 16-B load per
//     lane plus the 2*R4 halo floats), staged through a one-row LDS buffer for
//     the horizontal pass (the only cross-lane exchange);
//   - the horizontal results of the last RS >= 2r+1 rows live in a register
//     ring; steps are generated at compile time (vo_static_for) so every ring
//     and prefetch index is a constant; the vertical pass runs on float2 column
//     pairs (packed v_pk_* math, IEEE per element);
//   - G_i is stored as 16-B non-temporal row segments.  DoG planes are never
//     materialised: D_{i-1} = G_i - G_{i-1} is formed where it is consumed
//     (extremum test, refinement), the same float subtraction.
// The steady-state loop issues the same memory operations on every path (no
// conditional loads or stores: rows past the band are valid reflected rows,
// masked-off columns store into the row's padding column), so the compiler's
// s_waitcnt counting keeps P rows of loads in flight instead of draining.
// TH is a multiple of RS; the last band is shifted up to end at row R (rows
// computed twice are bit-identical).  Arithmetic per output is exactly
// k_blur_fused's (row pass, then column pass, same order).
// ---------------------------------------------------------------------------
typedef float vo_f2 __attribute__((ext_vector_type(2)));
typedef int vo_i2 __attribute__((ext_vector_type(2)));
typedef int vo_i4 __attribute__((ext_vector_type(4)));
typedef float vo_f4 __attribute__((ext_vector_type(4)));

// compile-time loop: f(std::integral_constant<int, 0>) ... f(<N-1>), so array
// indices derived from the counter are constants (register-resident rings)
template <typename F, int... I>
__device__ __forceinline__ void vo_static_for_impl(F&& f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void vo_static_for(F&& f) { vo_static_for_impl(f, std::make_integer_sequence<int, N>{}); }

__device__ inline int xcd_remap(int bid, int n)
{
    // consecutive logical ids on the same XCD (blocks are dealt round-robin over 8 XCDs)
    const int q = n >> 3, rm = n & 7, xcd = bid & 7, idx = bid >> 3;
    return xcd < rm ? xcd * (q + 1) + idx : rm * (q + 1) + (xcd - rm) * q + idx;
}

#define BS_P 4            // prefetch depth (rows); 6 for the octave-0 base measured the same


// Scale-space kernels raise their wave priority.  The feature stream's kernels (k_desc,
// k_orient) are VALU-bound and run beside the scale space of the next batch; a SIMD arbitrates
// VALU issue by priority, then age, so a freshly dispatched blur wave next to older descriptor
// waves only got their leftover issue slots.
#ifndef VO_SS_SETPRIO
#define VO_SS_SETPRIO 2
#endif
__device__ __forceinline__ void vo_ss_prio()
{
    if constexpr (VO_SS_SETPRIO > 0) __builtin_amdgcn_s_setprio(VO_SS_SETPRIO);
}
// halo floats each side, rounded up to whole CPL-column vectors; staged row length
__host__ __device__ constexpr int bs_rh(int r, int cpl) { return (r + cpl - 1) / cpl * cpl; }
__host__ __device__ constexpr int bs_rw(int r, int cpl) { return 64 * cpl + 2 * bs_rh(r, cpl); }
// Row-window exchange of the streaming blur.  Each lane holds CPL consecutive columns of the
// input row; the row pass needs r columns either side.  Halo-lane layout (bs_hl: 4-column lanes,
// r <= kBlurDppMaxR): the wave covers 64*CPL input columns starting RH left of its output
// strip, its outer RH/CPL lanes each side hold only halo columns and store nothing, and the
// neighbours' columns arrive by whole-wave DPP shifts (wave_shr:1 / wave_shl:1, one VALU op
// per column per level).  No halo loads, no halo upsampling, no LDS round trip: per row the
// LDS exchange cost 2 ds_write_b128 (13 LDS cycles each, at half rate from one wave) + (1 +
// 2 rh/4) ds_read_b128, which base_probe measured at ~180 of the octave-0 base kernel's ~430 us.
// (r >= 6, and the r = 5 level with 2-column lanes, keep the LDS exchange: measured faster)
constexpr int kBlurDppMaxR = 5;
__host__ __device__ constexpr bool bs_hl(int r, int cpl, int tag)
{
    return cpl == 4 && r <= kBlurDppMaxR && !(tag & 32);
}
// output columns per strip
__host__ __device__ constexpr int bs_sw(int r, int cpl, int tag) { return 64 * cpl - (bs_hl(r, cpl, tag) ? 2 * bs_rh(r, cpl) : 0); }

enum : int { VO_DPP_WAVE_SHL1 = 0x130, VO_DPP_WAVE_SHR1 = 0x138 };
template <int CTRL>
__device__ __forceinline__ float vo_dpp(float src)
{
    // lane 0 (wave_shr) / lane 63 (wave_shl) has no source lane and keeps its own value
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(src), __float_as_int(src), CTRL, 0xF, 0xF, false));
}

// w[RH + j] = column (lane's first column + j) for j in [-RAD, CPL - 1 + RAD]: level s of the
// window is the wave shifted by s lanes (only the components the row pass reads).  The first
// and last RH/CPL lanes get shifted-in values they never use (they produce no output).
template <int RAD, int CPL, typename vec_t>
__device__ __forceinline__ void vo_dpp_window(const vec_t& vm, float* w)
{
    constexpr int RH = bs_rh(RAD, CPL), NL = RH / CPL;
    float L[CPL], Rt[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) w[RH + k] = L[k] = Rt[k] = vm[k];
#pragma unroll
    for (int s = 1; s <= NL; ++s) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            if (k >= s * CPL - RAD) {
                L[k] = vo_dpp<VO_DPP_WAVE_SHR1>(L[k]);
                w[RH - s * CPL + k] = L[k];
            }
            if (CPL - 1 - k >= s * CPL - RAD) {
                Rt[k] = vo_dpp<VO_DPP_WAVE_SHL1>(Rt[k]);
                w[RH + s * CPL + k] = Rt[k];
            }
        }
    }
}


// u8 source of the octave-0 base level (TAG & 4): the x2 upsample is formed per input row from
// source bytes the wave staged in LDS when it started (every source row its band reads, the
// strip's byte columns).  The row loop then issues no vector-memory load at all: on gfx9 stores
// and loads share one in-order vmcnt, so a row prefetched from HBM P steps ahead also waited for
// the P steps of 16-B stores issued before it -- the base kernel's stream of 1 GB of stores was
// paced by its tiny u8 loads.  With the loads gone the loop never waits on vmcnt.
struct U8Src { const uint8_t* p; int ld, rows, cols; };
#ifndef VO_BASE_MAX_TH
#define VO_BASE_MAX_TH 96         // 8.7 KB of staged rows: 16 one-wave workgroups per CU fit (128: 11.1 KB, 14)
#endif
constexpr int kBaseMaxTH = VO_BASE_MAX_TH;                    // band height bound of the staged form
// staged row length in dwords: the upsampled span of a wave (64 CPL columns + 2 RH halo) needs
// (64 CPL + 2 RH) / 2 + 3 source bytes; + 3 for the row's misalignment, + 4 for the word pair
__host__ __device__ constexpr int bs_u8_dw(int r, int cpl) { return ((64 * cpl + 2 * bs_rh(r, cpl)) / 2 + 3 + 3 + 4 + 3) / 4; }
// staged rows: a band reads F + TH upsampled rows (F = 2r + E, E < P), i.e. at most half as many
// source rows + 3 (the neighbour row of each end, rounding)
__host__ __device__ constexpr int bs_u8_rows(int r) { return (2 * r + BS_P + kBaseMaxTH) / 2 + 4; }

__device__ __forceinline__ vo_f4 up4_from_words(uint32_t a0, uint32_t a1, uint32_t sa, uint32_t b0, uint32_t b1, uint32_t sb)
{
    // 4 source bytes (columns g2-1 .. g2+2) of rows ya, yb -> outputs x .. x+3 (x = 2*g2), as up_sample
    const uint32_t ba = __builtin_amdgcn_alignbyte(a1, a0, sa), bb = __builtin_amdgcn_alignbyte(b1, b0, sb);
    // up_sample's 0.75 ha + 0.25 hb, ha = 0.75 a + 0.25 b, is exact in fp32 for bytes (every
    // partial is a multiple of 1/16 below 256), so it equals (9 A[xa] + 3 A[xb] + 3 B[xa] +
    // B[xb]) / 16: one byte permute + one v_dot4_u32_u8 per output instead of ~10 VALU.
    float r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t xa = 1 + (i >> 1), xb = (i & 1) ? xa + 1 : xa - 1;
        const uint32_t sel = xa | xb << 8 | (4 + xa) << 16 | (4 + xb) << 24;   // bytes of {bb:ba}
        const uint32_t q = __builtin_amdgcn_perm(bb, ba, sel);
        r[i] = (float)__builtin_amdgcn_udot4(q, 0x01030309u, 0u, false) * 0.0625f;
    }
    return vo_f4{r[0], r[1], r[2], r[3]};
}

template <int RAD, bool EDGE, int TAG, int CPL>
__device__ __forceinline__ void blur_stream_body(const float* __restrict__ sp, int pitch, int R, int C,
                                                 float* __restrict__ g_out, const Kern& K,
                                                 int x0, int y0, int TH, float* rb, const U8Src& u8,
                                                 float* __restrict__ nbo, uint32_t* __restrict__ stg)
{
    // CPL columns per lane (4: 256-column strips, 16-B accesses; 2: 128-column strips,
    // 8-B accesses, half the ring registers -> more waves for the smaller octaves)
    typedef float vec_t __attribute__((ext_vector_type(CPL)));
    constexpr bool UP = (TAG & 4) != 0;
    static_assert(!UP || CPL == 4, "the fused x2 upsample uses 4 columns per lane");
    constexpr bool XCH = bs_hl(RAD, CPL, TAG);             // halo-lane layout + DPP window exchange
    constexpr int SW = 64 * CPL;                           // input columns per wave
    constexpr int P = BS_P;                                // prefetch depth = steps per loop block
    constexpr int RH = bs_rh(RAD, CPL);                    // halo rounded to whole vectors
    constexpr int NQ = 1 + 2 * RH / CPL;                   // vector reads per lane window
    constexpr int NP = CPL / 2;                            // float2 column pairs per lane
    constexpr int NR = 2 * RAD + P;                        // ring: 2r carried rows + P new per block
    constexpr int F = (2 * RAD + P - 1) / P * P;           // ring-fill steps (no output)
    constexpr int E = F - 2 * RAD;                         // extra rows read above the band
    constexpr int RW = bs_rw(RAD, CPL);                    // staged row floats
    // the staged form's LDS (stg) holds the source rows of at most kBaseMaxTH-row bands; the
    // launcher caps TH, and a taller band (a probe or a future launcher) stores nothing rather
    // than staging past stg into the other shared arrays (wave-uniform, before any LDS use)
    if constexpr ((TAG & 4) != 0) {
        if (TH > kBaseMaxTH) return;
    }
    const int lane = threadIdx.x;
    const int xl = x0 - (XCH ? RH : 0) + CPL * lane;      // XCH: x0 is the first output column
    // halo lanes: [0, RH/CPL) left, [RH/CPL, 2*RH/CPL) right.  The others load lane 0's
    // segment (same cache line) and stage it into a private dummy LDS slot, so every
    // lane issues the same instructions.
    const bool hl = lane < RH / CPL, hr = !hl && lane < 2 * RH / CPL;
    const int hx = XCH ? xl : hl ? x0 - RH + CPL * lane : hr ? x0 + SW + CPL * (lane - RH / CPL) : x0 - RH;
    const int hpos = hl ? CPL * lane : hr ? RH + SW + CPL * (lane - RH / CPL) : -1;
    float* const dummy = rb + RW + CPL * lane;
    int cm[CPL], ch[CPL];                                  // border strips: reflect-101 source columns
    if (EDGE) {
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
            cm[i] = vo_reflect101(xl + i, C);
            ch[i] = vo_reflect101(hx + i, C);
        }
    }
    float k[RAD + 1];
#pragma unroll
    for (int j = 0; j <= RAD; ++j) k[j] = K.k[j];
    static_assert(P % 2 == 0, "the next-base rows are the even steps of a block");
    // buffer descriptors (wave-uniform: kernel arguments and block-derived offsets) of this
    // image's output plane and of the next octave's base plane (size 0 when not stored)
    const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(g_out, 0, R * pitch * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_nb =
        __builtin_amdgcn_make_buffer_rsrc(nbo, 0, nbo ? K.nb_rows * K.nb_pitch * 4 : 0, 0x00020000);

    // UP: stage the band's source rows [sr0, sr0 + nrs) -- bytes [s_lo, s_lo + 4 SWD) of each,
    // from the row's 4-B aligned start (misalignment m of row q: (delta + (sr0+q) ld + s_lo) & 3)
    // -- into stg[q][SWD] by dword buffer loads (bytes past the image read as 0, no fault)
    constexpr int SWD = bs_u8_dw(RAD, CPL);
    const int xs0 = x0 - RH;                               // first upsampled column of the wave's span
    const int s_lo = max(0, (xs0 >> 1) - 1);               // (>> 1: floor, xs0 may be negative on the left edge)
    int sr0 = 0;
    uint32_t delta = 0;
    if constexpr (UP) {
        const int p_lo = y0 - RAD - E, p_hi = y0 - RAD - E + F + TH - 1;
        int ymin = p_lo < 0 ? 0 : p_lo, ymax = p_hi >= R ? R - 1 : p_hi;
        if (p_lo < 0) ymax = max(ymax, min(-p_lo, R - 1));
        if (p_hi >= R) ymin = min(ymin, max(2 * R - 2 - p_hi, 0));
        sr0 = max(0, (ymin >> 1) - 1);
        const int sr1 = min(u8.rows - 1, (ymax >> 1) + 1);
        const int total = (sr1 - sr0 + 1) * SWD;           // <= bs_u8_rows(RAD) * SWD (kBaseMaxTH)
        delta = (uint32_t)(reinterpret_cast<uintptr_t>(u8.p) & 3);
        // range = the image's last byte rounded up to its dword: a buffer load returns 0 for a
        // whole dword that crosses the range's end, which would drop the last row's final bytes;
        // the rounded range stays inside that 4-B aligned word, so it never reaches another page
        const uint32_t span = delta + (uint32_t)(u8.rows - 1) * (uint32_t)u8.ld + (uint32_t)u8.cols;
        const __amdgpu_buffer_rsrc_t rs_in =
            __builtin_amdgcn_make_buffer_rsrc((void*)(u8.p - delta), 0, (int)((span + 3u) & ~3u), 0x00020000);
        constexpr int SCH = 16;                            // loads in flight per lane per round
        for (int t0 = 0; t0 < total; t0 += 64 * SCH) {
            uint32_t v[SCH];
#pragma unroll
            for (int q = 0; q < SCH; ++q) {
                const int t = t0 + 64 * q + lane;
                const int row = t / SWD, k = t - row * SWD;
                const uint32_t ro = delta + (uint32_t)(sr0 + row) * (uint32_t)u8.ld + (uint32_t)s_lo;
                v[q] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs_in, t < total ? (ro & ~3u) + 4u * (uint32_t)k : 0x80000000u, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < SCH; ++q)
                if (t0 + 64 * q + lane < total) stg[t0 + 64 * q + lane] = v[q];
        }
        __syncthreads();                                   // one-wave block: LDS writes before the reads
    }
    // UP: byte offset of source column x of source row y inside its staged row
    auto s_off = [&](int y, int x) {
        return (y - sr0) * (4 * SWD) + (x - s_lo) + (int)((delta + (uint32_t)y * (uint32_t)u8.ld + (uint32_t)s_lo) & 3u);
    };
    const uint8_t* const stg8 = reinterpret_cast<const uint8_t*>(stg);

    // Prefetch slots.  The DPP layout keeps two sets and alternates them block by block: block
    // parity b consumes set b and refills set 1-b, so a slot's old value is dead before its
    // register is loaded again.  With one set the scheduler hoisted each refill above the last
    // use of the value it replaces, the allocator gave the refill other registers, and the copy
    // back at the loop edge waited for the load (vmcnt(1) once per block).  (The LDS-staged
    // layout consumes a slot before its refill by a barrier and keeps one set.)
    constexpr int NSET = XCH ? 2 : 1;
    vec_t pf[NSET * P], ph[NSET * P];
    typedef uint32_t u2_t __attribute__((ext_vector_type(2)));
    u2_t pw[UP && !EDGE ? NSET * P : 1][4];                // UP: raw words (ya main, yb main, ya halo, yb halo)
    vo_f2 H[NR][NP];
    // UP: source byte column of the first of the 4 bytes feeding outputs xl.. / hx..
    const int gm = (xl >> 1) - 1, gh = (hx >> 1) - 1;

    auto gather = [&](const float* rowp, const int* idx) {
        vec_t v;
#pragma unroll
        for (int i = 0; i < CPL; ++i) v[i] = rowp[idx[i]];
        return v;
    };

    // input row of step kk, reflected (reflect-101).  DPP layout: one fold by selects -- no loop
    // in the step's control flow, which otherwise split the step into blocks and cost a vmcnt(0)
    // per block pair; the launch guarantees R > r + P + 2, so a band reads at most r + E < R - 1
    // rows beyond either edge.  (The LDS layout keeps the general form: the select form raised
    // its register count past 256.)
    auto yref = [&](int kk) {
        const int p = y0 - RAD - E + kk;
        if constexpr (XCH) return p < 0 ? -p : (p >= R ? 2 * R - 2 - p : p);
        else return vo_reflect101(p, R);
    };
    // loads for step kk into prefetch slot SL: input row y0-r-E+kk (reflected)
    // UP: the word pair of the staged row holding source byte column x (LDS, 4-B aligned)
    auto s_words = [&](int y, int x) {
        const int o = s_off(y, x);
        const uint32_t* w = stg + (o >> 2);
        return u2_t{w[0], w[1]};
    };
#define VO_BS_LOAD(KK, SL)                                                                        \
    do {                                                                                          \
        const int yin_ = yref(KK);                                                                \
        if constexpr (UP) {                                                                       \
            if constexpr (!EDGE) {                                                                \
                const int ya_ = yin_ >> 1;                                                        \
                const int yb_ = (yin_ & 1) ? min(ya_ + 1, u8.rows - 1) : max(ya_ - 1, 0);         \
                pw[SL][0] = s_words(ya_, gm);                                                     \
                pw[SL][1] = s_words(yb_, gm);                                                     \
                if constexpr (!XCH) {                                                             \
                    pw[SL][2] = s_words(ya_, gh);                                                 \
                    pw[SL][3] = s_words(yb_, gh);                                                 \
                }                                                                                 \
            }                                                                                     \
        } else {                                                                                  \
            const float* rowp_ = sp + (size_t)yin_ * pitch;                                       \
            if constexpr (!EDGE) {                                                                \
                pf[SL] = *reinterpret_cast<const vec_t*>(rowp_ + xl);                             \
                if (!(TAG & 64) && !XCH) ph[SL] = *reinterpret_cast<const vec_t*>(rowp_ + hx);   \
            } else {                                                                              \
                pf[SL] = gather(rowp_, cm);                                                       \
                if constexpr (!XCH) ph[SL] = gather(rowp_, ch);                                   \
            }                                                                                     \
        }                                                                                         \
    } while (0)

    // row kk's own and halo vectors from prefetch slot SL (UP: the x2 upsample formed here)
    auto fetch = [&](auto sl_c, int kk, vec_t& vm, vec_t& vh) {
        constexpr int SL = decltype(sl_c)::value;
        vm = pf[SL];
        if constexpr (!XCH) vh = ph[SL];
        if constexpr (UP) {
            // the prefetch of steps past the band's end read its last row again: same row here
            const int yin = yref(min(kk, F + TH - 1));
            const int ya = yin >> 1, yb = (yin & 1) ? min(ya + 1, u8.rows - 1) : max(ya - 1, 0);
            if constexpr (!EDGE) {
                vm = up4_from_words(pw[SL][0].x, pw[SL][0].y, (uint32_t)s_off(ya, gm) & 3u, pw[SL][1].x, pw[SL][1].y,
                                    (uint32_t)s_off(yb, gm) & 3u);
                if constexpr (!XCH)
                    vh = up4_from_words(pw[SL][2].x, pw[SL][2].y, (uint32_t)s_off(ya, gh) & 3u, pw[SL][3].x, pw[SL][3].y,
                                        (uint32_t)s_off(yb, gh) & 3u);
            } else {                                      // border strips: reflected columns, bytes from LDS
                // up_sample's expressions on the staged bytes
                auto up_at = [&](int x) {
                    const int xa = x >> 1, xb = (x & 1) ? (xa + 1 < u8.cols ? xa + 1 : u8.cols - 1) : (xa > 0 ? xa - 1 : 0);
                    const float ha = 0.75f * (float)stg8[s_off(ya, xa)] + 0.25f * (float)stg8[s_off(ya, xb)];
                    const float hb = 0.75f * (float)stg8[s_off(yb, xa)] + 0.25f * (float)stg8[s_off(yb, xb)];
                    return 0.75f * ha + 0.25f * hb;
                };
#pragma unroll
                for (int i = 0; i < CPL; ++i) {
                    vm[i] = up_at(cm[i]);
                    if constexpr (!XCH) vh[i] = up_at(ch[i]);
                }
            }
        }
    };
    // P steps kk0 .. kk0+P-1: exchange input row kk's window (DPP, or staged through LDS),
    // prefetch row kk+P, horizontal pass into ring slot 2r+u, and (STORE) the vertical pass
    // over ring slots u .. u+2r for output row y0 + kk - F; then the ring shifts down by P.
    auto block = [&](int kk0, auto store_c, auto par_c) {
        constexpr int B = decltype(par_c)::value;           // slot set consumed (NSET = 2: 1 - B refilled)
        vo_static_for<P>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            constexpr int SC = B * P + u, SN = ((B + 1) % NSET) * P + u;
            const int kk = kk0 + u;
            float w[CPL * NQ];
            if constexpr (XCH) {
#pragma unroll
                for (int i = 0; i < CPL * NQ; ++i) w[i] = 0.0f;
                vec_t vm, vh;
                fetch(std::integral_constant<int, SC>{}, kk, vm, vh);
                VO_BS_LOAD(min(kk + P, F + TH - 1), SN);  // past the band's end: its last row again (an L2 hit)
                vo_dpp_window<RAD, CPL>(vm, w);
            } else {
                float* const row = rb;
                vec_t vm, vh;
                fetch(std::integral_constant<int, SC>{}, kk, vm, vh);
                if (!(TAG & 32)) {                        // TAG & 32: probe variant without LDS staging
                    *reinterpret_cast<vec_t*>(row + RH + CPL * lane) = vm;
                    *reinterpret_cast<vec_t*>(hpos >= 0 ? row + hpos : dummy) = vh;
                }
                __syncthreads();                          // one-wave block: orders the LDS row only
                VO_BS_LOAD(min(kk + P, F + TH - 1), SN);  // past the band's end: its last row again (an L2 hit)
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const vec_t t = (TAG & 32) ? (q & 1 ? vh : vm) : *reinterpret_cast<const vec_t*>(row + CPL * lane + CPL * q);
#pragma unroll
                    for (int i = 0; i < CPL; ++i) w[CPL * q + i] = t[i];
                }
            }
            // Row pass on column pairs (x, x+1), x = RH + 2c even: packed v_pk_add / v_pk_fma
            // (IEEE per element: the scalar acc = k0*s0; acc = fmaf(kj, s[-j] + s[+j], acc)).
            // Tap j reads the pairs {w[x-j], w[x+1-j]} and {w[x+j], w[x+1+j]}: aligned pairs
            // E[m] = {w[2m], w[2m+1]} for even j, shifted pairs O[m] = {w[2m+1], w[2m+2]}
            // (formed once per row) for odd j -- half the row-pass VALU of the scalar form.
            constexpr int NW = CPL * NQ;
            vo_f2 E[NW / 2], O[NW / 2 - 1];
#pragma unroll
            for (int m = 0; m < NW / 2; ++m) E[m] = vo_f2{w[2 * m], w[2 * m + 1]};
#pragma unroll
            for (int m = 0; m < NW / 2 - 1; ++m) O[m] = __builtin_shufflevector(E[m], E[m + 1], 1, 2);
#pragma unroll
            for (int c = 0; c < NP; ++c) {
                constexpr int X0 = RH;                    // x = X0 + 2c
                const int x = X0 + 2 * c;
                vo_f2 acc = vo_f2{k[0], k[0]} * E[x / 2];
                if (!(TAG & 8))                           // TAG & 8: probe variant without the row pass
#pragma unroll
                    for (int j = 1; j <= RAD; ++j) {
                        const vo_f2 a = (j & 1) ? O[(x - j - 1) / 2] : E[(x - j) / 2];
                        const vo_f2 b = (j & 1) ? O[(x + j - 1) / 2] : E[(x + j) / 2];
                        acc = __builtin_elementwise_fma(vo_f2{k[j], k[j]}, a + b, acc);
                    }
                H[2 * RAD + u][c] = acc;
            }
            // store_c: 0 ring fill (no output), 1 output, 2 decided per step (kk >= F; the
            // stores are issued either way, dropped during the fill)
            constexpr int MODE = decltype(store_c)::value;
            if constexpr (MODE != 0) {
                vec_t g;
                if constexpr (MODE == 2) g = vec_t{};
                if (MODE == 1 || kk >= F) {
#pragma unroll
                    for (int c = 0; c < NP; ++c) {
                        vo_f2 acc = vo_f2{k[0], k[0]} * H[u + RAD][c];
                        if (!(TAG & 16))                  // TAG & 16: probe variant without the column pass
#pragma unroll
                            for (int j = 1; j <= RAD; ++j)
                                acc = __builtin_elementwise_fma(vo_f2{k[j], k[j]}, H[u + RAD - j][c] + H[u + RAD + j][c], acc);
                        g[2 * c] = acc.x;
                        g[2 * c + 1] = acc.y;
                    }
                }
                // nothing reads a plane's row padding (columns >= C), so lanes past the last
                // column store nothing (3 % of the octave-0 level writes); XCH: the halo lanes
                // store nothing either.  Buffer stores whose inactive lanes get an out-of-range
                // offset (the hardware drops them): every step issues the same VMEM instructions
                // unconditionally.  (A store -- or a prefetch -- under a branch made the compiler's
                // waitcnt pass assume it might have been skipped and drain the queue with
                // vmcnt(0) once per block, so the rows prefetched P steps ahead were waited for
                // 1-3 steps after issue.)
                const int y = y0 + kk - F;
                const bool act = (!XCH || (lane >= RH / CPL && lane < 64 - RH / CPL)) && xl < C && y < R &&
                                 (MODE == 1 || (kk >= F && kk < F + TH));
                constexpr uint32_t OOB = 0x80000000u;
                const uint32_t vo = act ? (uint32_t)(y * pitch + xl) * 4u : OOB;
                constexpr int AUX = (TAG & 2) ? 0 : 2;           // 2: non-temporal (TAG & 2: cached store variant)
                if constexpr (CPL == 4)
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(vo_i4, g), rs_out, vo, 0, AUX);
                else
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(vo_i2, g), rs_out, vo, 0, AUX);
                // next octave's base (level L; K.nb unset: a zero-size buffer drops it): even rows
                // -- the even steps u, since y0, F and kk0 - F are multiples of P -- and the lane's
                // even columns (xl is even)
                if constexpr ((u & 1) == 0 && !(TAG & 1)) {        // (the octave-0 base, TAG & 1, never stores one)
                    const int yn = y >> 1, c0 = xl >> 1;
                    const bool rowok = act && yn < K.nb_rows;
                    const uint32_t nbase = (uint32_t)(yn * K.nb_pitch + c0) * 4u;
                    const float g0 = g[0];
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(g0), rs_nb, rowok && c0 < K.nb_cols ? nbase : OOB,
                                                          0, 0);
                    if constexpr (CPL == 4) {
                        const float g2 = g[2];
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(g2), rs_nb,
                                                              rowok && c0 + 1 < K.nb_cols ? nbase + 4u : OOB, 0, 0);
                    }
                }
            }
            if constexpr (!XCH) __syncthreads();
        });
#pragma unroll
        for (int q = 0; q < 2 * RAD; ++q)
#pragma unroll
            for (int c = 0; c < NP; ++c) H[q][c] = H[q + P][c];
    };

    vo_static_for<P>([&](auto uc) { VO_BS_LOAD(decltype(uc)::value, decltype(uc)::value); });
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    if constexpr (NSET == 1) {
#pragma unroll 1
        for (int kk0 = 0; kk0 < F; kk0 += P) block(kk0, I0{}, I0{});               // ring fill
#pragma unroll 1
        for (int kk0 = F; kk0 < F + TH; kk0 += P) block(kk0, I1{}, I0{});          // TH % P == 0
    } else {
        // pairs of blocks (set 0, then set 1) from the ring fill on; a pair's second block past
        // the band's end only re-reads its last row and stores nothing
#pragma unroll 1
        for (int kk0 = 0; kk0 < F + TH; kk0 += 2 * P) {
            block(kk0, I2{}, I0{});
            block(kk0 + P, I2{}, I1{});
        }
    }
#undef VO_BS_LOAD
}

// TAG: 0 level blur, 1 octave-0 base from a float plane, 5 octave-0 base with the x2
// upsample of the u8 image fused (isrc); instrumentation variants used only by
// tools/blur_probe.hip: 2 cached stores, 8 no row pass, 16 no column pass,
// 32 no LDS staging, 64 no halo loads.  CPL: columns per lane (4 or 2).
#ifndef VO_BLUR_OCC3_MAXR
#define VO_BLUR_OCC3_MAXR 6       // radii up to this run at 3 waves per SIMD (168 VGPRs), larger at 2
#endif
#ifndef VO_BASE_WAVES
#define VO_BASE_WAVES 3           // register budget of the staged octave-0 base (TAG & 4), waves per SIMD
#endif
template <int RAD, int TAG, int CPL = 4>
__global__ __launch_bounds__(64, (TAG & 4) ? VO_BASE_WAVES : (RAD <= VO_BLUR_OCC3_MAXR || CPL == 2) ? 3 : 2) void k_blur_stream(
    const float* __restrict__ src, size_t splane, size_t dplane, int pitch, int R, int C, float* __restrict__ g_out, Kern K,
    int n_strips, int n_bands, int TH, ImageSrc isrc, int in_rows, int in_cols)
{
    vo_ss_prio();
    constexpr int RH = bs_rh(RAD, CPL), SW = bs_sw(RAD, CPL, TAG);   // output columns per strip
    constexpr bool XCH = bs_hl(RAD, CPL, TAG);
    // LDS exchange: staged row + per-lane dummy halo slots (unused with the DPP exchange)
    __shared__ __attribute__((aligned(16))) float rb[XCH ? 4 : bs_rw(RAD, CPL) + 64 * CPL];
    // TAG & 4: the band's staged u8 source rows (10.2 KB at r = 5)
    __shared__ uint32_t stg[(TAG & 4) ? bs_u8_rows(RAD) * bs_u8_dw(RAD, CPL) : 1];
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = bid % n_strips, tb = bid / n_strips;
    const int band = tb % n_bands, img = tb / n_bands;
    // the last band is cut to the plane (rounded up to whole P-row blocks, rows >= R not
    // stored) instead of being shifted up over its neighbour's rows (2.4 % re-computed rows
    // at 750 rows / 128-row bands)
    const int x0 = strip * SW, y0 = band * TH;
    const int THb = min(TH, (R - y0 + BS_P - 1) / BS_P * BS_P);
    const size_t os = img * splane, od = img * dplane;
    U8Src u8{nullptr, 0, in_rows, in_cols};
    int margin = 0;
    if (TAG & 4) {
        u8.p = ((img & 1) ? isrc.right : isrc.left) + (size_t)(img >> 1) * isrc.frame_stride;
        u8.ld = isrc.ld;
        // the interior form reads source bytes g2-1 .. g2+2 for outputs 2 g2 .. 2 g2 + 3 with no
        // clamp: the span must end >= 2 columns before the plane's edge (16: the strips of the
        // validated pre-staging layout)
        margin = 16;
    }
    float* const nbo = K.nb ? K.nb + od : nullptr;
    if (x0 - RH < 0 || (XCH ? x0 - RH + 64 * CPL : x0 + SW + RH) + margin > C)
        blur_stream_body<RAD, true, TAG, CPL>(src + os, pitch, R, C, g_out + od, K, x0, y0, THb, rb, u8, nbo, stg);
    else
        blur_stream_body<RAD, false, TAG, CPL>(src + os, pitch, R, C, g_out + od, K, x0, y0, THb, rb, u8, nbo, stg);
}

// next octave base: G0 of octave o = G_L of octave o-1 decimated by 2.  Grid (column blocks of
// 256, rows, images): no index divisions (the grid-stride form spent ~57 VALU per element on
// 64-bit div/mod).
__global__ __launch_bounds__(256) void k_down(const float* __restrict__ src, size_t splane, int spitch,
                                              float* __restrict__ dst, size_t dplane, int dpitch, int C)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, img = blockIdx.z;
    if (x < C) dst[img * dplane + (size_t)y * dpitch + x] = src[img * splane + (size_t)(2 * y) * spitch + 2 * x];
}

// ---------------------------------------------------------------------------
// Small octaves in one launch: one workgroup per image builds every level of
// octaves o_first .. n_oct-1 in LDS (planes of <= VO_SMALL_PX pixels), so the
// ~6 latency-bound launches per tiny octave (5 blurs + downsample) become one.
// Octave o_first's base is the 2x decimation of G_L of octave o_first-1 (from
// HBM); later bases are decimated from the LDS copy of G_L.  Every level is
// written to its arena plane (the extremum test, refinement and descriptors
// read them).  Per-output arithmetic = k_blur_fused (row pass, then column
// pass, acc = k0*s0; acc = fmaf(kj, s[-j] + s[+j], acc)); reflect-101 indices
// come from per-octave LDS tables.
// ---------------------------------------------------------------------------
#ifndef VO_SMALL_PX
#define VO_SMALL_PX 9216          // largest plane of the LDS path: 3 planes + the next base fit in 160 KB
#endif
#ifndef VO_SMALL_T
#define VO_SMALL_T 1024
#endif

// Register-blocked passes of k_small_pyr: one thread computes SMV consecutive outputs along the
// filter direction from the SMV + 2r inputs it reads once (reflect-101 through the tables only
// near the plane's edges), so a tap costs no LDS reads: the per-tap form read two table entries
// and two values per tap and output (~52 LDS reads per output at r = 13) and was LDS-bound.
// Per output: acc = k0 s0; acc = fmaf(kj, s[-j] + s[+j], acc), j = 1..r (the spec's order).
constexpr int SMV = 8;
template <int RAD>
__device__ __forceinline__ void small_pass(const float* __restrict__ src, float* __restrict__ dst, float* __restrict__ gdst,
                                           int gpitch, int R, int C, bool rows, const float* __restrict__ kk,
                                           const int* __restrict__ tab, int tid)
{
    // rows: items (y, x0 = 8q) along rows; else items (x, y0 = 8q) down columns.  Consecutive
    // threads take consecutive lines (row pass: rows C floats apart, C odd or not a multiple of
    // 64 at these octaves; column pass: adjacent columns), not consecutive runs of one line (8
    // floats apart: an 8-way LDS bank conflict)
    const int len = rows ? C : R, other = rows ? R : C, runs = (len + SMV - 1) / SMV;
    float k[RAD + 1];
#pragma unroll
    for (int j = 0; j <= RAD; ++j) k[j] = kk[j];
    for (int it = tid; it < other * runs; it += VO_SMALL_T) {
        const int q = it / other, line = it - q * other, p0 = q * SMV;
        const int stride = rows ? 1 : C;
        const float* s0 = rows ? src + line * C : src + line;
        float w[SMV + 2 * RAD];
        if (p0 - RAD >= 0 && p0 + SMV - 1 + RAD < len) {
#pragma unroll
            for (int j = 0; j < SMV + 2 * RAD; ++j) w[j] = s0[(p0 - RAD + j) * stride];
        } else {
#pragma unroll
            for (int j = 0; j < SMV + 2 * RAD; ++j) w[j] = s0[tab[min(p0 + j, len - 1 + 2 * RAD)] * stride];
        }
#pragma unroll
        for (int v = 0; v < SMV; ++v) {
            if (p0 + v >= len) break;
            float acc = k[0] * w[RAD + v];
#pragma unroll
            for (int j = 1; j <= RAD; ++j) acc = fmaf(k[j], w[RAD + v - j] + w[RAD + v + j], acc);
            const int y = rows ? line : p0 + v, x = rows ? p0 + v : line;
            dst[y * C + x] = acc;
            if (gdst) gdst[(size_t)y * gpitch + x] = acc;
        }
    }
}

__global__ __launch_bounds__(VO_SMALL_T) void k_small_pyr(const Pyramid* __restrict__ py, float* __restrict__ arena,
                                                          int o_first, int rtab, int cap, int bcap)
{
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int img = blockIdx.x, tid = threadIdx.x;
    const int L = py->L, NL = L + 3;
    float* cur = sm;                                  // G_{i-1}   (cap = the largest plane, a multiple of 4)
    float* tmp = sm + cap;                            // row-pass output
    float* nxt = sm + 2 * cap;                        // G_i
    float* base = sm + 3 * cap;                       // next octave's G_0 (bcap = the largest such plane)
    int* ridx = reinterpret_cast<int*>(base + bcap);                  // reflect-101 tables
    int* cidx = ridx + rtab;                          // rtab >= rows + 2r of every octave here
    for (int o = o_first; o < py->n_oct; ++o) {
        const OctGeom& g = py->oct[o];
        const int R = g.rows, C = g.cols, RC = R * C;
        float* gplane = arena + img * py->istride;
        // ---- G_0 ----
        if (o == o_first) {
            const OctGeom& pg = py->oct[o - 1];
            const float* sp = arena + pg.g_off[L] + img * py->istride;
            for (int e = tid; e < RC; e += VO_SMALL_T) {
                const int y = e / C, x = e - y * C;
                cur[e] = sp[(size_t)(2 * y) * pg.pitch + 2 * x];
            }
        } else {
            for (int e = tid; e < RC; e += VO_SMALL_T) cur[e] = base[e];
        }
        __syncthreads();
        for (int e = tid; e < RC; e += VO_SMALL_T) {
            const int y = e / C, x = e - y * C;
            gplane[g.g_off[0] + (size_t)y * g.pitch + x] = cur[e];
        }
        // ---- levels 1 .. L+2 ----
        for (int i = 1; i < NL; ++i) {
            const int r = py->krad[i];
            const float* kk = py->kern[i];
            for (int t = tid; t < R + 2 * r; t += VO_SMALL_T) ridx[t] = vo_reflect101(t - r, R);
            for (int t = tid; t < C + 2 * r; t += VO_SMALL_T) cidx[t] = vo_reflect101(t - r, C);
            __syncthreads();
            float* const gl = gplane + g.g_off[i];
            switch (r) {                                                  // the default sigmas' radii
#define VO_SMALL_R(RR)                                                                        \
    case RR:                                                                                  \
        small_pass<RR>(cur, tmp, nullptr, 0, R, C, true, kk, cidx, tid);                      \
        __syncthreads();                                                                      \
        small_pass<RR>(tmp, nxt, gl, g.pitch, R, C, false, kk, ridx, tid);                    \
        break;
            VO_SMALL_R(5) VO_SMALL_R(6) VO_SMALL_R(8) VO_SMALL_R(10) VO_SMALL_R(13)
#undef VO_SMALL_R
            default:
                for (int e = tid; e < RC; e += VO_SMALL_T) {                 // row pass
                    const int y = e / C, x = e - y * C;
                    const float* row = cur + y * C;
                    float acc = kk[0] * row[x];
                    for (int j = 1; j <= r; ++j) acc = fmaf(kk[j], row[cidx[x + r - j]] + row[cidx[x + r + j]], acc);
                    tmp[e] = acc;
                }
                __syncthreads();
                for (int e = tid; e < RC; e += VO_SMALL_T) {                 // column pass
                    const int y = e / C, x = e - y * C;
                    float acc = kk[0] * tmp[e];
                    for (int j = 1; j <= r; ++j) acc = fmaf(kk[j], tmp[ridx[y + r - j] * C + x] + tmp[ridx[y + r + j] * C + x], acc);
                    nxt[e] = acc;
                    gl[(size_t)y * g.pitch + x] = acc;
                }
            }
            __syncthreads();
            if (i == L && o + 1 < py->n_oct) {                           // next octave's base: decimated G_L
                const int C2 = py->oct[o + 1].cols, R2 = py->oct[o + 1].rows;
                for (int e = tid; e < R2 * C2; e += VO_SMALL_T) {
                    const int y = e / C2, x = e - y * C2;
                    base[e] = nxt[(2 * y) * C + 2 * x];
                }
            }
            float* t2 = cur; cur = nxt; nxt = t2;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// extrema: masks, scan, emit
// ---------------------------------------------------------------------------
__device__ __forceinline__ void decode_word(const Pyramid* __restrict__ py, int w, int& o, int& layer, int& row, int& k)
{
    const int L = py->L;
    int b = 0;
    const int nb = py->n_oct * L;
    while (b + 1 < nb && py->wbase[b + 1] <= w) ++b;
    o = b / L;
    layer = b - o * L + 1;
    int rel = w - py->wbase[b];
    int wr = py->wrow[o];
    row = VO_SIFT_BORDER + rel / wr;
    k = rel - (rel / wr) * wr;
}

// ---------------------------------------------------------------------------
// 26-neighbour extremum test, streaming.  One wave per (image, octave, strip
// of 128 columns, band of VO_EXT_BAND interior rows); lane l owns the adjacent
// columns xs+2l and xs+2l+1.  The wave walks the band's rows (+1 above and below):
// per row it loads the L+3 Gaussian levels (one coalesced 8-B load + one halo
// column: xs-1 in lane 0, xs+128 in lane 63), forms D_l = G_{l+1} - G_l (never
// stored), reduces each level to its horizontal 3-max/3-min -- the outer neighbours
// xs+2l-1 and xs+2l+2 arrive by one DPP wave shift each, lanes 0 / 63 keeping their
// halo column -- and keeps the last 3 rows of those in a register window (rows
// unrolled by 3, static slots).  Row t-1 is then tested: val >= max of its 3x3x3
// block (val included) <=> val >= all 26 neighbours.  The two ballots per (row,
// layer) are the strip's even- and odd-column words (bit l = column xs+2l+c);
// k_seg_emit interleaves each pair back into column order.  Input rows are
// prefetched 3 rows ahead; lanes past the plane's last column (row padding) load nothing.
// ---------------------------------------------------------------------------

// whole-wave lane shifts on the VALU (GFX9 DPP wave_shr:1 / wave_shl:1) instead of
// LDS-routed ds_bpermute shuffles; the lane without a source keeps its own value
__device__ __forceinline__ float vo_wave_shr1_or(float old, float x)   // lane i <- lane i-1; lane 0 <- old
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(x), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float vo_wave_shl1_or(float old, float x)   // lane i <- lane i+1; lane 63 <- old
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(x), 0x130, 0xf, 0xf, false));
}

template <int L>
__global__ __launch_bounds__(64) void k_ext_stream(const Pyramid* __restrict__ py, const float* __restrict__ arena,
                                                   unsigned long long* __restrict__ mask, float thr, int n_img, int u_first,
                                                   int u_last)
{
    vo_ss_prio();
    constexpr int NG = L + 3, ND = L + 2, W = 3;      // Gaussian levels, DoG levels, row window
    const int lane = threadIdx.x;
    const int u_all = xcd_remap(blockIdx.x, gridDim.x);
    // units [u_first, u_last) of every image (a range of octaves; those below a fused prefix
    // are tested by k_octave)
    const int nu = u_last - u_first;
    const int img = u_all / nu;
    int u = u_first + u_all - img * nu;
    int o = 0;
    while (o + 1 < py->n_oct && py->ebase[o + 1] <= u) ++o;
    o = __builtin_amdgcn_readfirstlane(o);
    u -= py->ebase[o];
    const OctGeom& g = py->oct[o];
    const int rows = g.rows, cols = g.cols, pitch = g.pitch;
    const int ns = py->estrips[o];
    const int strip = u % ns, band = u / ns;
    const int ir = rows - 2 * VO_SIFT_BORDER;
    const int r0 = VO_SIFT_BORDER + band * VO_EXT_BAND;                 // first tested row
    const int nrow = min(VO_EXT_BAND, ir - band * VO_EXT_BAND);          // tested rows in this band
    const int xs = strip * 128, xa = xs + 2 * lane, xb = xa + 1;
    // halo columns: lane 63 -> xs+128, the others xs-1 (used by lane 0; same cache line)
    const int hx = lane == 63 ? xs + 128 : max(xs - 1, 0);
    const float* base = arena + img * py->istride;
    size_t goff[NG];
#pragma unroll
    for (int lv = 0; lv < NG; ++lv) goff[lv] = g.g_off[lv];
    const int wr = py->wrow[o];
    unsigned long long* mrow = mask + (size_t)img * py->n_words;
#if VO_EXT_BSTORE
    // mask words by buffer stores issued by every lane every row: lanes other than 0/1 (and rows
    // past the band) get an out-of-range offset and the hardware drops them -- no store branch
    const __amdgpu_buffer_rsrc_t rs_m = __builtin_amdgcn_make_buffer_rsrc(mrow, 0, py->n_words * 8, 0x00020000);
#endif
    int wb[L];                                       // mask word base per layer, hoisted: the mask
#pragma unroll                                       // stores could alias *py for the compiler
    for (int l = 0; l < L; ++l) wb[l] = py->wbase[o * L + l];
    const bool in0 = xa >= VO_SIFT_BORDER && xa < cols - VO_SIFT_BORDER;
    const bool in1 = xb >= VO_SIFT_BORDER && xb < cols - VO_SIFT_BORDER;

    typedef float f2_t __attribute__((ext_vector_type(2)));
    f2_t pm[W][NG];                                  // prefetched columns {xa, xa+1}, per window slot
    float ph[W][NG];                                 // prefetched halo column
    f2_t hmx[W][ND], hmn[W][ND];                     // horizontal 3-max / 3-min per row slot
    f2_t dc[W][L];                                   // D of layers 1..L per row slot (centres)

#define VO_ET_LOAD(T, SL)                                                                          \
    do {                                                                                           \
        const int y_ = min(r0 - 1 + (T), rows - 1);                                                \
        const float* rp_ = base + (size_t)y_ * pitch;                                              \
        _Pragma("unroll") for (int lv = 0; lv < NG; ++lv) {                                        \
            if (xa < cols) pm[SL][lv] = *reinterpret_cast<const f2_t*>(rp_ + goff[lv] + xa);      \
            ph[SL][lv] = rp_[goff[lv] + hx];                                                       \
        }                                                                                          \
    } while (0)

    // one row step: D, horizontal reductions into slot SL; if TEST, test row in slot (SL+2)%3
    auto step = [&](int t, auto sl_c, auto test_c) {
        constexpr int SL = decltype(sl_c)::value;
        f2_t d[ND];
        float hd[ND];
#pragma unroll
        for (int lv = 0; lv < ND; ++lv) {
            d[lv] = pm[SL][lv + 1] - pm[SL][lv];
            hd[lv] = ph[SL][lv + 1] - ph[SL][lv];
        }
        // refill the slot with row t+3 -- only rows the band uses (r0-1 .. r0+nrow): the last
        // steps' prefetches were 3 wasted rows per 30-row band (~9 % of the kernel's fetches)
        if (t + W <= nrow + 1) VO_ET_LOAD(t + W, SL);
#pragma unroll
        for (int lv = 0; lv < ND; ++lv) {
            // outer neighbours: xa-1 = lane l-1's xb (lane 0: its halo xs-1), xb+1 = lane
            // l+1's xa (lane 63: its halo xs+128) -- a lane without a source keeps `old` = hd
            const float la = vo_wave_shr1_or(hd[lv], d[lv].y), rb = vo_wave_shl1_or(hd[lv], d[lv].x);
            hmx[SL][lv] = f2_t{fmaxf(fmaxf(la, d[lv].x), d[lv].y), fmaxf(fmaxf(d[lv].x, d[lv].y), rb)};
            hmn[SL][lv] = f2_t{fminf(fminf(la, d[lv].x), d[lv].y), fminf(fminf(d[lv].x, d[lv].y), rb)};
        }
#pragma unroll
        for (int l = 0; l < L; ++l) dc[SL][l] = d[l + 1];
        if constexpr (decltype(test_c)::value) {
            constexpr int A = (SL + 1) % W, M = (SL + 2) % W;   // rows t-2, t-1 (tested)
            const int r = r0 + t - 2;
            f2_t mx3[ND], mn3[ND];
#pragma unroll
            for (int lv = 0; lv < ND; ++lv) {
                mx3[lv] = f2_t{fmaxf(fmaxf(hmx[A][lv].x, hmx[M][lv].x), hmx[SL][lv].x),
                               fmaxf(fmaxf(hmx[A][lv].y, hmx[M][lv].y), hmx[SL][lv].y)};
                mn3[lv] = f2_t{fminf(fminf(hmn[A][lv].x, hmn[M][lv].x), hmn[SL][lv].x),
                               fminf(fminf(hmn[A][lv].y, hmn[M][lv].y), hmn[SL][lv].y)};
            }
#pragma unroll
            for (int layer = 1; layer <= L; ++layer) {
                bool e[2];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const float val = c ? dc[M][layer - 1].y : dc[M][layer - 1].x;
                    const float bmx = fmaxf(fmaxf(c ? mx3[layer - 1].y : mx3[layer - 1].x, c ? mx3[layer].y : mx3[layer].x),
                                            c ? mx3[layer + 1].y : mx3[layer + 1].x);
                    const float bmn = fminf(fminf(c ? mn3[layer - 1].y : mn3[layer - 1].x, c ? mn3[layer].y : mn3[layer].x),
                                            c ? mn3[layer + 1].y : mn3[layer + 1].x);
                    // |val| > thr && (val > 0 ? val >= bmx : val <= bmn), as lane-mask compares
                    e[c] = ((val > thr) & (val >= bmx)) | ((val < -thr) & (val <= bmn));
                }
                const uint64_t w0 = __ballot(e[0] & in0), w1 = __ballot(e[1] & in1);
                const int k = 2 * strip + lane;               // wr is even: both words exist
#if VO_EXT_BSTORE
                const uint32_t mo = (lane < 2 && t - 2 < nrow) ? (uint32_t)(wb[layer - 1] + (r - VO_SIFT_BORDER) * wr + k) * 8u
                                                               : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(vo_i2, (uint64_t)(lane ? w1 : w0)), rs_m, mo, 0, 0);
#else
                if (lane < 2 && t - 2 < nrow)
                    mrow[wb[layer - 1] + (size_t)(r - VO_SIFT_BORDER) * wr + k] = lane ? w1 : w0;
#endif
            }
        }
    };

    vo_static_for<W>([&](auto c) { VO_ET_LOAD(decltype(c)::value, decltype(c)::value); });
    step(0, std::integral_constant<int, 0>{}, std::false_type{});
    step(1, std::integral_constant<int, 1>{}, std::false_type{});
#pragma unroll 1
    for (int t0 = 2; t0 < nrow + 2; t0 += W) {
        step(t0, std::integral_constant<int, 2>{}, std::true_type{});
        step(t0 + 1, std::integral_constant<int, 0>{}, std::true_type{});
        step(t0 + 2, std::integral_constant<int, 1>{}, std::true_type{});
    }
#undef VO_ET_LOAD
}

// The inner part of the extremum test (VO_EXT_INNER, the default): the same streaming wave with
// only G_1 .. G_{L+1} loaded -- D_1 .. D_L, the centres of every layer and every neighbour level
// except D_0 (layer 1's lower neighbour, G_1 - G_0) and D_{L+1} (layer L's upper one).  A bit is
// set when its centre passes |val| > thr and the extremum test against those streamed levels;
// k_refine completes the test for layers 1 and L (val >= / <= the 9 values of D_0 / D_{L+1})
// before anything else and rejects the centres that fail it.  val >= max of the 27 <=> val >=
// the max of each part, so the keypoints are the full test's; 2 of the L + 3 planes leave the
// streamed bytes (4 (L + 1) B per octave px).  Measured: the extremum test 3.28 -> 2.34 ms, k_refine
// 0.39 -> 0.77 ms isolated (the partial candidates), +3.5-3.9 % stereo frames/s.
template <int L>
__global__ __launch_bounds__(64) void k_ext_inner(const Pyramid* __restrict__ py, const float* __restrict__ arena,
                                                   unsigned long long* __restrict__ mask, float thr, int n_img, int u_first,
                                                   int u_last)
{
    vo_ss_prio();
    constexpr int NG = L + 1, ND = L, W = 3;          // streamed levels G_1..G_{L+1}, DoG D_1..D_L
    const int lane = threadIdx.x;
    const int u_all = xcd_remap(blockIdx.x, gridDim.x);
    const int nu = u_last - u_first;
    const int img = u_all / nu;
    int u = u_first + u_all - img * nu;
    int o = 0;
    while (o + 1 < py->n_oct && py->ebase[o + 1] <= u) ++o;
    o = __builtin_amdgcn_readfirstlane(o);
    u -= py->ebase[o];
    const OctGeom& g = py->oct[o];
    const int rows = g.rows, cols = g.cols, pitch = g.pitch;
    const int ns = py->estrips[o];
    const int strip = u % ns, band = u / ns;
    const int ir = rows - 2 * VO_SIFT_BORDER;
    const int r0 = VO_SIFT_BORDER + band * VO_EXT_BAND;
    const int nrow = min(VO_EXT_BAND, ir - band * VO_EXT_BAND);
    const int xs = strip * 128, xa = xs + 2 * lane, xb = xa + 1;
    const int hx = lane == 63 ? xs + 128 : max(xs - 1, 0);
    const float* base = arena + img * py->istride;
    size_t goff[NG];
#pragma unroll
    for (int lv = 0; lv < NG; ++lv) goff[lv] = g.g_off[lv + 1];
    const int wr = py->wrow[o];
    unsigned long long* mrow = mask + (size_t)img * py->n_words;
#if VO_EXT_BSTORE
    const __amdgpu_buffer_rsrc_t rs_m = __builtin_amdgcn_make_buffer_rsrc(mrow, 0, py->n_words * 8, 0x00020000);
#endif
    int wb[L];
#pragma unroll
    for (int l = 0; l < L; ++l) wb[l] = py->wbase[o * L + l];
    const bool in0 = xa >= VO_SIFT_BORDER && xa < cols - VO_SIFT_BORDER;
    const bool in1 = xb >= VO_SIFT_BORDER && xb < cols - VO_SIFT_BORDER;

    typedef float f2_t __attribute__((ext_vector_type(2)));
    f2_t pm[W][NG];
    float ph[W][NG];
    f2_t hmx[W][ND], hmn[W][ND];
    f2_t dc[W][L];

#define VO_ES_LOAD(T, SL)                                                                          \
    do {                                                                                           \
        const int y_ = min(r0 - 1 + (T), rows - 1);                                                \
        const float* rp_ = base + (size_t)y_ * pitch;                                              \
        _Pragma("unroll") for (int lv = 0; lv < NG; ++lv) {                                        \
            if (xa < cols) pm[SL][lv] = *reinterpret_cast<const f2_t*>(rp_ + goff[lv] + xa);      \
            ph[SL][lv] = rp_[goff[lv] + hx];                                                       \
        }                                                                                          \
    } while (0)

    auto step = [&](int t, auto sl_c, auto test_c) {
        constexpr int SL = decltype(sl_c)::value;
        f2_t d[ND];
        float hd[ND];
#pragma unroll
        for (int lv = 0; lv < ND; ++lv) {
            d[lv] = pm[SL][lv + 1] - pm[SL][lv];
            hd[lv] = ph[SL][lv + 1] - ph[SL][lv];
        }
        if (t + W <= nrow + 1) VO_ES_LOAD(t + W, SL);
#pragma unroll
        for (int lv = 0; lv < ND; ++lv) {
            const float la = vo_wave_shr1_or(hd[lv], d[lv].y), rb = vo_wave_shl1_or(hd[lv], d[lv].x);
            hmx[SL][lv] = f2_t{fmaxf(fmaxf(la, d[lv].x), d[lv].y), fmaxf(fmaxf(d[lv].x, d[lv].y), rb)};
            hmn[SL][lv] = f2_t{fminf(fminf(la, d[lv].x), d[lv].y), fminf(fminf(d[lv].x, d[lv].y), rb)};
        }
#pragma unroll
        for (int l = 0; l < L; ++l) dc[SL][l] = d[l];
        if constexpr (decltype(test_c)::value) {
            constexpr int A = (SL + 1) % W, M = (SL + 2) % W;
            const int r = r0 + t - 2;
            const bool live = t - 2 < nrow;
            f2_t mx3[ND], mn3[ND];
#pragma unroll
            for (int lv = 0; lv < ND; ++lv) {
                mx3[lv] = f2_t{fmaxf(fmaxf(hmx[A][lv].x, hmx[M][lv].x), hmx[SL][lv].x),
                               fmaxf(fmaxf(hmx[A][lv].y, hmx[M][lv].y), hmx[SL][lv].y)};
                mn3[lv] = f2_t{fminf(fminf(hmn[A][lv].x, hmn[M][lv].x), hmn[SL][lv].x),
                               fminf(fminf(hmn[A][lv].y, hmn[M][lv].y), hmn[SL][lv].y)};
            }
#pragma unroll
            for (int layer = 1; layer <= L; ++layer) {
                // streamed DoG D_k sits at index k - 1: D_layer always, D_{layer-1} if layer >= 2,
                // D_{layer+1} if layer <= L - 1
                bool pos[2], neg[2];
                float val[2];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    val[c] = c ? dc[M][layer - 1].y : dc[M][layer - 1].x;
                    float bmx = c ? mx3[layer - 1].y : mx3[layer - 1].x;
                    float bmn = c ? mn3[layer - 1].y : mn3[layer - 1].x;
                    if (layer >= 2) {
                        bmx = fmaxf(bmx, c ? mx3[layer - 2].y : mx3[layer - 2].x);
                        bmn = fminf(bmn, c ? mn3[layer - 2].y : mn3[layer - 2].x);
                    }
                    if (layer <= L - 1) {
                        bmx = fmaxf(bmx, c ? mx3[layer].y : mx3[layer].x);
                        bmn = fminf(bmn, c ? mn3[layer].y : mn3[layer].x);
                    }
                    pos[c] = (val[c] > thr) & (val[c] >= bmx);
                    neg[c] = (val[c] < -thr) & (val[c] <= bmn);
                }
                const uint64_t w0 = __ballot((pos[0] | neg[0]) & in0), w1 = __ballot((pos[1] | neg[1]) & in1);
                const int k = 2 * strip + lane;
#if VO_EXT_BSTORE
                const uint32_t mo = (lane < 2 && live) ? (uint32_t)(wb[layer - 1] + (r - VO_SIFT_BORDER) * wr + k) * 8u
                                                       : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(vo_i2, (uint64_t)(lane ? w1 : w0)), rs_m, mo, 0, 0);
#else
                if (lane < 2 && live)
                    mrow[wb[layer - 1] + (size_t)(r - VO_SIFT_BORDER) * wr + k] = lane ? w1 : w0;
#endif
            }
        }
    };

    vo_static_for<W>([&](auto c) { VO_ES_LOAD(decltype(c)::value, decltype(c)::value); });
    step(0, std::integral_constant<int, 0>{}, std::false_type{});
    step(1, std::integral_constant<int, 1>{}, std::false_type{});
#pragma unroll 1
    for (int t0 = 2; t0 < nrow + 2; t0 += W) {
        step(t0, std::integral_constant<int, 2>{}, std::true_type{});
        step(t0 + 1, std::integral_constant<int, 0>{}, std::true_type{});
        step(t0 + 2, std::integral_constant<int, 1>{}, std::true_type{});
    }
#undef VO_ES_LOAD
}

// Block-wide exclusive scan of one value per thread (1024 threads).
__device__ __forceinline__ uint32_t block_exscan_1024(uint32_t v, uint32_t* sh, uint32_t* total)
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

// Compaction in (octave, layer, row, column) order, three coalesced passes:
// per-segment popcounts (1024 words), per-image exclusive scan of segments,
// then each segment block scans its words and emits candidates.
__global__ __launch_bounds__(256) void k_seg_count(const unsigned long long* __restrict__ mask, uint32_t* __restrict__ segc,
                                                   int nw, int nseg)
{
    __shared__ uint32_t red[4];
    const int img = blockIdx.y, seg = blockIdx.x, tid = threadIdx.x;
    const unsigned long long* m = mask + (size_t)img * nw;
    uint32_t cnt = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int wd = seg * VO_SEG_WORDS + q * 256 + tid;
        if (wd < nw) cnt += (uint32_t)__popcll(m[wd]);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
    if ((tid & 63) == 0) red[tid >> 6] = cnt;
    __syncthreads();
    if (tid == 0) segc[(size_t)img * nseg + seg] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(1024) void k_seg_scan(uint32_t* __restrict__ segc, int* __restrict__ n_cand, int* __restrict__ n_acc,
                                                   int nseg)
{
    if (threadIdx.x == 0) n_acc[blockIdx.x] = 0;           // k_refine appends this image's accepted candidates
    __shared__ uint32_t sh[32];
    const int img = blockIdx.x, tid = threadIdx.x;
    uint32_t v = tid < nseg ? segc[(size_t)img * nseg + tid] : 0u;
    uint32_t total;
    const uint32_t ex = block_exscan_1024(v, sh, &total);
    if (tid < nseg) segc[(size_t)img * nseg + tid] = ex;
    if (tid == 0) n_cand[img] = (int)total;
}

__device__ __forceinline__ uint32_t block_exscan_256(uint32_t v, uint32_t* sh)
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
    uint32_t before = 0;
    for (int q = 0; q < wid; ++q) before += sh[q];
    return before + x - v;
}

// bit i of x -> bit 2i
__device__ __forceinline__ unsigned long long vo_spread32(uint32_t x)
{
    unsigned long long v = x;
    v = (v | v << 16) & 0x0000FFFF0000FFFFull;
    v = (v | v << 8) & 0x00FF00FF00FF00FFull;
    v = (v | v << 4) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | v << 2) & 0x3333333333333333ull;
    v = (v | v << 1) & 0x5555555555555555ull;
    return v;
}

__global__ __launch_bounds__(256) void k_seg_emit(const Pyramid* __restrict__ py, const unsigned long long* __restrict__ mask,
                                                  const uint32_t* __restrict__ segoff, uint32_t* __restrict__ cand,
                                                  int cand_cap)
{
    __shared__ uint32_t sh[4];
    const int img = blockIdx.y, seg = blockIdx.x, tid = threadIdx.x;
    const int nw = py->n_words;
    const unsigned long long* m = mask + (size_t)img * nw;
    const int w0 = seg * VO_SEG_WORDS + tid * 4;     // 4 consecutive words per thread
    unsigned long long mw[4];
    uint32_t cnt = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        mw[q] = (w0 + q < nw) ? m[w0 + q] : 0ull;
        cnt += (uint32_t)__popcll(mw[q]);
    }
    // k_ext_stream writes a strip's words as (even columns, odd columns); w0 and every mask
    // row start are even, so each (q, q+1) pair is one strip: interleave into column order
#pragma unroll
    for (int q = 0; q < 4; q += 2) {
        const unsigned long long ev = mw[q], od = mw[q + 1];
        mw[q] = vo_spread32((uint32_t)ev) | vo_spread32((uint32_t)od) << 1;
        mw[q + 1] = vo_spread32((uint32_t)(ev >> 32)) | vo_spread32((uint32_t)(od >> 32)) << 1;
    }
    uint32_t idx = segoff[(size_t)img * py->n_seg + seg] + block_exscan_256(cnt, sh);
    if (!cnt) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        unsigned long long mm = mw[q];
        if (!mm) continue;
        int o, layer, r, k;
        decode_word(py, w0 + q, o, layer, r, k);
        while (mm) {
            const int bit = __ffsll((long long)mm) - 1;
            mm &= mm - 1;
            if (idx < (uint32_t)cand_cap) cand[(size_t)img * cand_cap + idx] = pack_cand(o, layer, r, 64 * k + bit);
            idx++;
        }
    }
}

// ---------------------------------------------------------------------------
// refinement + orientation: one wave (block of 64) per candidate
// ---------------------------------------------------------------------------
// Flat item space over images: item t of image i is t - pre[i] for
// pre[i] <= t < pre[i+1], pre[i+1] = pre[i] + min(counts[i], cap).  The prefix
// is built once per block in LDS (all threads call flat_setup); flat_find is
// then a binary search instead of a per-item walk over the images.
// Cross-lane trees without LDS (gfx950 v_permlane32_swap / v_permlane16_swap and DPP row shifts).
// wave_tree_sum: lane 0's value is the pairwise tree of the shfl_down(32, 16, .., 1) loop, bit for
// bit (each step adds lane l + st to lane l), returned to every lane.
template <typename T>
__device__ __forceinline__ T wave_tree_sum(T v)
{
    auto bits = [](T x) { return __builtin_bit_cast(int, x); };
    auto val = [](int x) { return __builtin_bit_cast(T, x); };
    v = v + val(__builtin_amdgcn_permlane32_swap(bits(v), bits(v), false, false)[1]);   // lanes < 32: v[l + 32]
    v = v + val(__builtin_amdgcn_permlane16_swap(bits(v), bits(v), false, false)[1]);   // lanes < 16: v[l + 16]
    v = v + val(__builtin_amdgcn_update_dpp(0, bits(v), 0x108, 0xF, 0xF, true));        // row_shl:8
    v = v + val(__builtin_amdgcn_update_dpp(0, bits(v), 0x104, 0xF, 0xF, true));        // row_shl:4
    v = v + val(__builtin_amdgcn_update_dpp(0, bits(v), 0x102, 0xF, 0xF, true));        // row_shl:2
    v = v + val(__builtin_amdgcn_update_dpp(0, bits(v), 0x101, 0xF, 0xF, true));        // row_shl:1
    return val(__builtin_amdgcn_readlane(bits(v), 0));
}
// maximum over the 64 lanes (order-free), returned to every lane
__device__ __forceinline__ float wave_max(float v)
{
    auto bits = [](float x) { return __float_as_int(x); };
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_permlane32_swap(bits(v), bits(v), false, false)[1]));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_permlane16_swap(bits(v), bits(v), false, false)[1]));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(bits(v), bits(v), 0x108, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(bits(v), bits(v), 0x104, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(bits(v), bits(v), 0x102, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(bits(v), bits(v), 0x101, 0xF, 0xF, false)));
    return __int_as_float(__builtin_amdgcn_readlane(bits(v), 0));
}
// inclusive prefix sum over the 64 lanes (integers): row shifts, then the row broadcasts
__device__ __forceinline__ int wave_incl_scan(int x)
{
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 into rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 into rows 2, 3
    return x;
}

#define VO_FLAT_MAX_IMG (2 * VO_MAX_BATCH + 2)   // 2 * max_batch + 2 image slots
__device__ __forceinline__ long flat_setup(const int* __restrict__ counts, int cap, int n_img, int* pre)
{
    const int tid = threadIdx.x, nt = blockDim.x;
    __shared__ int carry;
    if (tid == 0) { carry = 0; pre[0] = 0; }
    __syncthreads();
    for (int b0 = 0; b0 < n_img; b0 += 64) {          // the first wave scans 64 images per round
        if (tid < 64) {
            const int i = b0 + tid;
            const int c = i < n_img ? min(counts[i], cap) : 0;
            const int x = wave_incl_scan(c);               // (wave 0 whole: tid < 64)
            const int base = carry;
            if (i < n_img) pre[i + 1] = base + x;
            const int tot = __builtin_amdgcn_readlane(x, 63);
            if (tid == 0) carry = base + tot;
        }
        __syncthreads();
    }
    (void)nt;
    return pre[n_img];
}

__device__ __forceinline__ void flat_find(const int* pre, int n_img, long t, int& img, int& k)
{
    int lo = 0, hi = n_img - 1;                       // largest i with pre[i] <= t
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= t) lo = mid; else hi = mid - 1;
    }
    img = lo;
    k = (int)(t - pre[lo]);
}

// flat_find for one whole wave (all 64 lanes active, t wave-uniform): the prefix is nondecreasing,
// so the image is the number of i in [1, n_img) with pre[i] <= t -- one round of independent LDS
// reads and ballots instead of a binary search's chain of dependent reads
__device__ __forceinline__ void flat_find_wave(const int* pre, int n_img, long t, int& img, int& k)
{
    const int lane = threadIdx.x & 63;
    int cnt = 0;
#pragma unroll
    for (int b = 0; b < VO_FLAT_MAX_IMG; b += 64) {
        if (b >= n_img - 1) break;                      // uniform
        const int i = b + 1 + lane;
        cnt += __popcll(__ballot(i < n_img && pre[i] <= t));
    }
    img = cnt;
    k = (int)(t - pre[cnt]);
}

// sqrtf(x), correctly rounded, for x == +0 or 2^-96 <= x < inf: the compiler's IEEE sqrt less its
// small-argument scaling and special-class select -- v_sqrt_f32 and the same two one-ulp
// residual corrections, so the value is sqrtf's.  The gradient magnitudes call it on sums of
// squares and fall back to sqrtf for the whole wave if any lane has 0 < x < 2^-96.
__device__ __forceinline__ float vo_sqrtf_big(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u), sup = __uint_as_float(__float_as_uint(s) + 1u);
    const float rdn = fmaf(-sdn, s, x), rup = fmaf(-sup, s, x);
    const float s1 = rdn <= 0.0f ? sdn : s;
    return rup > 0.0f ? sup : s1;
}
__device__ __forceinline__ float vo_grad_mag(float dx, float dy)
{
    const float x = dx * dx + dy * dy;
    float m = vo_sqrtf_big(x);
    if (__builtin_expect(__ballot(x > 0.0f && x < 0x1p-96f) != 0ull, 0)) m = sqrtf(x);   // wave-uniform
    return m;
}

#define DAT(p, P, y, x) ((p)[(size_t)(y) * (P) + (x)])

// 3x3 Cramer solve in double (same expression tree as oracle solve3)
__device__ __forceinline__ void solve3_dev(const float H[9], const float b[3], float X[3])
{
    double a00 = H[0], a01 = H[1], a02 = H[2], a10 = H[3], a11 = H[4], a12 = H[5], a20 = H[6], a21 = H[7], a22 = H[8];
    double c00 = a11 * a22 - a12 * a21, c01 = a10 * a22 - a12 * a20, c02 = a10 * a21 - a11 * a20;
    double det = a00 * c00 - a01 * c01 + a02 * c02;
    if (det == 0.0) { X[0] = X[1] = X[2] = 0.0f; return; }
    double b0 = b[0], b1 = b[1], b2 = b[2];
    double x0 = b0 * c00 - a01 * (b1 * a22 - a12 * b2) + a02 * (b1 * a21 - a11 * b2);
    double x1 = a00 * (b1 * a22 - a12 * b2) - b0 * c01 + a02 * (a10 * b2 - b1 * a20);
    double x2 = a00 * (a11 * b2 - b1 * a21) - a01 * (a10 * b2 - b1 * a20) + b0 * c02;
    double inv = 1.0 / det;
    X[0] = (float)(x0 * inv); X[1] = (float)(x1 * inv); X[2] = (float)(x2 * inv);
}

// Refinement (adjustLocalExtrema + contrast/edge tests): one LANE per candidate.
// The interpolation loop is the same expression sequence as the oracle's; lanes
// of a wave work on different candidates (divergent iteration counts are fine).
// Writes the refined fields of CandOut with npk = -1 (accepted, orientation
// pending) or 0 (rejected).
#ifndef VO_REFINE_BLOCKS
#define VO_REFINE_BLOCKS 512      // grid-stride workgroups of 256 lanes (one lane per candidate)
#endif
__global__ __launch_bounds__(256) void k_refine(const Pyramid* __restrict__ py, const float* __restrict__ arena,
                                                const uint32_t* __restrict__ cand, const int* __restrict__ n_cand,
                                                CandOut* __restrict__ cout, int* __restrict__ acc, int* __restrict__ n_acc,
                                                uint32_t* __restrict__ knpk,
                                                int cand_cap, int n_img, float contrast_thr, float edge_thr, float sigma)
{
    const int L = py->L;
    __shared__ int fpre[VO_FLAT_MAX_IMG + 1];
    const long total = flat_setup(n_cand, cand_cap, n_img, fpre);
    for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
        int img, kidx;
        flat_find(fpre, n_img, t, img, kidx);
        const uint32_t pc = cand[(size_t)img * cand_cap + kidx];
        const int c0 = pc & 4095, r0 = (pc >> 12) & 4095, layer0 = (pc >> 24) & 7, o = pc >> 27;
        const OctGeom& g = py->oct[o];
        const int rows = g.rows, cols = g.cols, P = g.pitch;
        const size_t lstride = g.g_off[1] - g.g_off[0];    // next Gaussian level of the same image
#define DOGV(p, P, y, x) (DAT((p) + lstride, P, y, x) - DAT(p, P, y, x))
        CandOut* out = cout + (size_t)img * cand_cap + kidx;
        // ---- adjustLocalExtrema ----
        const float img_scale = 1.0f / 255.0f;
        const float ds = img_scale * 0.5f, ss = img_scale, cs = img_scale * 0.25f;
        int r = r0, c = c0, layer = layer0;
        float xi = 0, xr = 0, xc = 0;
        int it = 0;
        bool ok = true;
        // the last step's terms at its (r, c, layer): the contrast / edge tests below need exactly
        // these (the loop only exits with ok at convergence, without moving), so they are kept
        // instead of re-read
        float kD[3] = {0, 0, 0}, kv = 0, kxx = 0, kyy = 0, kxy = 0;
#if VO_EXT_INNER
        // the extremum test's remaining part (k_ext_inner streams G_1 .. G_{L+1} only): a centre of
        // layer 1 / L must also be >= (val > 0) or <= (val < 0) the 9 values of D_0 / D_{L+1}
        // around it.  It passed the rest of the 26-neighbour test with |val| > thr, so this is
        // the dense kernel's mask bit exactly; a candidate that fails is rejected here.
        if (layer0 == 1 || layer0 == L) {
            const float* gb = arena + img * py->istride;
            const float v = DOGV(gb + g.g_off[layer0], P, r0, c0);
            // v >= the max of the 9 <=> v >= each: the value straight below / above first (2 loads;
            // most partial candidates that fail, fail there), the other 8 only if it passes
            auto beats = [&](float d) { return v > 0.0f ? v >= d : v <= d; };
            if (layer0 == 1) ok = beats(DOGV(gb + g.g_off[0], P, r0, c0));
            if (layer0 == L) ok = ok && beats(DOGV(gb + g.g_off[L + 1], P, r0, c0));
            if (ok) {
                float mx = -INFINITY, mn = INFINITY;
                auto ring = [&](const float* pl) {
#pragma unroll
                    for (int q = 0; q < 9; ++q) {
                        if (q == 4) continue;
                        const float d = DOGV(pl, P, r0 + q / 3 - 1, c0 + q % 3 - 1);
                        mx = fmaxf(mx, d); mn = fminf(mn, d);
                    }
                };
                if (layer0 == 1) ring(gb + g.g_off[0]);
                if (layer0 == L) ring(gb + g.g_off[L + 1]);
                ok = v > 0.0f ? v >= mx : v <= mn;
            }
        }
        if (ok)
#endif
        for (; it < VO_SIFT_MAX_INTERP; ++it) {
            const float* gb = arena + img * py->istride;
            const float* im = gb + g.g_off[layer];          // DoG level l = G_{l+1} - G_l (VO_DOG)
            // the neighbour levels as +-lstride from im (the planes of an octave are lstride
            // apart), so the loads DOGV(pv) / DOGV(nx) share with DOGV(im) are one load each
            const float* pv = im - lstride;
            const float* nx = im + lstride;
            float dD[3] = {(DOGV(im, P, r, c + 1) - DOGV(im, P, r, c - 1)) * ds,
                           (DOGV(im, P, r + 1, c) - DOGV(im, P, r - 1, c)) * ds,
                           (DOGV(nx, P, r, c) - DOGV(pv, P, r, c)) * ds};
            const float vc = DOGV(im, P, r, c);
            float v2 = vc * 2.0f;
            float dxx = (DOGV(im, P, r, c + 1) + DOGV(im, P, r, c - 1) - v2) * ss;
            float dyy = (DOGV(im, P, r + 1, c) + DOGV(im, P, r - 1, c) - v2) * ss;
            float dss = (DOGV(nx, P, r, c) + DOGV(pv, P, r, c) - v2) * ss;
            float dxy = (DOGV(im, P, r + 1, c + 1) - DOGV(im, P, r + 1, c - 1) - DOGV(im, P, r - 1, c + 1) + DOGV(im, P, r - 1, c - 1)) * cs;
            float dxs = (DOGV(nx, P, r, c + 1) - DOGV(nx, P, r, c - 1) - DOGV(pv, P, r, c + 1) + DOGV(pv, P, r, c - 1)) * cs;
            float dys = (DOGV(nx, P, r + 1, c) - DOGV(nx, P, r - 1, c) - DOGV(pv, P, r + 1, c) + DOGV(pv, P, r - 1, c)) * cs;
            float H[9] = {dxx, dxy, dxs, dxy, dyy, dys, dxs, dys, dss};
            kD[0] = dD[0]; kD[1] = dD[1]; kD[2] = dD[2]; kv = vc; kxx = dxx; kyy = dyy; kxy = dxy;
            float X[3];
            solve3_dev(H, dD, X);
            xi = -X[2]; xr = -X[1]; xc = -X[0];
            if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
            const float big = (float)(0x7fffffff / 3);
            if (fabsf(xi) > big || fabsf(xr) > big || fabsf(xc) > big) { ok = false; break; }
            c += vo_round(xc); r += vo_round(xr); layer += vo_round(xi);
            if (layer < 1 || layer > L || c < VO_SIFT_BORDER || c >= cols - VO_SIFT_BORDER ||
                r < VO_SIFT_BORDER || r >= rows - VO_SIFT_BORDER) { ok = false; break; }
        }
        if (it >= VO_SIFT_MAX_INTERP) ok = false;
        float xo = 0, yo = 0, scl = 0, resp = 0;
        if (ok) {
            float tt = kD[0] * xc + kD[1] * xr + kD[2] * xi;
            float contr = kv * img_scale + tt * 0.5f;
            if (fabsf(contr) * (float)L < contrast_thr) ok = false;
            const float dxx = kxx, dyy = kyy, dxy = kxy;
            float tr = dxx + dyy, det = dxx * dyy - dxy * dxy;
            if (det <= 0 || tr * tr * edge_thr >= (edge_thr + 1) * (edge_thr + 1) * det) ok = false;
            xo = (float)c + xc;
            yo = (float)r + xr;
            scl = sigma * vo_expf(((float)layer + xi) / (float)L * 0.693147181f);
            resp = fabsf(contr);
        }
        // Every candidate's record is stored, although with the accepted list (VO_ACC_LIST,
        // VO_NPK_COMPACT) nothing reads a rejected one's: storing only the accepted ones (~13 %)
        // cut k_refine's own time 1.14 -> 0.98 ms and its PMC bytes 5.34 -> 4.84 GB per 256-frame
        // step, but the step got 3 % slower (10181 -> 9878 stereo frames/s on one box, the level
        // blurs beside it 20.4 -> 21.6 ms in situ, profiles/r06_s_ab_round6_bisect.txt; re-measured
        // with the full path: configs[1] -2.4 %, full path within noise, r06_v_ab_fullpath_cpl_refine.txt)
        out->xo = xo; out->yo = yo; out->scl = scl; out->response = resp;
        out->o = o; out->layer = layer; out->r = r; out->c = c;
        out->npk = ok ? -1 : 0;
#if VO_NPK_COMPACT
        knpk[(size_t)img * cand_cap + kidx] = ok ? 0xFFFFFFFFu : 0u;   // k_orient writes the accepted ones' count
#endif
        // the accepted candidates as a list (k_orient walks only those: on KITTI-00 street frames
        // ~6 in 7 candidates are rejected here, profiles/r05_d_content_pmc_*); the list order is
        // free -- every result is stored at its candidate's index
#if VO_ACC_LIST
        // one atomic per (wave, image): the lanes of a wave hold consecutive candidates, one image
        // (two at an image boundary); per-lane atomics on 128 counters serialised k_refine 7x
        unsigned long long todo = __ballot(ok);
        while (todo) {
            const int leader = __builtin_ctzll(todo);
            const int limg = __shfl(img, leader);
            const unsigned long long m = __ballot(ok && img == limg);
            int base = 0;
            if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(n_acc + limg, __popcll(m));
            base = __shfl(base, leader);
            if (ok && img == limg) acc[(size_t)limg * cand_cap + base + __popcll(m & ((1ull << (threadIdx.x & 63)) - 1ull))] = kidx;
            todo &= ~m;
        }
#endif
#undef DOGV
    }
}

// One histogram weight to fixed point: vo_desc_fx_quant's floor(v + 1/2) is v_cvt_rpi_i32_f32
// (exact: v + 1/2 is representable for every weight, v < 2^22; tests/test_gpu_golden.py and the
// descriptor parity tests hold it to the oracle's floorf bit for bit)
__device__ __forceinline__ uint32_t desc_fxq(float v)
{
    int r;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(v));
    return (uint32_t)r;
}

// Orientation assignment: one wave per accepted candidate (npk == -1).  Each
// lane accumulates its samples' fixed-point weights (vo_desc_fx_quant, 2^-10)
// into histogram column l mod NC, hp[bin][column] (column c's words lie in LDS
// banks c mod 64; zeroed with 16-B stores); the 36 bins are then summed over the
// NC columns in 64 bits (integer sums: identical to the oracle's sequential
// total), lane b reading bin b's partials in a rotated order.  Samples are
// processed 4 per lane per iteration with every gradient load issued first.
// Smoothing, peak test and interpolation as the oracle.  (A column's u32 partial
// of one bin holds < 11k samples' weights: windows up to NC x 11k samples.)
// 16 histogram columns (lanes l, l+16, l+32, l+48 share one through returnless LDS adds): 2.3 KB
// of histogram instead of 10.5 KB at 64 columns -- 32 columns took k_orient 0.68 -> 0.53 ms (5
// waves per SIMD instead of 3.75), 16 columns 0.46-0.48 -> 0.44 ms isolated and 0.63-0.66 -> 0.57
// in situ, where the LDS it leaves goes to the blur waves sharing its CUs (profiles/r04_zc_*)
#ifndef VO_ORIENT_COLS
#define VO_ORIENT_COLS 16
#endif
#ifndef VO_ORIENT_WAVES
#define VO_ORIENT_WAVES 1
#endif
// The orientation assignment of one accepted candidate by the whole wave (k_orient's body):
// histogram, smoothing, peaks; writes out->ang[0..npk),
// out->npk and *knpk_slot.  Returns npk (wave-uniform).
template <int HS>
__device__ __forceinline__ int orient_candidate(const Pyramid* __restrict__ py, const float* __restrict__ arena, CandOut* out,
                                                uint32_t* knpk_slot, int img, uint32_t* hp, float* tf, float* hs)
{
    constexpr int NC = VO_ORIENT_COLS;
    const int lane = threadIdx.x;
    const int o = __builtin_amdgcn_readfirstlane(out->o), layer = __builtin_amdgcn_readfirstlane(out->layer);
    const int r = __builtin_amdgcn_readfirstlane(out->r), c = __builtin_amdgcn_readfirstlane(out->c);
    const float scl = out->scl;
    const OctGeom& g = py->oct[o];
    const int rows = g.rows, cols = g.cols, P = g.pitch;
    // ---- orientation histogram ----
    const float* gim = arena + g.g_off[layer] + img * py->istride;
    const int radius = vo_round(VO_SIFT_ORI_RADIUS * scl);
    const float sigw = VO_SIFT_ORI_SIG * scl;
    const float expf_scale = -1.0f / (2.0f * sigw * sigw);
    typedef uint32_t u4_t __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int b2 = 4 * lane; b2 < HS * NC; b2 += 256) *reinterpret_cast<u4_t*>(&hp[b2]) = u4_t{0u, 0u, 0u, 0u};
    __syncthreads();
#if defined(VO_ORIENT_DIAG)
    const int side = 2 * radius + 1, nsamp = 0;  // diagnostic build (timing only): no sample loop
#else
    const int side = 2 * radius + 1, nsamp = side * side;
#endif
    const float inv_side = 1.0f / (float)side;          // (s + 0.5) * inv_side is exact enough to floor (s < 2^22)
    // gradient loads through a buffer resource based at gim - P - 1: one 32-bit lane offset
    // (the window row as a 24-bit multiply of the clamped row step), row y as one 12-B load
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void*)(gim - P - 1), 0, 0x7FFFFFF0, 0x00020000);
    const int c_off = r * P + c;                      // wave-uniform
    constexpr int U = 4;
    for (int s0 = lane; s0 < nsamp; s0 += 64 * U) {
        float gx[U], gy[U];
        int ii[U], jj[U];
        bool okk[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {                 // indices, bounds, gradient loads
            const int s = s0 + 64 * q;
            const float sf = (float)s, iqf = truncf((sf + 0.5f) * inv_side);
            const int i = (int)iqf - radius, j = (int)(sf - iqf * (float)side) - radius;   // exact: < 2^24
            const int y = r + i, x = c + j;
            ii[q] = i; jj[q] = j;
            okk[q] = (s < nsamp) & (y > 0) & (y < rows - 1) & (x > 0) & (x < cols - 1);
            // every lane loads (clamped to the interior, weight masked below): no branches
            const int ic = min(max(i, 1 - r), rows - 2 - r), jc = min(max(j, 1 - c), cols - 2 - c);
            const int vo = 4 * (c_off + __mul24(ic, P) + jc);
            typedef int i3_t __attribute__((ext_vector_type(3)));
            const i3_t h = __builtin_amdgcn_raw_buffer_load_b96(grs, vo, 4 * P, 0);
            gx[q] = __int_as_float(h.z) - __int_as_float(h.x);
            gy[q] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(grs, vo + 4, 0, 0)) -
                    __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(grs, vo + 4, 8 * P, 0));
        }
#pragma unroll
        for (int q = 0; q < U; ++q) {
            const float dx = gx[q], dy = gy[q];
            // one exp of the combined argument (i^2 + j^2 exact in float); a separable table
            // (vo_sift_wt, as k_desc uses) measured slower here: 0.60 vs 0.55 ms isolated -- its
            // two dependent LDS reads per sample cost more than the exp (profiles/r04_d_*)
            const float fi = (float)ii[q], fj = (float)jj[q];
            const float w = vo_expf_nonpos((fi * fi + fj * fj) * expf_scale);   // arg in [-21, 0]
            float mag = vo_grad_mag(dx, dy);
            float ori = vo_atan2_deg(dy, dx);
            int bin = vo_round((float)VO_SIFT_ORI_BINS / 360.0f * ori);   // ori in [0, 360): bin in [0, 36]
            if (bin >= VO_SIFT_ORI_BINS) bin -= VO_SIFT_ORI_BINS;
            const uint32_t qv = desc_fxq((w * mag) * VO_DESC_FX_SCALE);
            // private column, bank = lane; masked samples add 0; a returnless LDS add, so the
            // update does not wait for the column's old value
            atomicAdd(&hp[bin * NC + (lane & (NC - 1))], okk[q] ? qv : 0u);
        }
    }
    __syncthreads();
    if (lane < VO_SIFT_ORI_BINS) {
        uint64_t acc = 0;                             // bin = lane; step q reads column (q + lane) mod NC
        for (int q = 0; q < NC; ++q) acc += hp[lane * NC + ((q + lane) & (NC - 1))];
        tf[lane] = vo_hist_fx_to_float(acc);
    }
    __syncthreads();
    const int n = VO_SIFT_ORI_BINS;
    float hv = -INFINITY;
    if (lane < n) {
        float m2 = tf[(lane + n - 2) % n], m1 = tf[(lane + n - 1) % n], p1 = tf[(lane + 1) % n], p2 = tf[(lane + 2) % n];
        hv = (m2 + p2) * (1.0f / 16.0f) + (m1 + p1) * (4.0f / 16.0f) + tf[lane] * (6.0f / 16.0f);
        hs[lane] = hv;
    }
    const float mx = wave_max(hv);
    __syncthreads();
    const float mag_thr = mx * VO_SIFT_ORI_PEAK;
    bool pk = false;
    float ang = 0.0f;
    if (lane < n) {
        const int l = lane > 0 ? lane - 1 : n - 1, r2 = lane < n - 1 ? lane + 1 : 0;
        const float hl = hs[l], hr = hs[r2];
        if (hv > hl && hv > hr && hv >= mag_thr) {
            pk = true;
            float bin = (float)lane + 0.5f * (hl - hr) / (hl - 2.0f * hv + hr);
            bin = bin < 0 ? (float)n + bin : bin >= (float)n ? bin - (float)n : bin;
            ang = 360.0f - (360.0f / (float)n) * bin;
            if (fabsf(ang - 360.0f) < VO_FLT_EPSILON) ang = 0.0f;
        }
    }
    const unsigned long long bal = __ballot(pk);
    if (pk) {
        const int rank = __popcll(bal & ((1ull << lane) - 1ull));
        out->ang[rank] = ang;
    }
    __syncthreads();
    if (lane == 0) {
        out->npk = __popcll(bal);
#if VO_NPK_COMPACT
        *knpk_slot = (uint32_t)__popcll(bal);
#endif
    }
    return __popcll(bal);
}

template <int HS>
__global__ __launch_bounds__(64, VO_ORIENT_WAVES) void k_orient(const Pyramid* __restrict__ py, const float* __restrict__ arena,
                                               const int* __restrict__ n_acc, const int* __restrict__ acc,
                                               CandOut* __restrict__ cout, uint32_t* __restrict__ knpk, int cand_cap, int n_img)
{
    // HS: bins per lane column (>= 36).  Layout hp[bin * 64 + lane].
    constexpr int NC = VO_ORIENT_COLS;             // histogram columns: lane l adds into column l % NC
    static_assert(HS >= VO_SIFT_ORI_BINS && (HS * NC) % 4 == 0 && (NC == 64 || NC == 32 || NC == 16), "columns hold the 36 bins");
    __shared__ __attribute__((aligned(16))) uint32_t hp[HS * NC];
    __shared__ float tf[VO_SIFT_ORI_BINS];
    __shared__ float hs[VO_SIFT_ORI_BINS];
    extern __shared__ int fpre[];                    // n_img + 1 ints (dynamic: sized by the launch)
    const long total = flat_setup(n_acc, cand_cap, n_img, fpre);
    for (long t = blockIdx.x; t < total; t += gridDim.x) {
        int img, a;
        flat_find_wave(fpre, n_img, t, img, a);
#if VO_ACC_LIST
        const int kidx = __builtin_amdgcn_readfirstlane(acc[(size_t)img * cand_cap + a]);
#else
        const int kidx = a;                              // every candidate (n_acc = n_cand)
#endif
        CandOut* out = cout + (size_t)img * cand_cap + kidx;
        if (!VO_ACC_LIST && __builtin_amdgcn_readfirstlane(out->npk) != -1) continue;
        orient_candidate<HS>(py, arena, out, knpk + (size_t)img * cand_cap + kidx, img, hp, tf, hs);
    }
}

// per image exclusive scan of npk -> koff, n_kp. grid n_img, block 1024
__global__ __launch_bounds__(1024) void k_scan_cands(const CandOut* __restrict__ cout, const int* __restrict__ n_cand,
                                                     uint32_t* __restrict__ koff, int* __restrict__ n_kp, int cand_cap)
{
    __shared__ uint32_t sh[32];
    const int img = blockIdx.x, tid = threadIdx.x;
    int n = n_cand[img];
    if (n > cand_cap) n = cand_cap;
    const CandOut* co = cout + (size_t)img * cand_cap;
    uint32_t* ko = koff + (size_t)img * cand_cap;
    const int chunk = (n + 1023) / 1024;
    const int a = tid * chunk, e = min(a + chunk, n);
    uint32_t s = 0;
#if VO_NPK_COMPACT
    // the peak counts as k_refine / k_orient left them in koff (4 B per candidate instead of a
    // CandOut line each), scanned in place
    (void)co;
    for (int k = a; k < e; ++k) s += ko[k];
    uint32_t total;
    uint32_t base = block_exscan_1024(s, sh, &total);
    for (int k = a; k < e; ++k) { const uint32_t v = ko[k]; ko[k] = base; base += v; }
#else
    for (int k = a; k < e; ++k) s += (uint32_t)co[k].npk;
    uint32_t total;
    uint32_t base = block_exscan_1024(s, sh, &total);
    for (int k = a; k < e; ++k) { ko[k] = base; base += (uint32_t)co[k].npk; }
#endif
    if (tid == 0) n_kp[img] = (int)total;
}

// one thread per accepted candidate (k_refine's list; each writes its own keypoint slots, so the
// list order does not matter)
__global__ void k_expand(const CandOut* __restrict__ cout, const int* __restrict__ n_acc, const int* __restrict__ acc,
                         const uint32_t* __restrict__ koff, vo_keypoint* __restrict__ kp, KpInt* __restrict__ kpi,
                         int cand_cap, int kp_cap, int n_img, int upsample)
{
    __shared__ int fpre[VO_FLAT_MAX_IMG + 1];
    const long total = flat_setup(n_acc, cand_cap, n_img, fpre);
    for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
        int img, a;
        flat_find(fpre, n_img, t, img, a);
        const int k = VO_ACC_LIST ? acc[(size_t)img * cand_cap + a] : a;
        const CandOut& co = cout[(size_t)img * cand_cap + k];
        const int npk = co.npk;
        if (!npk) continue;
        const uint32_t base = koff[(size_t)img * cand_cap + k];
        // octave pixel k <-> original 2^o k / 2 - 0.25 (half-pixel-centre upsample); +1 = 1-based
        const float oscale = (float)(1 << co.o) * (upsample ? 0.5f : 1.0f);
        const float loc_off = upsample ? 0.75f : 1.0f;
        for (int p = 0; p < npk; ++p) {
            const uint32_t idx = base + p;
            if (idx >= (uint32_t)kp_cap) break;
            vo_keypoint q;
            q.x = co.xo * oscale + loc_off;
            q.y = co.yo * oscale + loc_off;
            q.size = co.scl * 2.0f * oscale;
            q.angle = co.ang[p];
            q.response = co.response;
            q.octave = co.o - (upsample ? 1 : 0);
            q.layer = co.layer;
            q.scale = co.scl * oscale;
            kp[(size_t)img * kp_cap + idx] = q;
            KpInt qi;
            qi.xo = co.xo; qi.yo = co.yo; qi.scl = co.scl; qi.angle = co.ang[p];
            qi.o = co.o; qi.layer = co.layer; qi.pad0 = 0; qi.pad1 = 0;
            kpi[(size_t)img * kp_cap + idx] = qi;
        }
    }
}

// ---------------------------------------------------------------------------
// descriptor: one wave (block of 64) per keypoint
// ---------------------------------------------------------------------------
#define DW VO_SIFT_DESCR_W
#define DN VO_SIFT_DESCR_BINS
// bin stride DN + 1: o0 in [0, DN) so o0 + 1 <= DN -- one wrap bin per cell, folded into bin 0
#define DBS (DN + 1)
#define DHIST ((DW + 2) * (DW + 2) * DBS)
// Histogram copies: lane l adds into copy (l & (DCOPIES-1)), so neighbouring samples
// (same cell, often the same orientation bin) no longer serialise on one LDS address.
// Copy stride DCS = 324 dwords (= 4 mod 64 banks).  Measured (SQ_LDS_BANK_CONFLICT /
// SQ_LDS_IDX_ACTIVE): 0.50 at 324; 0.62 at 336 (16 mod 64, disjoint bank windows for the 9
// bins of a cell in the four copies), same k_desc time -- the adds scatter over cells and
// orientation bins, and the LDS is ~46 % busy, so k_desc is bound by its per-sample VALU.
// u32 fixed point (vo_desc_fx_quant) sums are order-free, so the copies are folded after
// the loop without changing a bit.
#define DCS 324
#ifndef VO_DESC_COPIES
#define VO_DESC_COPIES 4
#endif
#ifndef VO_DESC_WAVES
#define VO_DESC_WAVES 5           // waves per SIMD the register budget is sized for (96 VGPRs)
#endif
#ifndef VO_DESC_U
#define VO_DESC_U 2               // blocks of 64 samples per batch
#endif

// The keypoint's descriptor window tables into LDS (hdr, rtab, wtab; layout of dt_stride): its rotation,
// radius, sample count, row table -- each window row i's column interval [jlo, jhi] inside the
// rotated 4x4-cell square and the image interior, flattened by a prefix sum -- and the separable
// window weights.  Ends with the tables visible to the whole wave.
// One packed row entry per window row r: (index of the row's first sample) | (its first column j,
// int16) << 16; entry nrows is the sample count, entries nrows+1 .. nrows+8 a 0xFFFF sentinel
// start.  Starts fit 16 bits: a window never holds more than its (2 r + 1)^2 square, which
// the cap r <= VO_SIFT_DESCR_RMAX = 127 bounds by 65025 (the rotated square alone is
// ~2 r^2 + O(r) samples, but a capped radius can leave the whole square inside it).
static_assert((2 * VO_SIFT_DESCR_RMAX + 1) * (2 * VO_SIFT_DESCR_RMAX + 1) <= 0xFFFF, "16-bit row starts");
__device__ __forceinline__ void desc_tables(const Pyramid* __restrict__ py, KpInt q, int dcap, uint32_t* hdr, uint32_t* rtab,
                                            float* wtab, int lane)
{
    q.o = __builtin_amdgcn_readfirstlane(q.o);
    q.layer = __builtin_amdgcn_readfirstlane(q.layer);
    const OctGeom& g = py->oct[q.o];
    const int rows = g.rows, cols = g.cols;
    float ori = 360.0f - q.angle;
    if (fabsf(ori - 360.0f) < VO_FLT_EPSILON) ori = 0.0f;
    const int px = vo_round(q.xo), pyy = vo_round(q.yo);
    float sin_t, cos_t;
    vo_sincos_deg(ori, &sin_t, &cos_t);
    const float exp_scale = -1.0f / ((float)(DW * DW) * 0.5f);
    const float hist_width = VO_SIFT_DESCR_SCL * q.scl;
    int radius = vo_round(hist_width * 1.4142135623730951f * (float)(DW + 1) * 0.5f);
#if defined(VO_DESC_DIAG) && VO_DESC_DIAG >= 2
    radius = 0;                                  // diagnostic build (timing only): no window tables
#endif
    if (radius > g.dmax) radius = g.dmax;
    if (radius > VO_SIFT_DESCR_RMAX) radius = VO_SIFT_DESCR_RMAX;
    radius = min(radius, dcap);                 // (never binds: dcap bounds every refined scale)
    cos_t = cos_t / hist_width;
    sin_t = sin_t / hist_width;
    {
        const float wsc = exp_scale / (hist_width * hist_width);
        // x 32 per factor: the product carries the fixed-point pre-scale 2^10 (exact, powers of two)
        for (int k2 = lane; k2 <= radius; k2 += 64) wtab[k2] = vo_sift_wt(wsc, k2) * 32.0f;
    }
    // Only ~half of the (2r+1)^2 window lies inside the rotated 4x4-cell square.  Each
    // window row i gets a conservative column interval [jlo, jhi] (a superset: +-2
    // columns of margin over the real-arithmetic bounds, clamped to the image
    // interior); rows are flattened with a prefix sum, and the exact float test below
    // still decides every sample, so the histogram is unchanged (fixed-point sums are
    // order-free) while the wave no longer idles through rejected samples.
    const int nrows = 2 * radius + 1;
    const float inv_ct = fabsf(cos_t) > 1e-9f ? 1.0f / cos_t : 0.0f, inv_st = fabsf(sin_t) > 1e-9f ? 1.0f / sin_t : 0.0f;
    for (int rr = lane; rr < nrows; rr += 64) {
        const int i = rr - radius, r = pyy + i;
        int jlo = -radius, jhi = radius;
        if (r <= 0 || r >= rows - 1) { jlo = 1; jhi = 0; }
        else {
            // |j*ct - i*st| < lim  and  |j*st + i*ct| < lim  (rbin = r_rot + 1.5 in (-1, DW)); lim is
            // 1e-3 bin widths wider than the test below, far above the float error of the test
            // (~1e-6) and of these bounds (< 1e-4 columns at r <= RMAX), so [floor(a), ceil(b)]
            // holds every accepted column
            const float fi = (float)i, lim = 0.5f * DW + 0.5f + 1e-3f, cap = (float)(radius + 2);
            if (fabsf(cos_t) > 1e-9f) {
                float a = (fi * sin_t - lim) * inv_ct, b = (fi * sin_t + lim) * inv_ct;
                if (a > b) { const float t2 = a; a = b; b = t2; }
                a = fminf(fmaxf(a, -cap), cap); b = fminf(fmaxf(b, -cap), cap);
                jlo = max(jlo, (int)floorf(a)); jhi = min(jhi, (int)ceilf(b));
            } else if (fabsf(fi * sin_t) >= lim) { jlo = 1; jhi = 0; }
            if (fabsf(sin_t) > 1e-9f) {
                float a = (-fi * cos_t - lim) * inv_st, b = (-fi * cos_t + lim) * inv_st;
                if (a > b) { const float t2 = a; a = b; b = t2; }
                a = fminf(fmaxf(a, -cap), cap); b = fminf(fmaxf(b, -cap), cap);
                jlo = max(jlo, (int)floorf(a)); jhi = min(jhi, (int)ceilf(b));
            } else if (fabsf(fi * cos_t) >= lim) { jlo = 1; jhi = 0; }
            jlo = max(jlo, 1 - px); jhi = min(jhi, cols - 2 - px);
            // trim the superset to the exact set: the float test in k_desc is monotone
            // in j on each side (rotations of a row are monotone float sequences),
            // so the accepted columns form one interval inside [jlo, jhi]
            const float fi_s = (float)i * sin_t, fi_c = (float)i * cos_t;
            auto inside = [&](int j) {
                const float cr = (float)j * cos_t - fi_s, rr2 = (float)j * sin_t + fi_c;
                const float rb = rr2 + (float)(DW / 2) - 0.5f, cb = cr + (float)(DW / 2) - 0.5f;
                return rb > -1.0f && rb < (float)DW && cb > -1.0f && cb < (float)DW;
            };
            while (jlo <= jhi && !inside(jlo)) ++jlo;
            while (jhi >= jlo && !inside(jhi)) --jhi;
        }
        // row length for now (prefixed below), first column in the high half
        rtab[rr] = (uint32_t)(jhi >= jlo ? jhi - jlo + 1 : 0) | ((uint32_t)(uint16_t)(int16_t)jlo << 16);
    }
    __syncthreads();
    {   // wave-parallel exclusive prefix over the rows (<= 2*RMAX+1): lane owns a chunk of rows
        constexpr int PER_MAX = (2 * VO_SIFT_DESCR_RMAX + 1 + 63) / 64;
        const int per = (nrows + 63) >> 6, r0w = lane * per;
        uint32_t ent[PER_MAX];
        int sum = 0;
#pragma unroll
        for (int q2 = 0; q2 < PER_MAX; ++q2) {
            ent[q2] = (q2 < per && r0w + q2 < nrows) ? rtab[r0w + q2] : 0u;
            sum += (int)(ent[q2] & 0xFFFFu);
        }
        const int inc = wave_incl_scan(sum);
        int acc = inc - sum;
#pragma unroll
        for (int q2 = 0; q2 < PER_MAX; ++q2)
            if (q2 < per && r0w + q2 < nrows) { rtab[r0w + q2] = (uint32_t)acc | (ent[q2] & 0xFFFF0000u); acc += (int)(ent[q2] & 0xFFFFu); }
        if (lane == 63) { rtab[nrows] = (uint32_t)inc; hdr[DT_NSAMP] = (uint32_t)inc; }
        if (lane < 8) rtab[nrows + 1 + lane] = 0xFFFFu;
        if (lane == 0) {
            hdr[DT_ORI] = __float_as_uint(ori); hdr[DT_PX] = (uint32_t)px; hdr[DT_PY] = (uint32_t)pyy;
            hdr[DT_RADIUS] = (uint32_t)radius; hdr[DT_COS] = __float_as_uint(cos_t); hdr[DT_SIN] = __float_as_uint(sin_t);
            hdr[DT_NROWS] = (uint32_t)nrows; hdr[DT_O] = (uint32_t)q.o; hdr[DT_LAYER] = (uint32_t)q.layer;
        }
    }
    __syncthreads();
}

// The descriptor of one keypoint by the whole wave (k_desc's body): window tables, sample loop, histogram fold, normalisation, u8 quantisation;
// writes dst[0..128) and *mdst.  hfx: DCOPIES * DCS words of LDS; dyn: dt_stride(dcap) words.
template <int DCOPIES>
__device__ __forceinline__ void desc_keypoint(const Pyramid* __restrict__ py, const float* __restrict__ arena, const KpInt q,
                                              int img, int dcap, uint32_t* hfx, uint32_t* dyn, uint8_t* dst, DescMeta* mdst)
{
    const int lane = threadIdx.x;
    const float bins_per_deg = (float)DN / 360.0f;
    static_assert((DCOPIES * DCS) % 4 == 0, "16-B zeroing");
    typedef uint32_t u4z_t __attribute__((ext_vector_type(4)));
    for (int b = 4 * lane; b < DCOPIES * DCS; b += 256) *reinterpret_cast<u4z_t*>(&hfx[b]) = u4z_t{0u, 0u, 0u, 0u};
    desc_tables(py, q, dcap, dyn, dyn + dt_rtab_off(), reinterpret_cast<float*>(dyn + dt_wtab_off(dcap)), lane);
    const uint32_t* const hdr = dyn;
    const uint32_t* const rtab = dyn + dt_rtab_off();
    const float* const wtab = reinterpret_cast<const float*>(dyn + dt_wtab_off(dcap));
    const int o = __builtin_amdgcn_readfirstlane((int)hdr[DT_O]), layer = __builtin_amdgcn_readfirstlane((int)hdr[DT_LAYER]);
    const OctGeom& g = py->oct[o];
    const int P = g.pitch;
    const float* gim = arena + g.g_off[layer] + img * py->istride;
    const float ori = __uint_as_float(hdr[DT_ORI]);
    const int px = (int)hdr[DT_PX], pyy = (int)hdr[DT_PY], radius = (int)hdr[DT_RADIUS];
    const float cos_t = __uint_as_float(hdr[DT_COS]), sin_t = __uint_as_float(hdr[DT_SIN]);
#if defined(VO_DESC_DIAG) && VO_DESC_DIAG >= 1
    const int nsamp = 0;                         // diagnostic build (timing only): no sample loop
#else
    const int nsamp = (int)hdr[DT_NSAMP];
#endif
    uint32_t* hc = hfx + (lane & (DCOPIES - 1)) * DCS;
    // one sample: weights, bins, fixed-point LDS atomics
    auto accum = [&](float c_rot, float r_rot, float w, float dx, float dy) {
        float rbin = r_rot + (float)(DW / 2) - 0.5f;
        float cbin = c_rot + (float)(DW / 2) - 0.5f;
        float ang = vo_atan2_deg(dy, dx);
        float mag = vo_grad_mag(dx, dy) * w;         // = (|grad| w_ij) 2^10 exactly (w from the x 32 table)
        float obin = (ang - ori) * bins_per_deg;
        // floors kept in float ((float)(int)floorf(v) == floorf(v) here); the cell index is an
        // exact small-integer float expression, one conversion; obin in [-8, 8] so the circular
        // wrap of o0 is a mask (DN = 8)
        const float fr0 = floorf(rbin), fc0 = floorf(cbin), fo0 = floorf(obin);
        rbin -= fr0; cbin -= fc0; obin -= fo0;
        const int o0 = (int)fo0 & (DN - 1);
        // histogram word of cell (fr0 + 1, fc0 + 1): ((fr0 + 1) (DW + 2) + fc0 + 1) DBS as two
        // exact small-integer fmas (< 2^24), one conversion
        const float cell_w = fmaf(fr0, (float)((DW + 2) * DBS), fmaf(fc0, (float)DBS, (float)((DW + 3) * DBS)));
        float v_r1 = mag * rbin, v_r0 = mag - v_r1;
        float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
        float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
        float v_rco111 = v_rc11 * obin, v_rco110 = v_rc11 - v_rco111;
        float v_rco101 = v_rc10 * obin, v_rco100 = v_rc10 - v_rco101;
        float v_rco011 = v_rc01 * obin, v_rco010 = v_rc01 - v_rco011;
        float v_rco001 = v_rc00 * obin, v_rco000 = v_rc00 - v_rco001;
        uint32_t* h = hc + (int)cell_w + o0;
        atomicAdd(h, desc_fxq(v_rco000));
        atomicAdd(h + 1, desc_fxq(v_rco001));
        atomicAdd(h + DBS, desc_fxq(v_rco010));
        atomicAdd(h + DBS + 1, desc_fxq(v_rco011));
        atomicAdd(h + (DW + 2) * DBS, desc_fxq(v_rco100));
        atomicAdd(h + (DW + 2) * DBS + 1, desc_fxq(v_rco101));
        atomicAdd(h + (DW + 3) * DBS, desc_fxq(v_rco110));
        atomicAdd(h + (DW + 3) * DBS + 1, desc_fxq(v_rco111));
    };
    // the gradient neighbours of a listed sample (every listed sample is interior): x+1, x-1 as
    // one 12-B load (through a 3-float type declared with the 4-B alignment the address has),
    // y-1, y+1
    // buffer loads with one 32-bit lane offset: the resource starts at the sample's row y-1
    // column x-1 for offset 0 (gim - P - 1), so row y-1 is +4 B, row y (x-1..x+1) +4P B and
    // row y+1 +8P + 4 B -- no 64-bit address arithmetic per sample; the row offset is a
    // 24-bit multiply (|i| <= RMAX, P < 2^23)
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void*)(gim - P - 1), 0, 0x7FFFFFF0, 0x00020000);
    const int c_off = pyy * P + px;                  // wave-uniform
    auto grad_loads = [&](int i, int j, float* g4) {
        const int vo = 4 * (c_off + __mul24(i, P) + j);
        typedef int i3_t __attribute__((ext_vector_type(3)));
        const i3_t h = __builtin_amdgcn_raw_buffer_load_b96(grs, vo, 4 * P, 0);
        g4[0] = __int_as_float(h.z); g4[1] = __int_as_float(h.x);
        g4[2] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(grs, vo + 4, 0, 0));
        g4[3] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(grs, vo + 4, 8 * P, 0));
    };
    {   // Block lookup: the 64 samples bs .. bs+63 of a block start in row rb (wave-uniform) and
        // span a few rows; every lane reads the same K+2 table entries (LDS broadcast, one round
        // trip) and selects its row by comparing its sample index with the row starts -- no
        // per-lane walk, no dependent LDS chain.  Rows past rb+K (short rows at a rotated
        // window's corners, rows of zero length above the image) take another round.
        // The gradient loads of the next U blocks are issued before the current U blocks are
        // accumulated (two slot sets, a pair of batches per loop iteration; the loads of a
        // batch past the window are clamped to its last sample, so every iteration issues
        // the same loads and the wait counts stay exact).
        constexpr int U = VO_DESC_U, K = 4;
        int rb = 0;                                      // wave-uniform row of the next block's first sample
        auto locate = [&](int bs, int& i_o, int& j_o) {
            const int sc = min(bs + lane, nsamp - 1), last = min(bs + 63, nsamp - 1);
            uint32_t sel = rtab[rb];
            int row = rb;
            for (;;) {
                const uint32_t* tb = rtab + rb;
                uint32_t e[K + 2];
#pragma unroll
                for (int k = 1; k <= K + 1; ++k) e[k] = tb[k];
#pragma unroll
                for (int k = 1; k <= K; ++k) {
                    const bool c = (int)(e[k] & 0xFFFFu) <= sc;
                    sel = c ? e[k] : sel;
                    row += c ? 1 : 0;
                }
                if ((int)(e[K + 1] & 0xFFFFu) > last) break;   // uniform: every lane's row found
                rb += K;
            }
            i_o = row - radius;
            j_o = ((int)sel >> 16) + (sc - (int)(sel & 0xFFFFu));
            rb = __builtin_amdgcn_readlane(row, 63);
        };
        struct Slot { float g[4]; int i, j; };
        auto issue = [&](int sb, Slot (&S)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) locate(sb + 64 * u, S[u].i, S[u].j);
#pragma unroll
            for (int u = 0; u < U; ++u) grad_loads(S[u].i, S[u].j, S[u].g);
        };
        auto consume = [&](int sb, const Slot (&S)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (sb + 64 * u + lane < nsamp) {
                    const float fi = (float)S[u].i, fj = (float)S[u].j;
                    accum(fj * cos_t - fi * sin_t, fj * sin_t + fi * cos_t, wtab[abs(S[u].i)] * wtab[abs(S[u].j)],
                          S[u].g[0] - S[u].g[1], S[u].g[2] - S[u].g[3]);
                }
            }
        };
        if (nsamp > 0) {
            Slot A[U], B[U];
            int sb = 0;
            issue(0, A);
            for (;;) {
                issue(sb + 64 * U, B);
                consume(sb, A);
                sb += 64 * U;
                if (sb >= nsamp) break;
                issue(sb + 64 * U, A);
                consume(sb, B);
                sb += 64 * U;
                if (sb >= nsamp) break;
            }
        }
    }
    __syncthreads();
    // fold the circular orientation bins and convert; lane holds dst[lane], dst[lane+64]
    float dv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int kk = lane + 64 * h;
        const int cell = kk / DN, ob = kk - cell * DN;
        const int ci = cell / DW, cj = cell - ci * DW;
        const int base = ((ci + 1) * (DW + 2) + (cj + 1)) * DBS;
        uint32_t v = 0;
#pragma unroll
        for (int cp = 0; cp < DCOPIES; ++cp) {
            v += hfx[cp * DCS + base + ob];
            if (ob == 0) v += hfx[cp * DCS + base + DN];
        }
        dv[h] = vo_desc_fx_to_float(v);
    }
    const float nrm0 = wave_tree_sum(dv[0] * dv[0] + dv[1] * dv[1]);
    const float thr = sqrtf(nrm0) * VO_SIFT_DESCR_MAG_THR;
    dv[0] = dv[0] < thr ? dv[0] : thr;
    dv[1] = dv[1] < thr ? dv[1] : thr;
    const float nrm = sqrtf(wave_tree_sum(dv[0] * dv[0] + dv[1] * dv[1]));
    const float scale = VO_SIFT_DESCR_INT_FCTR / (nrm > VO_FLT_EPSILON ? nrm : VO_FLT_EPSILON);
    int qv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        float v = rintf(dv[h] * scale);
        qv[h] = v < 0.0f ? 0 : v > 255.0f ? 255 : (int)v;
    }
    dst[lane] = (uint8_t)qv[0];
    dst[lane + 64] = (uint8_t)qv[1];
    const int sum = wave_tree_sum(qv[0] + qv[1]), sq = wave_tree_sum(qv[0] * qv[0] + qv[1] * qv[1]);
    if (lane == 0) {
        DescMeta m;
        m.sum = sum;
        m.inv_norm = sq > 0 ? 1.0f / sqrtf((float)sq) : 0.0f;
        *mdst = m;
    }
    __syncthreads();
}

template <int DCOPIES>
__global__ __launch_bounds__(64, VO_DESC_WAVES) void k_desc(const Pyramid* __restrict__ py, const float* __restrict__ arena,
                                             const KpInt* __restrict__ kpi, const int* __restrict__ n_kp,
                                             uint8_t* __restrict__ desc,
                                             DescMeta* __restrict__ meta, int kp_cap, int n_img)
{
    static_assert(DCS >= DHIST, "copy stride holds a histogram");
    __shared__ __attribute__((aligned(16))) uint32_t hfx[DCOPIES * DCS];
    // Dynamic LDS, sized by the launch for this pyramid: the keypoint's window tables (desc_tables,
    // dt_stride(dcap) words: header, row table, separable window weights wtab[0 .. radius] --
    // vo_spec.h vo_sift_wt: w(i, j) = wtab[|i|] * wtab[|j|]) and the image prefix (n_img + 1).
    // (The tables as a separate full-occupancy launch, k_desc_prep, measured slower: 0.35 ms for
    // that launch against 0.23 ms they cost inside k_desc, profiles/r05_g_*.)  dcap bounds every keypoint's radius (the largest refined scale the parameters
    // allow, capped at VO_SIFT_DESCR_RMAX): ~0.6 KB at the default parameters, so the descriptor's
    // one-wave workgroups leave LDS for the scale-space waves that share their CUs.
    extern __shared__ uint32_t dyn[];
    const int dcap = py->dcap, ts = dt_stride(dcap);
    int* const fpre = reinterpret_cast<int*>(dyn + ts);
    const long total = flat_setup(n_kp, kp_cap, n_img, fpre);
    for (long t = blockIdx.x; t < total; t += gridDim.x) {
        int img, k;
        flat_find_wave(fpre, n_img, t, img, k);
        const KpInt q = kpi[(size_t)img * kp_cap + k];
        desc_keypoint<DCOPIES>(py, arena, q, img, dcap, hfx, dyn, desc + ((size_t)img * kp_cap + k) * VO_DESC_LEN,
                               meta + (size_t)img * kp_cap + k);
    }
}

// ---------------------------------------------------------------------------
// host enqueue
// ---------------------------------------------------------------------------
static Kern make_kern(const Pyramid& py, int level)
{
    Kern k;
    memset(&k, 0, sizeof(k));
    k.r = py.krad[level];
    for (int j = 0; j <= k.r; ++j) k.k[j] = py.kern[level][j];
    return k;
}

// hipFuncSetAttribute is a per-device setting: raise a kernel's dynamic-LDS limit to the CU's
// 160 KB once per (kernel, device), so a second context on another device gets it too
void raise_lds_limit(const void* fn)
{
    static std::mutex mu;
    static std::vector<std::pair<const void*, int>> done;
    int dev = 0;
    hipGetDevice(&dev);
    std::lock_guard<std::mutex> lock(mu);
    for (const auto& d : done)
        if (d.first == fn && d.second == dev) return;
    hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    done.push_back({fn, dev});
}

// -> true when the streaming kernel ran (it stores K.nb, the next octave's base, if set)
template <int RAD, int MODE>
static bool launch_blur_r(dim3 grid, hipStream_t s, const float* src, size_t plane, size_t dplane, int pitch, int R, int C,
                          float* g, float* d, const Kern& K, const ImageSrc& isrc, int in_rows, int in_cols, const char* name)
{
    const size_t lds = sizeof(float) * ft_lds_floats(K.r);
    if constexpr (MODE == 0 && RAD > 0) {
        // band height: a multiple of P, at most 128 rows, lowered on small octaves until the
        // launch has ~2048 waves (8 per CU; 1024 measured ~1.5 % slower) -- small planes are
        // latency-bound.  Level blurs of planes at most 1400 columns wide use 2 columns per
        // lane (128-column strips, half the ring registers): more waves and fewer idle lanes
        // at the narrow octaves, where the kernel is latency-bound rather than HBM-bound.
#ifndef VO_CPL2_MAXC
#define VO_CPL2_MAXC 1400
#endif
#ifndef VO_BLUR_MAX_TH
#define VO_BLUR_MAX_TH 128
#endif
#ifndef VO_BLUR_WAVES
#define VO_BLUR_WAVES 2048
#endif
        constexpr int kMaxTH = VO_BLUR_MAX_TH, kWaveTarget = VO_BLUR_WAVES, kCpl2MaxC = VO_CPL2_MAXC;
        const bool base = name[7] == 'b';
        // (2 columns per lane for the octave-0 levels of radius >= 13 / 10 / 8 too -- fewer registers,
        // so more of them fit beside the tracking matches of the full path: configs[1] -0.8 / -0.9 /
        // -4.3 %, full path within noise, profiles/r06_v_ab_fullpath_cpl_refine.txt)
        const int cpl = (!base && C <= kCpl2MaxC) ? 2 : 4;
        const int n_strips = (C + 64 * cpl - 1) / (64 * cpl);
        const long rows_total = (long)R * n_strips * grid.z;
        // (the staged octave-0 base stages at most kBaseMaxTH-row bands: its LDS is sized for them)
        int TH = (int)std::min<long>(base ? std::min(kMaxTH, kBaseMaxTH) : kMaxTH, rows_total / kWaveTarget);
        TH = std::max(BS_P, TH / BS_P * BS_P);
        if (R >= TH && R > RAD + BS_P + 2) {             // (one reflection fold per band edge)
            const int n_bands = (R + TH - 1) / TH;
#define VO_BS_GO(T, CP)                                                                                        \
    do {                                                                                                       \
        const int ns_ = (C + bs_sw(RAD, CP, T) - 1) / bs_sw(RAD, CP, T);                                       \
        VO_LAUNCH_NAMED(name, (k_blur_stream<RAD, T, CP>), dim3(ns_ * n_bands * (int)grid.z), dim3(64), 0, s, src, plane, \
                        dplane, pitch, R, C, g, K, ns_, n_bands, TH, isrc, in_rows, in_cols);                     \
    } while (0)
            if (base && src == nullptr) VO_BS_GO(5, 4);      // "k_blur_base" from the u8 image (x2 upsample fused)
            else if (base) VO_BS_GO(1, 4);
            else if (cpl == 2) VO_BS_GO(0, 2);
            else VO_BS_GO(0, 4);
#undef VO_BS_GO
            return true;
        }
    }
    // generic tiled form: kernel radii without a streaming instantiation, planes shorter than
    // one band (tiny images; GPU edge tests), and the non-upsampled / split octave-0 base
    if (lds > 64 * 1024) raise_lds_limit((const void*)k_blur_fused<RAD, MODE>);
    VO_LAUNCH_NAMED(MODE == 0 ? "k_blur_fused" : "k_blur_base", (k_blur_fused<RAD, MODE>), grid, dim3(256), lds, s, src,
                    plane, dplane, pitch, R, C, g, d, K, isrc, in_rows, in_cols);
    return false;
}

template <int MODE>
static bool launch_blur(dim3 grid, hipStream_t s, const float* src, size_t plane, size_t dplane, int pitch, int R, int C, float* g,
                        float* d, const Kern& K, const ImageSrc& isrc, int in_rows, int in_cols,
                        const char* name = MODE == 0 ? "k_blur_fused" : "k_blur_base")
{
    switch (K.r) {
    case 5: return launch_blur_r<5, MODE>(grid, s, src, plane, dplane, pitch, R, C, g, d, K, isrc, in_rows, in_cols, name);
    case 6: return launch_blur_r<6, MODE>(grid, s, src, plane, dplane, pitch, R, C, g, d, K, isrc, in_rows, in_cols, name);
    case 8: return launch_blur_r<8, MODE>(grid, s, src, plane, dplane, pitch, R, C, g, d, K, isrc, in_rows, in_cols, name);
    case 10: return launch_blur_r<10, MODE>(grid, s, src, plane, dplane, pitch, R, C, g, d, K, isrc, in_rows, in_cols, name);
    case 13: return launch_blur_r<13, MODE>(grid, s, src, plane, dplane, pitch, R, C, g, d, K, isrc, in_rows, in_cols, name);
    default: return launch_blur_r<0, MODE>(grid, s, src, plane, dplane, pitch, R, C, g, d, K, isrc, in_rows, in_cols, name);
    }
}

static float ext_threshold(const Pyramid& py, const vo_sift_params& p)
{
    return (float)floor(0.5 * p.contrast_threshold / py.L * 255.0);
}

// octaves [0, n) whose levels 1..L+2, extremum test and next base k_octave computes in one pass
// (octave.hip): a prefix of the octaves, below the LDS-sized ones.  Experimental: bit-exact but
// measured 2.4x slower than the per-level kernels on MI355X, so it is compiled only
// into the test build libvo_exp.so (VO_EXPERIMENTAL, selected there by vo_exp_set); the product
// library always takes the per-level kernels.
static int fused_octaves(const Pyramid& py)
{
#if VO_EXPERIMENTAL
    if (!g_exp_fused_octave) return 0;
    int n = 0;
    while (n < py.n_oct && octave_fused_ok(py, n)) ++n;
    return n;
#else
    (void)py;
    return 0;
#endif
}

// First octave from which every remaining octave fits the one-launch LDS path (k_small_pyr),
// its reflect-table length and dynamic LDS size.
// LDS holds 3 planes of the largest octave (cap floats), the largest next-octave base (bcap
// floats; both rounded up to a multiple of 4) and the reflect tables -- sized to the octaves at
// hand, not to VO_SMALL_PX, so a launch needs no more of a CU's LDS than its planes.
struct SmallPlan { int o_small, rtab, cap, bcap; size_t lds; };
static SmallPlan small_plan(const Pyramid& py)
{
    SmallPlan sp{py.n_oct, 0, 0, 0, 0};
    int maxr = 0;
    for (int i = 1; i < py.L + 3; ++i) maxr = std::max(maxr, py.krad[i]);
    for (int o = py.n_oct - 1; o >= 1; --o) {
        int rt = 0, ct = 0, cap = 0, bcap = 0;
        bool fits = true;
        for (int q = o; q < py.n_oct; ++q) {
            fits = fits && py.oct[q].rows * py.oct[q].cols <= VO_SMALL_PX;
            cap = std::max(cap, py.oct[q].rows * py.oct[q].cols);
            if (q > o) bcap = std::max(bcap, py.oct[q].rows * py.oct[q].cols);
            rt = std::max(rt, py.oct[q].rows + 2 * maxr);
            ct = std::max(ct, py.oct[q].cols + 2 * maxr);
        }
        cap = (cap + 3) & ~3;
        bcap = (bcap + 3) & ~3;
        const size_t lds = sizeof(float) * (3 * (size_t)cap + bcap) + sizeof(int) * (rt + ct);
        if (!fits || lds > 160 * 1024) break;
        sp = SmallPlan{o, rt, cap, bcap, lds};
    }
    return sp;
}

// The LDS-sized octaves (one k_small_pyr launch).  sift_enqueue_pyramid_tail enqueues it on the
// scale-space stream after the last level blur (its workgroups need ~120 KB of one CU's LDS; by
// then octave 0's extremum test has moved to the feature stream, so the previous batch's
// descriptor waves no longer hold every CU's LDS when it arrives -- DESIGN.md §9c).
int sift_small_octave(const Pyramid& py) { return small_plan(py).o_small; }

void sift_enqueue_small(const Pyramid& py, SiftBuffers& b, int n_img, hipStream_t s, const Pyramid* d_py)
{
    const SmallPlan sp = small_plan(py);
    if (sp.o_small >= py.n_oct) return;

    raise_lds_limit((const void*)k_small_pyr);
    VO_LAUNCH_NAMED("k_blur_small", k_small_pyr, dim3(n_img), dim3(VO_SMALL_T), sp.lds, s, d_py, b.arena, sp.o_small,
                    sp.rtab, sp.cap, sp.bcap);
}

void sift_enqueue_pyramid(const Pyramid& py, SiftBuffers& b, const ImageSrc& src, int n_img, const vo_sift_params& p,
                          hipStream_t s, const Pyramid* d_py, hipEvent_t ev_o0)
{
    const int L = py.L;
    float* A = b.arena;
    const SmallPlan sp = small_plan(py);
    const int o_small = sp.o_small;
    const int n_fused = std::min(fused_octaves(py), o_small);
    if (n_fused > 0) {
        // k_octave ORs its extremum words into the mask (strips share the words at their
        // boundaries): clear the fused octaves' words of every image first
        const size_t w0 = (size_t)py.wbase[0], w1 = (size_t)py.wbase[n_fused * L];
        hipMemset2DAsync(b.mask + w0, sizeof(unsigned long long) * py.n_words, 0, sizeof(unsigned long long) * (w1 - w0),
                         n_img, s);
    }
#if VO_EXPERIMENTAL
    const float thr = ext_threshold(py, p);
#endif
    bool base_done = false;                            // octave o's base already stored
    for (int o = 0; o < py.n_oct; ++o) {
        const OctGeom& g = py.oct[o];
        const int R = g.rows, C = g.cols;
        if (o == o_small) break;                       // octaves o_small.. : sift_enqueue_small
        dim3 gf((C + FT_W - 1) / FT_W, (R + FT_H - 1) / FT_H, n_img);
        if (o == 0) {
            Kern K0 = make_kern(py, 0);
            const int rows = p.upsample ? R / 2 : R, cols = p.upsample ? C / 2 : C;
            const int r0 = K0.r;
            const bool stream_r = r0 == 5 || r0 == 6 || r0 == 8 || r0 == 10 || r0 == 13;
            if (p.upsample && stream_r && R >= 64) {
                // level-0 blur straight from the u8 image, x2 upsample formed while staging rows
                launch_blur<0>(gf, s, nullptr, 0, py.istride, g.pitch, R, C, A + g.g_off[0], nullptr, K0, src, rows, cols,
                               "k_blur_base");
            } else {
                // u8 (x2 upsampled) -> float source plane in the scratch buffer, then the level-0 blur
                const dim3 qg((g.pitch / 4 + 255) / 256, R, n_img);
                if (p.upsample)
                    VO_LAUNCH(k_base_src<true>, qg, dim3(256), 0, s, src, rows, cols, b.tmp, g.plane, g.pitch, R, C, n_img);
                else
                    VO_LAUNCH(k_base_src<false>, qg, dim3(256), 0, s, src, rows, cols, b.tmp, g.plane, g.pitch, R, C, n_img);
                launch_blur<0>(gf, s, b.tmp, g.plane, py.istride, g.pitch, R, C, A + g.g_off[0], nullptr, K0, src, 0, 0,
                               "k_blur_base");
            }
        } else if (o - 1 >= n_fused && !base_done) {  // (a fused octave / level-L blur wrote it)
            const OctGeom& pg = py.oct[o - 1];
            VO_LAUNCH(k_down, dim3((C + 255) / 256, R, n_img), dim3(256), 0, s, A + pg.g_off[L], py.istride, pg.pitch,
                      A + g.g_off[0], py.istride, g.pitch, C);
        }
        base_done = false;
#if VO_EXPERIMENTAL
        if (o < n_fused) {
            octave_fused_launch(py, d_py, b, o, n_img, thr, s);
            continue;
        }
#endif
        for (int i = 1; i < L + 3; ++i) {
            Kern K = make_kern(py, i);
            // level L stores the next octave's base from its store path (no k_down pass: that
            // re-read the even rows of G_L whole, 1.5x its algorithmic bytes); k_small_pyr
            // decimates its own first base
            const bool emit = i == L && o + 1 < o_small;
            if (emit) {
                const OctGeom& ng = py.oct[o + 1];
                K.nb = A + ng.g_off[0];
                K.nb_pitch = ng.pitch; K.nb_rows = ng.rows; K.nb_cols = ng.cols;
            }
            const bool streamed = launch_blur<0>(gf, s, A + g.g_off[i - 1], py.istride, py.istride, g.pitch, R, C,
                                                 A + g.g_off[i], nullptr, K, src, 0, 0);
            if (emit) base_done = streamed;
        }
        if (o == 0 && ev_o0) hipEventRecord(ev_o0, s);           // octave 0 complete: its extremum test may start
    }
}

// grid of the wave-per-keypoint kernels (grid-stride over the flat keypoint space):
// 32768 one-wave workgroups (~7 keypoints each at 64 frames x ~1.8k): shorter tail than
// 8192 (k_desc 2.25 -> 2.05 ms, k_orient 0.77 -> 0.67 ms isolated) and workgroups turn over
// often enough for the scale-space stream's blurs to get slots while they run
#ifndef VO_FEATURE_GRID
#define VO_FEATURE_GRID 32768
#endif
constexpr int kFeatureGrid = VO_FEATURE_GRID;

// The extremum test of octaves [o_begin, o_end).  vo_api.hip enqueues it in two parts on the
// feature stream: octave 0 as soon as the scale-space stream records ev_o0 (beside the level blurs
// of octaves 1..), and octaves 1.. after the scale space's tail (VO_EXT_SPLIT).
void sift_enqueue_extrema(const Pyramid& py, SiftBuffers& b, int n_img, const vo_sift_params& p, hipStream_t s,
                          const Pyramid* d_py, int o_begin, int o_end)
{
    const int L = py.L;
    float* A = b.arena;
    const float thr = ext_threshold(py, p);
    const int u_first = py.ebase[std::max(o_begin, fused_octaves(py))], u_last = py.ebase[o_end];
    if (u_last > u_first) {
        const dim3 ge((u_last - u_first) * n_img);
#if VO_EXT_INNER
#define VO_EXT_K(LL) VO_LAUNCH(k_ext_inner<LL>, ge, dim3(64), 0, s, d_py, A, b.mask, thr, n_img, u_first, u_last)
#else
#define VO_EXT_K(LL) VO_LAUNCH(k_ext_stream<LL>, ge, dim3(64), 0, s, d_py, A, b.mask, thr, n_img, u_first, u_last)
#endif
        switch (L) {
        case 1: VO_EXT_K(1); break;
        case 2: VO_EXT_K(2); break;
        case 3: VO_EXT_K(3); break;
        case 4: VO_EXT_K(4); break;
        default: VO_EXT_K(5); break;
        }
#undef VO_EXT_K
    }
}

void sift_enqueue_pyramid_tail(const Pyramid& py, SiftBuffers& b, int n_img, const vo_sift_params& p, hipStream_t s,
                               const Pyramid* d_py, int ext_o_begin)
{
    sift_enqueue_small(py, b, n_img, s, d_py);
    sift_enqueue_extrema(py, b, n_img, p, s, d_py, ext_o_begin, py.n_oct);
}

// k_orient sums each bin per histogram column in u32 fixed point (VO_ORIENT_COLS columns; one
// weight < 361 * 2^10, |dI| <= 255), and a column receives 1/VO_ORIENT_COLS of the window's samples:
// the window fits while (2r + 1)^2 <= VO_ORIENT_COLS * floor(2^32 / (361 * 2^10)).  r bounds the
// orientation radius round(4.5 scl) for any refined scale (scl < sigma 2^((L + 0.5) / L), k_refine):
// sigma up to ~17 at L = 1, ~21 at L = 3.
bool sift_params_supported(const vo_sift_params& p)
{
    if (!(p.sigma > 0.0f) || !std::isfinite(p.sigma) || p.n_octave_layers < 1) return false;
    const double scl = p.sigma * std::exp2((p.n_octave_layers + 0.5) / p.n_octave_layers);
    const double r = std::ceil(VO_SIFT_ORI_RADIUS * scl) + 1;
    const double per_column = std::floor(4294967296.0 / (361.0 * VO_DESC_FX_SCALE));
    return (2 * r + 1) * (2 * r + 1) <= VO_ORIENT_COLS * per_column;
}

// Largest descriptor window radius any keypoint can have: k_refine accepts layer <= L with
// |xi| < 0.5, so the octave-relative scale stays below sigma 2^((L + 0.5) / L); the radius formula
// of k_desc on that bound, + 2 for float rounding, capped at VO_SIFT_DESCR_RMAX (sizes k_desc's LDS).
static int desc_radius_cap(const Pyramid& py, const vo_sift_params& p)
{
    const double scl = p.sigma * std::exp2((py.L + 0.5) / py.L);
    const double r = VO_SIFT_DESCR_SCL * scl * 1.4142135623730951 * (VO_SIFT_DESCR_W + 1) * 0.5;
    return (int)std::min<double>(VO_SIFT_DESCR_RMAX, std::ceil(r) + 2);
}

void sift_enqueue_features(const Pyramid& py, SiftBuffers& b, int n_img, const vo_sift_params& p, hipStream_t s,
                           const Pyramid* d_py)
{
    float* A = b.arena;
    const dim3 gs(py.n_seg > 0 ? py.n_seg : 1, n_img);
    VO_LAUNCH(k_seg_count, gs, dim3(256), 0, s, b.mask, b.woff, py.n_words, py.n_seg);
    VO_LAUNCH(k_seg_scan, dim3(n_img), dim3(1024), 0, s, b.woff, b.n_cand, b.n_acc, py.n_seg);
    VO_LAUNCH(k_seg_emit, gs, dim3(256), 0, s, d_py, b.mask, (const uint32_t*)b.woff, b.cand, b.cand_cap);
    VO_LAUNCH(k_refine, dim3(VO_REFINE_BLOCKS), dim3(256), 0, s, d_py, A, b.cand, b.n_cand, b.cout, b.acc, b.n_acc, b.koff, b.cand_cap, n_img,
              p.contrast_threshold, p.edge_threshold, p.sigma);
    const size_t fpre_bytes = sizeof(int) * (size_t)(n_img + 1);
    const int* n_walk = VO_ACC_LIST ? b.n_acc : b.n_cand;    // the accepted list, or every candidate
    const size_t dt_bytes = sizeof(uint32_t) * (size_t)dt_stride(py.dcap);
    VO_LAUNCH_NAMED("k_orient", (k_orient<36>), dim3(kFeatureGrid), dim3(64), fpre_bytes, s, d_py, A, n_walk, b.acc,
                    b.cout, b.koff, b.cand_cap, n_img);
    VO_LAUNCH(k_scan_cands, dim3(n_img), dim3(1024), 0, s, b.cout, b.n_cand, b.koff, b.n_kp, b.cand_cap);
    VO_LAUNCH(k_expand, dim3(256), dim3(256), 0, s, b.cout, n_walk, b.acc, b.koff, b.kp, b.kpi, b.cand_cap, b.kp_cap,
              n_img, p.upsample);
    // 4 histogram copies: 2 -> +4 %, 8 -> +33 % k_desc time (MI355X)
    // (capping k_desc's residency per CU with 8 / 16 / 28 KB of extra LDS per workgroup, to leave
    // the level blurs beside it more waves: 8886 / 8016 / 6877 against 10186 stereo frames/s --
    // the blurs gain 3 ms in situ, k_desc loses 3-11 ms, profiles/r06_t_ab_desc_lds_pad.txt)
    VO_LAUNCH_NAMED("k_desc", (k_desc<VO_DESC_COPIES>), dim3(kFeatureGrid), dim3(64), dt_bytes + fpre_bytes, s, d_py, A,
                    b.kpi, b.n_kp, b.desc, b.meta, b.kp_cap, n_img);
}

void sift_enqueue(const Pyramid& py, SiftBuffers& b, const ImageSrc& src, int n_img, const vo_sift_params& p,
                  hipStream_t s, const Pyramid* d_py)
{
    sift_enqueue_pyramid(py, b, src, n_img, p, s, d_py);
    sift_enqueue_pyramid_tail(py, b, n_img, p, s, d_py, 0);
    sift_enqueue_features(py, b, n_img, p, s, d_py);
}

}  // namespace vo
