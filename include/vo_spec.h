/*
 * vo_spec.h — deterministic arithmetic primitives shared by the HIP product
 * path and the CPU oracle.
 *
 * Why this file exists
 * --------------------
 * The reference (VO.m) calls closed MathWorks toolbox functions whose
 * internals are not available.  Our parity bar is therefore
 * "GPU result == CPU restatement, bit for bit" for every integer/index
 * output (keypoint sets, match index pairs, inlier masks).  That is only
 * possible if both sides evaluate *the same* sequence of IEEE-754 basic
 * operations.  Basic ops (+ - * / sqrt, fmaf, rint, floor, int<->float
 * casts) are correctly rounded on both gfx950 (hipcc default float mode) and
 * x86-64 SSE; libm transcendentals are NOT identical across the two.  So every
 * transcendental the path needs (exp, atan2, sin/cos, log) is defined here as
 * a fixed polynomial/range-reduction recipe built only from basic ops, and
 * both sides are compiled with -ffp-contract=off (explicit fmaf where wanted).
 *
 * These are *spec primitives*: they define what the path computes.  The KAT
 * tests (tests/test_spec_math.py) pin each one against libm/numpy to a stated
 * tolerance.
 *
 * Usable from C (gcc, oracle) and HIP (hipcc, product).
 */
#ifndef VO_SPEC_H
#define VO_SPEC_H

#include <stdint.h>

#if defined(__HIPCC__)
#define VO_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define VO_HD static inline
#endif

/* ------------------------------------------------------------------------ */
/* Bit casts                                                                 */
/* ------------------------------------------------------------------------ */
VO_HD float vo_u32_as_f32(uint32_t u) { union { uint32_t u; float f; } c; c.u = u; return c.f; }
VO_HD uint32_t vo_f32_as_u32(float f) { union { uint32_t u; float f; } c; c.f = f; return c.u; }
VO_HD double vo_u64_as_f64(uint64_t u) { union { uint64_t u; double f; } c; c.u = u; return c.f; }
VO_HD uint64_t vo_f64_as_u64(double f) { union { uint64_t u; double f; } c; c.f = f; return c.u; }

/* round-half-even to int (cvRound semantics for |x| < 2^31) */
VO_HD int vo_round(float x) { return (int)rintf(x); }
VO_HD int vo_floor(float x) { return (int)floorf(x); }

/* ------------------------------------------------------------------------ */
/* exp (float).  Range reduction x = k*ln2 + r, |r| <= ln2/2, degree-7 Taylor */
/* in Horner form with explicit fmaf.  Returns 0 for x < -87.  Max rel error */
/* vs libm ~2 ulp (pinned in tests).                                         */
/* ------------------------------------------------------------------------ */
VO_HD float vo_expf(float x)
{
    if (x < -87.0f) return 0.0f;
    if (x > 88.0f) x = 88.0f;
    float kf = rintf(x * 1.44269504088896341f);
    float r = x - kf * 0.693145751953125f;          /* ln2 hi (exact product for |k|<=128) */
    r = r - kf * 1.42860682030941723212e-6f;        /* ln2 lo */
    float p = 1.98412698e-4f;                       /* 1/5040 */
    p = fmaf(p, r, 1.38888889e-3f);                 /* 1/720 */
    p = fmaf(p, r, 8.33333333e-3f);                 /* 1/120 */
    p = fmaf(p, r, 4.16666667e-2f);                 /* 1/24 */
    p = fmaf(p, r, 1.66666667e-1f);                 /* 1/6 */
    p = fmaf(p, r, 0.5f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    int k = (int)kf;
    /* p in [0.7, 1.42]; scale by 2^k in two steps to stay normal */
    int k1 = k / 2, k2 = k - k1;
    float s1 = vo_u32_as_f32((uint32_t)(k1 + 127) << 23);
    float s2 = vo_u32_as_f32((uint32_t)(k2 + 127) << 23);
    return (p * s1) * s2;
}

/* vo_expf on [-87, 0], for callers whose argument is a bounded non-positive quadratic form (the
 * SIFT window weights): the clamps never fire there, and p * 2^k is formed by one ldexp instead
 * of two scale factors.  Both forms are the one correctly rounded value of p * 2^k (the first
 * scale product is exact), so the result equals vo_expf(x) bit for bit on the whole domain --
 * checked for every float in [-87, 0] by oracle_spec_check_expf_nonpos (tests/test_spec_math.py). */
VO_HD float vo_expf_nonpos(float x)
{
    float kf = rintf(x * 1.44269504088896341f);
    float r = x - kf * 0.693145751953125f;
    r = r - kf * 1.42860682030941723212e-6f;
    float p = 1.98412698e-4f;
    p = fmaf(p, r, 1.38888889e-3f);
    p = fmaf(p, r, 8.33333333e-3f);
    p = fmaf(p, r, 4.16666667e-2f);
    p = fmaf(p, r, 1.66666667e-1f);
    p = fmaf(p, r, 0.5f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    return ldexpf(p, (int)kf);
}

/* ------------------------------------------------------------------------ */
/* Reciprocal of d in [2^-100, 2^100] by an integer seed and three Newton    */
/* steps r <- r + r (1 - d r), each two fmaf: basic ops only, so GPU == CPU  */
/* bit for bit.  The seed 0x7EF311C3 - bits(d) is within 12.5 % of 1/d; the  */
/* steps square the relative error (1.6e-2, 2.4e-4, 6e-8), so the result is  */
/* within ~2 ulp of 1/d (pinned against 1/d in tests/test_spec_math.py).     */
/* On gfx950 it is 7 full-rate VALU ops against the IEEE division's 11, one  */
/* of them the quarter-rate v_rcp_f32.                       */
/* ------------------------------------------------------------------------ */
VO_HD float vo_rcp_nr(float d)
{
    float r = vo_u32_as_f32(0x7EF311C3u - vo_f32_as_u32(d));
    float e = fmaf(-d, r, 1.0f);
    r = fmaf(r, e, r);
    e = fmaf(-d, r, 1.0f);
    r = fmaf(r, e, r);
    e = fmaf(-d, r, 1.0f);
    return fmaf(r, e, r);
}

/* ------------------------------------------------------------------------ */
/* Descriptor window weight, separable.  OpenCV weighs a descriptor sample  */
/* by exp((c_rot^2 + r_rot^2) s) with c_rot^2 + r_rot^2 = (i^2 + j^2) /      */
/* hist_width^2 (a rotation).  The spec takes the product of the two         */
/* one-dimensional factors (s' = s / hist_width^2),                          */
/*   w(i, j) = vo_sift_wt(s', |i|) * vo_sift_wt(s', |j|),                    */
/* equal in exact arithmetic and within float rounding of OpenCV's value,    */
/* so k_desc reads both factors from a per-keypoint table of radius + 1      */
/* entries instead of evaluating an exp per sample.  k^2 s' must lie in      */
/* [-87, 0] (vo_expf_nonpos): at most ~1.6 over the rotated square.  (The    */
/* orientation window keeps one exp of (i^2 + j^2) s: there the table's two  */
/* LDS reads per sample measured slower than the exp)        */
/* ------------------------------------------------------------------------ */
VO_HD float vo_sift_wt(float s, int k) { return vo_expf_nonpos((float)(k * k) * s); }

/* ------------------------------------------------------------------------ */
/* atan2 in DEGREES, result in [0, 360): OpenCV's fastAtan2 (the published  */
/* 7th-order polynomial cv::hal::fastAtan2 applies in SIFT's orientation     */
/* histogram and descriptor), with lo = min(|x|,|y|), hi = max:              */
/*   c = lo / (hi + DBL_EPSILON),  a = (((p7 c^2 + p5) c^2 + p3) c^2 + p1) c */
/* in degrees, then the octant/quadrant folds.  Deterministic form: the      */
/* quotient is lo * vo_rcp_nr(hi + DBL_EPSILON) (within 2 ulp of OpenCV's    */
/* division) and the Horner steps are fmaf; select-only, no branches.  The   */
/* polynomial's own error against the true atan2 is < 0.01 deg.  A result    */
/* that rounds up to 360 (y < 0 at a vanishing angle) wraps to 0.            */
/* ------------------------------------------------------------------------ */
VO_HD float vo_atan2_deg(float y, float x)
{
    const float ax = fabsf(x), ay = fabsf(y);
    const int swap = ay > ax;
    const float lo = swap ? ax : ay, hi = swap ? ay : ax;
    const float c = lo * vo_rcp_nr(hi + 2.220446049250313e-16f);
    const float c2 = c * c;
    const float p1 = 0.9997878412794807f * 57.29577951308232f, p3 = -0.3258083974640975f * 57.29577951308232f;
    const float p5 = 0.1555786518463281f * 57.29577951308232f, p7 = -0.04432655554792128f * 57.29577951308232f;
    float a = fmaf(fmaf(fmaf(p7, c2, p5), c2, p3), c2, p1) * c;
    a = swap ? 90.0f - a : a;
    a = x < 0.0f ? 180.0f - a : a;
    a = y < 0.0f ? 360.0f - a : a;
    return a >= 360.0f ? 0.0f : a;
}

/* ------------------------------------------------------------------------ */
/* sin / cos of an angle given in DEGREES, any finite value.                 */
/* Reduction in degrees (exact fmodf-free: integer quadrant), then Taylor.   */
/* ------------------------------------------------------------------------ */
VO_HD void vo_sincos_deg(float deg, float *s_out, float *c_out)
{
    /* quadrant q = round(deg/90), residual in [-45, 45] degrees */
    float qf = rintf(deg * (1.0f / 90.0f));
    float rd = deg - qf * 90.0f;                      /* exact for |deg| < 2^15 */
    float r = rd * 0.017453292519943296f;             /* radians, |r| <= pi/4 */
    float r2 = r * r;
    float s = -2.50521084e-8f;                        /* -1/11! */
    s = fmaf(s, r2, 2.75573192e-6f);                  /* 1/9! */
    s = fmaf(s, r2, -1.98412698e-4f);                 /* -1/7! */
    s = fmaf(s, r2, 8.33333333e-3f);                  /* 1/5! */
    s = fmaf(s, r2, -1.66666667e-1f);                 /* -1/3! */
    s = s * r2;
    s = fmaf(s, r, r);
    float c = 2.08767570e-9f;                         /* 1/12! */
    c = fmaf(c, r2, -2.75573192e-7f);                 /* -1/10! */
    c = fmaf(c, r2, 2.48015873e-5f);                  /* 1/8! */
    c = fmaf(c, r2, -1.38888889e-3f);                 /* -1/6! */
    c = fmaf(c, r2, 4.16666667e-2f);                  /* 1/4! */
    c = fmaf(c, r2, -0.5f);
    c = fmaf(c, r2, 1.0f);
    int q = ((int)qf) & 3;
    float so, co;
    if (q == 0)      { so = s;  co = c;  }
    else if (q == 1) { so = c;  co = -s; }
    else if (q == 2) { so = -s; co = -c; }
    else             { so = -c; co = s;  }
    *s_out = so; *c_out = co;
}

/* ------------------------------------------------------------------------ */
/* double exp / log (host+device), basic ops only.                           */
/* ------------------------------------------------------------------------ */
VO_HD double vo_exp_d(double x)
{
    if (x < -708.0) return 0.0;
    if (x > 709.0) x = 709.0;
    double kf = rint(x * 1.4426950408889634);
    double r = x - kf * 6.93147180369123816490e-01;
    r = r - kf * 1.90821492927058770002e-10;
    /* Taylor to r^13, |r| <= 0.347 -> truncation < 1e-17 */
    double p = 1.0 / 6227020800.0;
    p = fma(p, r, 1.0 / 479001600.0);
    p = fma(p, r, 1.0 / 39916800.0);
    p = fma(p, r, 1.0 / 3628800.0);
    p = fma(p, r, 1.0 / 362880.0);
    p = fma(p, r, 1.0 / 40320.0);
    p = fma(p, r, 1.0 / 5040.0);
    p = fma(p, r, 1.0 / 720.0);
    p = fma(p, r, 1.0 / 120.0);
    p = fma(p, r, 1.0 / 24.0);
    p = fma(p, r, 1.0 / 6.0);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    int64_t k = (int64_t)kf;
    int64_t k1 = k / 2, k2 = k - k1;
    double s1 = vo_u64_as_f64((uint64_t)(k1 + 1023) << 52);
    double s2 = vo_u64_as_f64((uint64_t)(k2 + 1023) << 52);
    return (p * s1) * s2;
}

/* natural log for x > 0 (returns -inf-ish sentinel -1e308 for x <= 0) */
VO_HD double vo_log_d(double x)
{
    if (!(x > 0.0)) return -1.0e308;
    uint64_t u = vo_f64_as_u64(x);
    int e = (int)((u >> 52) & 0x7ff);
    if (e == 0) {                           /* subnormal: scale up */
        x = x * 18014398509481984.0;       /* 2^54 */
        u = vo_f64_as_u64(x);
        e = (int)((u >> 52) & 0x7ff) - 54;
    }
    e -= 1023;
    double m = vo_u64_as_f64((u & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL); /* [1,2) */
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    double s = (m - 1.0) / (m + 1.0);        /* |s| <= 0.1716 */
    double s2 = s * s;
    double p = 1.0 / 23.0;
    p = fma(p, s2, 1.0 / 21.0);
    p = fma(p, s2, 1.0 / 19.0);
    p = fma(p, s2, 1.0 / 17.0);
    p = fma(p, s2, 1.0 / 15.0);
    p = fma(p, s2, 1.0 / 13.0);
    p = fma(p, s2, 1.0 / 11.0);
    p = fma(p, s2, 1.0 / 9.0);
    p = fma(p, s2, 1.0 / 7.0);
    p = fma(p, s2, 1.0 / 5.0);
    p = fma(p, s2, 1.0 / 3.0);
    p = fma(p, s2, 1.0);
    double lm = 2.0 * s * p;
    return (double)e * 6.93147180559945286227e-01 + lm;
}

/* ------------------------------------------------------------------------ */
/* Philox4x32-10 counter-based RNG (Salmon et al., SC'11).                   */
/* ------------------------------------------------------------------------ */
typedef struct { uint32_t v[4]; } vo_u32x4;

VO_HD vo_u32x4 vo_philox4x32_10(vo_u32x4 ctr, uint32_t k0, uint32_t k1)
{
    for (int i = 0; i < 10; ++i) {
        uint64_t p0 = (uint64_t)0xD2511F53u * ctr.v[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr.v[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        vo_u32x4 n;
        n.v[0] = hi1 ^ ctr.v[1] ^ k0;
        n.v[1] = lo1;
        n.v[2] = hi0 ^ ctr.v[3] ^ k1;
        n.v[3] = lo0;
        ctr = n;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return ctr;
}

/* unbiased-enough index in [0, n) from a u32 (multiply-shift; spec) */
VO_HD uint32_t vo_rand_index(uint32_t r, uint32_t n) { return (uint32_t)(((uint64_t)r * n) >> 32); }

/* ------------------------------------------------------------------------ */
/* Fixed-point histogram accumulation.  Integer addition is associative, so  */
/* the GPU may add contributions in any order (LDS atomics, per-lane rows,   */
/* several copies) and still equal the oracle's serial loop bit for bit.     */
/* Orientation and descriptor histograms: unsigned 32-bit fixed point at     */
/* 2^-10.  A weight v >= 0 is pre-scaled by 2^10 (exact: a power of two) and  */
/* enters as rintf(v).  Overflow-free by construction, |dI| <= 255 so one     */
/* weight is < 361*2^10:                                                      */
/*  - descriptor: a spatial bin collects fewer than (2*hist_width+2)^2 <=     */
/*    5.5e3 samples once the radius is capped at VO_SIFT_DESCR_RMAX           */
/*    (hist_width <= 36.3): < 2.1e9 < 2^32;                                   */
/*  - orientation: bins are summed in 64 bits (any window size).              */
/* A bin converts back with one correct rounding: (float)sum * 2^-10.        */
/* Rounding: floor(v + 1/2) (half up).  v + 1/2 is exact for v < 2^22, far  */
/* above any weight, so this is one v_cvt_rpi_i32_f32 on the GPU.           */
/* ------------------------------------------------------------------------ */
#define VO_DESC_FX_SCALE 1024.0f
VO_HD uint32_t vo_desc_fx_quant(float v_scaled) { return (uint32_t)floorf(v_scaled + 0.5f); }
VO_HD float vo_desc_fx_to_float(uint32_t s) { return (float)s * (1.0f / VO_DESC_FX_SCALE); }
VO_HD float vo_hist_fx_to_float(uint64_t s) { return (float)s * (1.0f / VO_DESC_FX_SCALE); }

/* ------------------------------------------------------------------------ */
/* SIFT scale-space constants (spec, OpenCV-4.x conventions).  Computed on  */
/* the host by both the oracle and libvo with the deterministic exp/log     */
/* above, so the float kernels are identical.                                */
/* ------------------------------------------------------------------------ */
#define VO_SIFT_MAX_LAYERS 8      /* n_octave_layers <= 5 -> levels <= 8 */
#define VO_SIFT_MAX_OCTAVES 16
#define VO_SIFT_MAX_RADIUS 40
#define VO_SIFT_BORDER 5
#define VO_SIFT_MAX_INTERP 5
#define VO_SIFT_ORI_BINS 36
#define VO_SIFT_ORI_SIG 1.5f
#define VO_SIFT_ORI_RADIUS 4.5f   /* 3 * 1.5 */
#define VO_SIFT_ORI_PEAK 0.8f
#define VO_SIFT_DESCR_W 4
#define VO_SIFT_DESCR_BINS 8
#define VO_SIFT_DESCR_SCL 3.0f
#define VO_SIFT_DESCR_MAG_THR 0.2f
#define VO_SIFT_DESCR_INT_FCTR 512.0f
#define VO_SIFT_DESCR_RMAX 127     /* descriptor window radius cap (38 at the defaults); (2 RMAX + 1)^2 < 2^16 */
#define VO_SIFT_MAX_PEAKS 18      /* strict local maxima in a 36-bin circle */
#define VO_FLT_EPSILON 1.19209290e-07f

/* round-half-even for doubles (cvRound) */
VO_HD int vo_round_d(double x) { return (int)rint(x); }

/* number of octaves: cvRound(log2(min(base rows, cols)) - 2) - firstOctave */
VO_HD int vo_num_octaves(int rows, int cols, int upsample)
{
    int br = upsample ? rows * 2 : rows, bc = upsample ? cols * 2 : cols;
    int m = br < bc ? br : bc;
    double l2 = vo_log_d((double)m) / 0.69314718055994531;
    int n = vo_round_d(l2 - 2.0) + (upsample ? 1 : 0);
    if (n < 1) n = 1;
    if (n > VO_SIFT_MAX_OCTAVES) n = VO_SIFT_MAX_OCTAVES;
    return n;
}

/* sigma of the incremental blur producing level i (i=1..L+2) from level i-1;
 * sig[0] = sigma (the octave base's absolute blur). */
VO_HD void vo_level_sigmas(int L, double sigma, double* sig)
{
    sig[0] = sigma;
    for (int i = 1; i < L + 3; ++i) {
        double sig_prev = vo_exp_d((double)(i - 1) * 0.69314718055994531 / (double)L) * sigma;
        double sig_total = sig_prev * vo_exp_d(0.69314718055994531 / (double)L);
        sig[i] = sqrt(sig_total * sig_total - sig_prev * sig_prev);
    }
}

/* blur applied to the (upsampled) input to reach `sigma` (SIFT_INIT_SIGMA .5) */
VO_HD double vo_base_sigma(double sigma, int upsample)
{
    double init = upsample ? 1.0 : 0.5;     /* 0.5 * 2 when upsampled */
    double v = sigma * sigma - init * init;
    if (v < 0.01) v = 0.01;
    return sqrt(v);
}

/* Gaussian kernel (getGaussianKernel for float images, ksize = round(8s+1)|1).
 * Writes k[0..radius] (centre first); returns radius or -1 if > cap-1. */
VO_HD int vo_gauss_kernel(double s, float* k, int cap)
{
    int ksize = vo_round_d(s * 8.0 + 1.0) | 1;
    int r = ksize / 2;
    if (r + 1 > cap) return -1;
    double t[2 * VO_SIFT_MAX_RADIUS + 1];
    double sum = 0.0, scale2x = -0.5 / (s * s);
    for (int i = 0; i < ksize; ++i) {
        double x = (double)(i - r);
        t[i] = vo_exp_d(scale2x * x * x);
        sum += t[i];
    }
    sum = 1.0 / sum;
    for (int i = 0; i <= r; ++i) k[i] = (float)(t[r + i] * sum);
    return r;
}

/* reflect-101 border index (OpenCV BORDER_REFLECT_101, iterated) */
VO_HD int vo_reflect101(int p, int n)
{
    if (n == 1) return 0;
    while (p < 0 || p >= n) {
        if (p < 0) p = -p;
        else p = 2 * n - 2 - p;
    }
    return p;
}

#endif /* VO_SPEC_H */
