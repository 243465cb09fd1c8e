/*
 * sift_ref.c — CPU restatement of detectSIFTFeatures + extractFeatures
 * (VO.m:79-84).  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * "parity unpinned" vs MATLAB: the toolbox is closed.  The algorithm is the
 * published OpenCV-4.x SIFT (Lowe 2004 as implemented in opencv/modules/
 * features2d/src/sift.simd.hpp, which MATLAB's documented defaults match:
 * NumLayersInOctave 3, Sigma 1.6, ContrastThreshold 0.0133 = 0.04/3,
 * EdgeThreshold 10), restated with the deterministic choices written down in
 * DESIGN.md §3.1:
 *   - x2 bilinear upsample with half-pixel centres (exact in float),
 *   - separable Gaussian, reflect-101, symmetric fmaf accumulation order,
 *   - Cramer's rule in double for the 3x3 Newton step,
 *   - vo_spec.h exp/atan2/sincos,
 *   - orientation/descriptor histograms summed in 2^-10 fixed point (vo_spec.h
 *     VO_DESC_FX_SCALE = 1024: every contribution pre-scaled by 2^10, rounded
 *     to an integer, summed exactly),
 *   - descriptor norms as a 128 -> 1 pairwise tree,
 *   - keypoint order = (octave, layer, row, col) scan order, then peak bin.
 * Everything is plain C99 compiled with -ffp-contract=off.
 *
 * Built a second time with -DVO_CV_LITERAL (build/liboracle_cv.so) it is instead
 * the OpenCV-literal float SIFT those choices depart from: histograms accumulated
 * in float in OpenCV's sample order, OpenCV's fastAtan2 polynomial, libm
 * expf/sinf/cosf/powf, sequential float norms, no descriptor-radius cap, and
 * KeyPointsFilter::removeDuplicatedSorted (sort by x, y, size, angle; drop
 * exact duplicates).  tests/test_spec_divergence.py measures how far the spec
 * is from it.
 */
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "oracle.h"
#include "vo_spec.h"

#ifdef VO_CV_LITERAL
#include <float.h>
/* OpenCV's cv::fastAtan2 (degrees in [0, 360)): the published 7th-order polynomial */
static float cv_fast_atan2(float y, float x)
{
    const float p1 = 0.9997878412794807f * 57.29577951308232f, p3 = -0.3258083974640975f * 57.29577951308232f;
    const float p5 = 0.1555786518463281f * 57.29577951308232f, p7 = -0.04432655554792128f * 57.29577951308232f;
    float ax = fabsf(x), ay = fabsf(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.0f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.0f - a;
    if (y < 0) a = 360.0f - a;
    return a;
}
#define SIFT_EXPF(x) expf(x)
#define SIFT_ATAN2(y, x) cv_fast_atan2((y), (x))
#else
#define SIFT_EXPF(x) vo_expf(x)
#define SIFT_ATAN2(y, x) vo_atan2_deg((y), (x))
#endif

int oracle_num_octaves(int rows, int cols, int upsample) { return vo_num_octaves(rows, cols, upsample); }

int oracle_gauss_kernel(double sigma, float* k, int cap) { return vo_gauss_kernel(sigma, k, cap); }

/* x2 upsample, half-pixel centres: out = .75*near + .25*far (rows, then cols) */
void oracle_upsample(const uint8_t* img, int rows, int cols, int ld, float* out)
{
    int R = rows * 2, C = cols * 2;
    for (int y = 0; y < R; ++y) {
        int ya = y >> 1, yb = (y & 1) ? (ya + 1 < rows ? ya + 1 : rows - 1) : (ya > 0 ? ya - 1 : 0);
        for (int x = 0; x < C; ++x) {
            int xa = x >> 1, xb = (x & 1) ? (xa + 1 < cols ? xa + 1 : cols - 1) : (xa > 0 ? xa - 1 : 0);
            float ha = 0.75f * (float)img[ya * ld + xa] + 0.25f * (float)img[ya * ld + xb];
            float hb = 0.75f * (float)img[yb * ld + xa] + 0.25f * (float)img[yb * ld + xb];
            out[y * C + x] = 0.75f * ha + 0.25f * hb;
        }
    }
}

/* separable blur: horizontal then vertical; acc = k0*s0; acc = fmaf(kj, s[-j]+s[+j], acc) */
void oracle_blur(const float* src, float* dst, int rows, int cols, const float* k, int r)
{
    float* tmp = (float*)malloc(sizeof(float) * (size_t)rows * cols);
    for (int y = 0; y < rows; ++y) {
        const float* s = src + (size_t)y * cols;
        for (int x = 0; x < cols; ++x) {
            float acc = k[0] * s[x];
            for (int j = 1; j <= r; ++j)
                acc = fmaf(k[j], s[vo_reflect101(x - j, cols)] + s[vo_reflect101(x + j, cols)], acc);
            tmp[(size_t)y * cols + x] = acc;
        }
    }
    for (int y = 0; y < rows; ++y) {
        for (int x = 0; x < cols; ++x) {
            float acc = k[0] * tmp[(size_t)y * cols + x];
            for (int j = 1; j <= r; ++j)
                acc = fmaf(k[j], tmp[(size_t)vo_reflect101(y - j, rows) * cols + x] +
                                 tmp[(size_t)vo_reflect101(y + j, rows) * cols + x], acc);
            dst[(size_t)y * cols + x] = acc;
        }
    }
    free(tmp);
}

typedef struct {
    int rows, cols;
    float* g[VO_SIFT_MAX_LAYERS];
    float* d[VO_SIFT_MAX_LAYERS];
} octave_t;

typedef struct {
    int n_oct, L;
    octave_t oct[VO_SIFT_MAX_OCTAVES];
} pyramid_t;

static void build_pyramid(const uint8_t* img, int rows, int cols, int ld, const vo_sift_params* p,
                          pyramid_t* py)
{
    int L = p->n_octave_layers, up = p->upsample;
    py->L = L;
    py->n_oct = vo_num_octaves(rows, cols, up);
    double sig[VO_SIFT_MAX_LAYERS];
    vo_level_sigmas(L, p->sigma, sig);
    float kern[VO_SIFT_MAX_RADIUS + 1];

    int R = up ? rows * 2 : rows, C = up ? cols * 2 : cols;
    float* base = (float*)malloc(sizeof(float) * (size_t)R * C);
    if (up) oracle_upsample(img, rows, cols, ld, base);
    else for (int y = 0; y < rows; ++y) for (int x = 0; x < cols; ++x) base[(size_t)y * C + x] = (float)img[y * ld + x];

    for (int o = 0; o < py->n_oct; ++o) {
        octave_t* oc = &py->oct[o];
        if (o == 0) { oc->rows = R; oc->cols = C; }
        else { oc->rows = py->oct[o - 1].rows / 2; oc->cols = py->oct[o - 1].cols / 2; }
        size_t np = (size_t)oc->rows * oc->cols;
        for (int i = 0; i < L + 3; ++i) oc->g[i] = (float*)malloc(sizeof(float) * np);
        for (int i = 0; i < L + 2; ++i) oc->d[i] = (float*)malloc(sizeof(float) * np);
        if (o == 0) {
            int r = vo_gauss_kernel(vo_base_sigma(p->sigma, up), kern, VO_SIFT_MAX_RADIUS + 1);
            oracle_blur(base, oc->g[0], R, C, kern, r);
        } else {
            const octave_t* pr = &py->oct[o - 1];
            for (int y = 0; y < oc->rows; ++y)
                for (int x = 0; x < oc->cols; ++x)
                    oc->g[0][(size_t)y * oc->cols + x] = pr->g[L][(size_t)(2 * y) * pr->cols + 2 * x];
        }
        for (int i = 1; i < L + 3; ++i) {
            int r = vo_gauss_kernel(sig[i], kern, VO_SIFT_MAX_RADIUS + 1);
            oracle_blur(oc->g[i - 1], oc->g[i], oc->rows, oc->cols, kern, r);
        }
        for (int i = 0; i < L + 2; ++i)
            for (size_t q = 0; q < np; ++q) oc->d[i][q] = oc->g[i + 1][q] - oc->g[i][q];
    }
    free(base);
}

static void free_pyramid(pyramid_t* py)
{
    for (int o = 0; o < py->n_oct; ++o) {
        for (int i = 0; i < py->L + 3; ++i) free(py->oct[o].g[i]);
        for (int i = 0; i < py->L + 2; ++i) free(py->oct[o].d[i]);
    }
}

long oracle_pyramid(const uint8_t* img, int rows, int cols, int ld, const vo_sift_params* p, float* out)
{
    int n_oct = vo_num_octaves(rows, cols, p->upsample), L = p->n_octave_layers;
    long total = 0;
    int r = p->upsample ? rows * 2 : rows, c = p->upsample ? cols * 2 : cols;
    for (int o = 0; o < n_oct; ++o) {
        if (o) { r /= 2; c /= 2; }
        total += (long)(2 * L + 5) * r * c;
    }
    if (!out) return total;
    pyramid_t py;
    build_pyramid(img, rows, cols, ld, p, &py);
    long off = 0;
    for (int o = 0; o < py.n_oct; ++o) {
        size_t np = (size_t)py.oct[o].rows * py.oct[o].cols;
        for (int i = 0; i < L + 3; ++i) { memcpy(out + off, py.oct[o].g[i], np * 4); off += (long)np; }
        for (int i = 0; i < L + 2; ++i) { memcpy(out + off, py.oct[o].d[i], np * 4); off += (long)np; }
    }
    free_pyramid(&py);
    return total;
}

/* ---------------- extremum refinement (adjustLocalExtrema) ---------------- */
typedef struct {
    float xo, yo;    /* octave-local refined position */
    float xi;        /* layer offset */
    float scl;       /* octave-local scale: sigma * 2^((layer+xi)/L) */
    float response;
    int r, c, layer; /* integer refined location */
} refined_t;

#define AT(img, cols, y, x) ((img)[(size_t)(y) * (cols) + (x)])

/* 3x3 symmetric solve by Cramer's rule in double; returns 0 if singular */
static int solve3(const float H[9], const float b[3], float X[3])
{
    double a00 = H[0], a01 = H[1], a02 = H[2], a10 = H[3], a11 = H[4], a12 = H[5], a20 = H[6], a21 = H[7], a22 = H[8];
    double c00 = a11 * a22 - a12 * a21, c01 = a10 * a22 - a12 * a20, c02 = a10 * a21 - a11 * a20;
    double det = a00 * c00 - a01 * c01 + a02 * c02;
    if (det == 0.0) { X[0] = X[1] = X[2] = 0.0f; return 0; }
    double b0 = b[0], b1 = b[1], b2 = b[2];
    double x0 = b0 * c00 - a01 * (b1 * a22 - a12 * b2) + a02 * (b1 * a21 - a11 * b2);
    double x1 = a00 * (b1 * a22 - a12 * b2) - b0 * c01 + a02 * (a10 * b2 - b1 * a20);
    double x2 = a00 * (a11 * b2 - b1 * a21) - a01 * (a10 * b2 - b1 * a20) + b0 * c02;
    double inv = 1.0 / det;
    X[0] = (float)(x0 * inv); X[1] = (float)(x1 * inv); X[2] = (float)(x2 * inv);
    return 1;
}

static int refine(const pyramid_t* py, int o, int layer, int r, int c, const vo_sift_params* p, refined_t* out)
{
    const float img_scale = 1.0f / 255.0f;
    const float ds = img_scale * 0.5f, ss = img_scale, cs = img_scale * 0.25f;
    const octave_t* oc = &py->oct[o];
    int rows = oc->rows, cols = oc->cols, L = py->L;
    float xi = 0, xr = 0, xc = 0;
    int it = 0;
    for (; it < VO_SIFT_MAX_INTERP; ++it) {
        const float* im = oc->d[layer];
        const float* pv = oc->d[layer - 1];
        const float* nx = oc->d[layer + 1];
        float dD[3] = {(AT(im, cols, r, c + 1) - AT(im, cols, r, c - 1)) * ds,
                       (AT(im, cols, r + 1, c) - AT(im, cols, r - 1, c)) * ds,
                       (AT(nx, cols, r, c) - AT(pv, cols, r, c)) * ds};
        float v2 = AT(im, cols, r, c) * 2.0f;
        float dxx = (AT(im, cols, r, c + 1) + AT(im, cols, r, c - 1) - v2) * ss;
        float dyy = (AT(im, cols, r + 1, c) + AT(im, cols, r - 1, c) - v2) * ss;
        float dss = (AT(nx, cols, r, c) + AT(pv, cols, r, c) - v2) * ss;
        float dxy = (AT(im, cols, r + 1, c + 1) - AT(im, cols, r + 1, c - 1) - AT(im, cols, r - 1, c + 1) + AT(im, cols, r - 1, c - 1)) * cs;
        float dxs = (AT(nx, cols, r, c + 1) - AT(nx, cols, r, c - 1) - AT(pv, cols, r, c + 1) + AT(pv, cols, r, c - 1)) * cs;
        float dys = (AT(nx, cols, r + 1, c) - AT(nx, cols, r - 1, c) - AT(pv, cols, r + 1, c) + AT(pv, cols, r - 1, c)) * cs;
        float H[9] = {dxx, dxy, dxs, dxy, dyy, dys, dxs, dys, dss};
        float X[3];
        solve3(H, dD, X);
        xi = -X[2]; xr = -X[1]; xc = -X[0];
        if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
        const float big = (float)(0x7fffffff / 3);
        if (fabsf(xi) > big || fabsf(xr) > big || fabsf(xc) > big) return 0;
        c += vo_round(xc); r += vo_round(xr); layer += vo_round(xi);
        if (layer < 1 || layer > L || c < VO_SIFT_BORDER || c >= cols - VO_SIFT_BORDER ||
            r < VO_SIFT_BORDER || r >= rows - VO_SIFT_BORDER) return 0;
    }
    if (it >= VO_SIFT_MAX_INTERP) return 0;
    {
        const float* im = oc->d[layer];
        const float* pv = oc->d[layer - 1];
        const float* nx = oc->d[layer + 1];
        float dD[3] = {(AT(im, cols, r, c + 1) - AT(im, cols, r, c - 1)) * ds,
                       (AT(im, cols, r + 1, c) - AT(im, cols, r - 1, c)) * ds,
                       (AT(nx, cols, r, c) - AT(pv, cols, r, c)) * ds};
        float t = dD[0] * xc + dD[1] * xr + dD[2] * xi;
        float contr = AT(im, cols, r, c) * img_scale + t * 0.5f;
        if (fabsf(contr) * (float)L < p->contrast_threshold) return 0;
        float v2 = AT(im, cols, r, c) * 2.0f;
        float dxx = (AT(im, cols, r, c + 1) + AT(im, cols, r, c - 1) - v2) * ss;
        float dyy = (AT(im, cols, r + 1, c) + AT(im, cols, r - 1, c) - v2) * ss;
        float dxy = (AT(im, cols, r + 1, c + 1) - AT(im, cols, r + 1, c - 1) - AT(im, cols, r - 1, c + 1) + AT(im, cols, r - 1, c - 1)) * cs;
        float tr = dxx + dyy, det = dxx * dyy - dxy * dxy;
        float et = p->edge_threshold;
        if (det <= 0 || tr * tr * et >= (et + 1) * (et + 1) * det) return 0;
        out->xo = (float)c + xc;
        out->yo = (float)r + xr;
        out->xi = xi;
#ifdef VO_CV_LITERAL
        out->scl = p->sigma * powf(2.0f, ((float)layer + xi) / (float)L);
#else
        out->scl = p->sigma * vo_expf(((float)layer + xi) / (float)L * 0.693147181f);
#endif
        out->response = fabsf(contr);
        out->r = r; out->c = c; out->layer = layer;
    }
    return 1;
}

/* ---------------- orientation histogram ---------------- */
/* returns number of peaks written to angles[] */
static int orientations(const float* img, int rows, int cols, int r, int c, float scl, float* angles)
{
    const int n = VO_SIFT_ORI_BINS;
    int radius = vo_round(VO_SIFT_ORI_RADIUS * scl);
    float sigw = VO_SIFT_ORI_SIG * scl;
    float expf_scale = -1.0f / (2.0f * sigw * sigw);
#ifdef VO_CV_LITERAL
    float hfl[VO_SIFT_ORI_BINS];
    memset(hfl, 0, sizeof(hfl));
#else
    uint64_t hfx[VO_SIFT_ORI_BINS];
    memset(hfx, 0, sizeof(hfx));
#endif
    for (int i = -radius; i <= radius; ++i) {
        int y = r + i;
        if (y <= 0 || y >= rows - 1) continue;
        for (int j = -radius; j <= radius; ++j) {
            int x = c + j;
            if (x <= 0 || x >= cols - 1) continue;
            float dx = AT(img, cols, y, x + 1) - AT(img, cols, y, x - 1);
            float dy = AT(img, cols, y - 1, x) - AT(img, cols, y + 1, x);
            float w = SIFT_EXPF((float)(i * i + j * j) * expf_scale);
            float mag = sqrtf(dx * dx + dy * dy);
            float ori = SIFT_ATAN2(dy, dx);
            int bin = vo_round((float)n / 360.0f * ori);
            if (bin >= n) bin -= n;
            if (bin < 0) bin += n;
#ifdef VO_CV_LITERAL
            hfl[bin] += w * mag;
#else
            hfx[bin] += vo_desc_fx_quant((w * mag) * VO_DESC_FX_SCALE);
#endif
        }
    }
    float t[VO_SIFT_ORI_BINS], hist[VO_SIFT_ORI_BINS];
#ifdef VO_CV_LITERAL
    for (int k = 0; k < n; ++k) t[k] = hfl[k];
#else
    for (int k = 0; k < n; ++k) t[k] = vo_hist_fx_to_float(hfx[k]);
#endif
    float maxval = 0.0f;
    for (int k = 0; k < n; ++k) {
        float m2 = t[(k + n - 2) % n], m1 = t[(k + n - 1) % n], p1 = t[(k + 1) % n], p2 = t[(k + 2) % n];
        hist[k] = (m2 + p2) * (1.0f / 16.0f) + (m1 + p1) * (4.0f / 16.0f) + t[k] * (6.0f / 16.0f);
        if (k == 0 || hist[k] > maxval) maxval = hist[k];
    }
    float mag_thr = maxval * VO_SIFT_ORI_PEAK;
    int np = 0;
    for (int j = 0; j < n; ++j) {
        int l = j > 0 ? j - 1 : n - 1, r2 = j < n - 1 ? j + 1 : 0;
        if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
            float bin = (float)j + 0.5f * (hist[l] - hist[r2]) / (hist[l] - 2.0f * hist[j] + hist[r2]);
            bin = bin < 0 ? (float)n + bin : bin >= (float)n ? bin - (float)n : bin;
            float ang = 360.0f - (360.0f / (float)n) * bin;
            if (fabsf(ang - 360.0f) < VO_FLT_EPSILON) ang = 0.0f;
            angles[np++] = ang;
        }
    }
    return np;
}

/* ---------------- descriptor ---------------- */
static void descriptor(const float* img, int rows, int cols, float xo, float yo, float kp_angle, float scl,
                       uint8_t* out)
{
    const int d = VO_SIFT_DESCR_W, n = VO_SIFT_DESCR_BINS;
    float ori = 360.0f - kp_angle;
    if (fabsf(ori - 360.0f) < VO_FLT_EPSILON) ori = 0.0f;
    int px = vo_round(xo), py = vo_round(yo);
    float sin_t, cos_t;
#ifdef VO_CV_LITERAL
    cos_t = cosf(ori * (float)(3.14159265358979323846 / 180));
    sin_t = sinf(ori * (float)(3.14159265358979323846 / 180));
#else
    vo_sincos_deg(ori, &sin_t, &cos_t);
#endif
    const float bins_per_deg = (float)n / 360.0f;
    const float exp_scale = -1.0f / ((float)(d * d) * 0.5f);
    float hist_width = VO_SIFT_DESCR_SCL * scl;
    int radius = vo_round(hist_width * 1.4142135623730951f * (float)(d + 1) * 0.5f);
    int rmax = (int)sqrt((double)cols * cols + (double)rows * rows);
    if (radius > rmax) radius = rmax;
#ifdef VO_CV_LITERAL
    typedef float hist_t;                 /* OpenCV: float bins, no radius cap */
#define HQ(v) (v)
#else
    if (radius > VO_SIFT_DESCR_RMAX) radius = VO_SIFT_DESCR_RMAX;
    typedef uint32_t hist_t;
#define HQ(v) vo_desc_fx_quant(v)
#endif
    cos_t = cos_t / hist_width;
    sin_t = sin_t / hist_width;
#ifndef VO_CV_LITERAL
    /* separable window weight (vo_spec.h vo_sift_wt): exp((c_rot^2 + r_rot^2) exp_scale) =
     * exp(i^2 s) exp(j^2 s), s = exp_scale / hist_width^2 -- w(i, j) = wt[|i|] * wt[|j|] */
    const float wsc = exp_scale / (hist_width * hist_width);
    float wt[VO_SIFT_DESCR_RMAX + 1];
    for (int k = 0; k <= radius; ++k) wt[k] = vo_sift_wt(wsc, k);
#endif
    hist_t hfx[(VO_SIFT_DESCR_W + 2) * (VO_SIFT_DESCR_W + 2) * (VO_SIFT_DESCR_BINS + 2)];
    memset(hfx, 0, sizeof(hfx));
    for (int i = -radius; i <= radius; ++i) {
        for (int j = -radius; j <= radius; ++j) {
            float c_rot = (float)j * cos_t - (float)i * sin_t;
            float r_rot = (float)j * sin_t + (float)i * cos_t;
            float rbin = r_rot + (float)(d / 2) - 0.5f;
            float cbin = c_rot + (float)(d / 2) - 0.5f;
            int r = py + i, c = px + j;
            if (!(rbin > -1.0f && rbin < (float)d && cbin > -1.0f && cbin < (float)d &&
                  r > 0 && r < rows - 1 && c > 0 && c < cols - 1)) continue;
            float dx = AT(img, cols, r, c + 1) - AT(img, cols, r, c - 1);
            float dy = AT(img, cols, r - 1, c) - AT(img, cols, r + 1, c);
#ifdef VO_CV_LITERAL
            float w = SIFT_EXPF((c_rot * c_rot + r_rot * r_rot) * exp_scale);
#else
            float w = wt[i < 0 ? -i : i] * wt[j < 0 ? -j : j];
#endif
            float ang = SIFT_ATAN2(dy, dx);
#ifdef VO_CV_LITERAL
            float mag = sqrtf(dx * dx + dy * dy) * w;
#else
            float mag = (sqrtf(dx * dx + dy * dy) * w) * VO_DESC_FX_SCALE;   /* exact power-of-two pre-scale */
#endif
            float obin = (ang - ori) * bins_per_deg;
            int r0 = vo_floor(rbin), c0 = vo_floor(cbin), o0 = vo_floor(obin);
            rbin -= (float)r0; cbin -= (float)c0; obin -= (float)o0;
            if (o0 < 0) o0 += n;
            if (o0 >= n) o0 -= n;
            float v_r1 = mag * rbin, v_r0 = mag - v_r1;
            float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
            float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
            float v_rco111 = v_rc11 * obin, v_rco110 = v_rc11 - v_rco111;
            float v_rco101 = v_rc10 * obin, v_rco100 = v_rc10 - v_rco101;
            float v_rco011 = v_rc01 * obin, v_rco010 = v_rc01 - v_rco011;
            float v_rco001 = v_rc00 * obin, v_rco000 = v_rc00 - v_rco001;
            int idx = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
            hfx[idx] += HQ(v_rco000);
            hfx[idx + 1] += HQ(v_rco001);
            hfx[idx + (n + 2)] += HQ(v_rco010);
            hfx[idx + (n + 3)] += HQ(v_rco011);
            hfx[idx + (d + 2) * (n + 2)] += HQ(v_rco100);
            hfx[idx + (d + 2) * (n + 2) + 1] += HQ(v_rco101);
            hfx[idx + (d + 3) * (n + 2)] += HQ(v_rco110);
            hfx[idx + (d + 3) * (n + 2) + 1] += HQ(v_rco111);
        }
    }
    float dst[VO_DESC_LEN];
    for (int i = 0; i < d; ++i)
        for (int j = 0; j < d; ++j) {
            int idx = ((i + 1) * (d + 2) + (j + 1)) * (n + 2);
            hfx[idx] += hfx[idx + n];
            hfx[idx + 1] += hfx[idx + n + 1];
#ifdef VO_CV_LITERAL
            for (int k = 0; k < n; ++k) dst[(i * d + j) * n + k] = hfx[idx + k];
#else
            for (int k = 0; k < n; ++k) dst[(i * d + j) * n + k] = vo_desc_fx_to_float(hfx[idx + k]);
#endif
        }
#undef HQ
#ifdef VO_CV_LITERAL
    /* OpenCV: sequential float sums */
    float nrm2 = 0;
    for (int k = 0; k < VO_DESC_LEN; ++k) nrm2 += dst[k] * dst[k];
    float thr = sqrtf(nrm2) * VO_SIFT_DESCR_MAG_THR;
    nrm2 = 0;
    for (int k = 0; k < VO_DESC_LEN; ++k) { float v = dst[k] < thr ? dst[k] : thr; dst[k] = v; nrm2 += v * v; }
    float nrm = sqrtf(nrm2);
#else
    /* norms: pairwise tree 128 -> 1 (stride 64, 32, ..., 1) */
    float s[VO_DESC_LEN];
    for (int k = 0; k < VO_DESC_LEN; ++k) s[k] = dst[k] * dst[k];
    for (int st = 64; st >= 1; st >>= 1) for (int k = 0; k < st; ++k) s[k] = s[k] + s[k + st];
    float thr = sqrtf(s[0]) * VO_SIFT_DESCR_MAG_THR;
    for (int k = 0; k < VO_DESC_LEN; ++k) { float v = dst[k] < thr ? dst[k] : thr; dst[k] = v; s[k] = v * v; }
    for (int st = 64; st >= 1; st >>= 1) for (int k = 0; k < st; ++k) s[k] = s[k] + s[k + st];
    float nrm = sqrtf(s[0]);
#endif
    float scale = VO_SIFT_DESCR_INT_FCTR / (nrm > VO_FLT_EPSILON ? nrm : VO_FLT_EPSILON);
    for (int k = 0; k < VO_DESC_LEN; ++k) {
        float v = rintf(dst[k] * scale);
        out[k] = (uint8_t)(v < 0.0f ? 0 : v > 255.0f ? 255 : (int)v);
    }
}

#ifdef VO_CV_LITERAL
/* KeyPointsFilter::removeDuplicatedSorted: sort by (x, y, size, angle), drop entries whose
 * x, y, size and angle all equal the previous kept one (descriptors follow their keypoint) */
static const vo_keypoint* g_sort_kps;
static int cv_kp_less(const void* a, const void* b)
{
    const vo_keypoint *p = &g_sort_kps[*(const int*)a], *q = &g_sort_kps[*(const int*)b];
    if (p->x != q->x) return p->x < q->x ? -1 : 1;
    if (p->y != q->y) return p->y < q->y ? -1 : 1;
    if (p->size != q->size) return p->size > q->size ? -1 : 1;    /* OpenCV: larger size first */
    if (p->angle != q->angle) return p->angle < q->angle ? -1 : 1;
    if (p->response != q->response) return p->response > q->response ? -1 : 1;
    if (p->octave != q->octave) return p->octave > q->octave ? -1 : 1;
    return *(const int*)a - *(const int*)b;
}

static int cv_remove_duplicated_sorted(vo_keypoint* kps, uint8_t* desc, int n)
{
    int* ord = (int*)malloc(sizeof(int) * (n + 1));
    for (int i = 0; i < n; ++i) ord[i] = i;
    g_sort_kps = kps;
    qsort(ord, n, sizeof(int), cv_kp_less);
    vo_keypoint* k2 = (vo_keypoint*)malloc(sizeof(vo_keypoint) * (n + 1));
    uint8_t* d2 = desc ? (uint8_t*)malloc((size_t)(n + 1) * VO_DESC_LEN) : NULL;
    int m = 0;
    for (int i = 0; i < n; ++i) {
        const vo_keypoint* k = &kps[ord[i]];
        if (m > 0 && k->x == k2[m - 1].x && k->y == k2[m - 1].y && k->size == k2[m - 1].size && k->angle == k2[m - 1].angle)
            continue;
        k2[m] = *k;
        if (d2) memcpy(d2 + (size_t)m * VO_DESC_LEN, desc + (size_t)ord[i] * VO_DESC_LEN, VO_DESC_LEN);
        m++;
    }
    memcpy(kps, k2, sizeof(vo_keypoint) * m);
    if (d2) memcpy(desc, d2, (size_t)m * VO_DESC_LEN);
    free(ord); free(k2); free(d2);
    return m;
}
#endif

/* ---------------- detect + describe ---------------- */
int oracle_sift(const uint8_t* img, int rows, int cols, int ld, const vo_sift_params* p,
                vo_keypoint* kps, uint8_t* desc, int capacity)
{
    pyramid_t py;
    build_pyramid(img, rows, cols, ld, p, &py);
    const int L = py.L;
    const float thr = (float)floor(0.5 * p->contrast_threshold / L * 255.0);
    const float up_scale = p->upsample ? 0.5f : 1.0f;
    int count = 0;
    for (int o = 0; o < py.n_oct; ++o) {
        const octave_t* oc = &py.oct[o];
        int R = oc->rows, C = oc->cols;
        for (int i = 1; i <= L; ++i) {
            const float* cur = oc->d[i];
            const float* prv = oc->d[i - 1];
            const float* nxt = oc->d[i + 1];
            for (int r = VO_SIFT_BORDER; r < R - VO_SIFT_BORDER; ++r) {
                for (int c = VO_SIFT_BORDER; c < C - VO_SIFT_BORDER; ++c) {
                    float val = AT(cur, C, r, c);
                    if (!(fabsf(val) > thr)) continue;
                    int ext = 1;
                    if (val > 0) {
                        for (int dy = -1; dy <= 1 && ext; ++dy)
                            for (int dx = -1; dx <= 1; ++dx) {
                                if (!(val >= AT(prv, C, r + dy, c + dx) && val >= AT(nxt, C, r + dy, c + dx) &&
                                      val >= AT(cur, C, r + dy, c + dx))) { ext = 0; break; }
                            }
                    } else {
                        for (int dy = -1; dy <= 1 && ext; ++dy)
                            for (int dx = -1; dx <= 1; ++dx) {
                                if (!(val <= AT(prv, C, r + dy, c + dx) && val <= AT(nxt, C, r + dy, c + dx) &&
                                      val <= AT(cur, C, r + dy, c + dx))) { ext = 0; break; }
                            }
                    }
                    if (!ext) continue;
                    refined_t kp;
                    if (!refine(&py, o, i, r, c, p, &kp)) continue;
                    float angles[VO_SIFT_MAX_PEAKS + 2];
                    const float* gimg = oc->g[kp.layer];
                    int np = orientations(gimg, R, C, kp.r, kp.c, kp.scl, angles);
                    /* octave pixel k <-> upsampled pixel 2^o k <-> original 2^o k / 2 - 0.25
                       (half-pixel-centre x2 upsample); +1 for MATLAB 1-based Location */
                    float oscale = (float)(1 << o) * up_scale;
                    float loc_off = p->upsample ? 0.75f : 1.0f;
                    for (int a = 0; a < np; ++a) {
                        if (count < capacity) {
                            vo_keypoint* k = &kps[count];
                            k->x = kp.xo * oscale + loc_off;
                            k->y = kp.yo * oscale + loc_off;
                            k->size = kp.scl * 2.0f * oscale;
                            k->angle = angles[a];
                            k->response = kp.response;
                            k->octave = o - (p->upsample ? 1 : 0);
                            k->layer = kp.layer;
                            k->scale = kp.scl * oscale;
                            if (desc) descriptor(gimg, R, C, kp.xo, kp.yo, angles[a], kp.scl, desc + (size_t)count * VO_DESC_LEN);
                        }
                        count++;
                    }
                }
            }
        }
    }
    free_pyramid(&py);
#ifdef VO_CV_LITERAL
    if (count <= capacity) count = cv_remove_duplicated_sorted(kps, desc, count);
#endif
    return count;
}
