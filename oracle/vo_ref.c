/*
 * vo_ref.c — CPU restatement of the VO.m per-frame path outside SIFT.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  "parity unpinned" vs MATLAB.
 *
 *   oracle_match        matchFeatures defaults (VO.m:87,283,293,311,323)
 *   oracle_track        find_remaining_points (VO.m:280-334)
 *   oracle_triangulate  triangulate, linear DLT + SVD null vector (VO.m:113-116)
 *   oracle_p3p          P3P (Grunert's quartic, Haralick et al. 1994 review)
 *   oracle_estworldpose estworldpose: P3P inside MSAC (VO.m:123-127)
 *   oracle_landmarks    VO.m:145-158 + CreateLandmarksFromFeatures.m:1-21
 *   oracle_run_sequence VO.m:64-232 (loop, state, quirks Q1-Q5)
 * Spec choices are written down in DESIGN.md §3.
 */
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "oracle.h"
#include "vo_spec.h"

/* ======================================================================= */
/* matchFeatures                                                            */
/* ======================================================================= */
static float inv_norm_u8(const uint8_t* a)
{
    int32_t s = 0;
    for (int k = 0; k < VO_DESC_LEN; ++k) s += (int32_t)a[k] * (int32_t)a[k];
    return s > 0 ? 1.0f / sqrtf((float)s) : 0.0f;
}

/* normalized SSD from the exact integer dot product */
static float ssd_u8(const uint8_t* a, const uint8_t* b, float ia, float ib)
{
    int32_t d = 0;
    for (int k = 0; k < VO_DESC_LEN; ++k) d += (int32_t)a[k] * (int32_t)b[k];
    float c = ((float)d * ia) * ib;
    return 2.0f - 2.0f * c;
}

#ifdef VO_CV_LITERAL
/* MATLAB-literal matchFeatures (Exhaustive, SSD, Prenormalized false): single rows
 * normalised to unit L2 in float, SSD as a sequential float sum of squared differences */
static void unit_rows(const uint8_t* A, const int* ia, int n, float* out)
{
    for (int i = 0; i < n; ++i) {
        const uint8_t* a = A + (size_t)ia[i] * VO_DESC_LEN;
        float s = 0;
        for (int k = 0; k < VO_DESC_LEN; ++k) s += (float)a[k] * (float)a[k];
        float nrm = sqrtf(s);
        for (int k = 0; k < VO_DESC_LEN; ++k) out[(size_t)i * VO_DESC_LEN + k] = nrm > 0 ? (float)a[k] / nrm : 0.0f;
    }
}

static int match_idx(const uint8_t* A, const int* ia, int n1, const uint8_t* B, const int* ib, int n2,
                     const vo_match_params* p, int* out1, int* out2)
{
    float* fa = (float*)malloc(sizeof(float) * VO_DESC_LEN * (n1 > 0 ? n1 : 1));
    float* fb = (float*)malloc(sizeof(float) * VO_DESC_LEN * (n2 > 0 ? n2 : 1));
    unit_rows(A, ia, n1, fa);
    unit_rows(B, ib, n2, fb);
    const float T = p->match_threshold * 0.04f;
    int P = 0;
    for (int i = 0; i < n1; ++i) {
        const float* a = fa + (size_t)i * VO_DESC_LEN;
        float best = INFINITY, second = INFINITY;
        int bidx = -1;
        for (int j = 0; j < n2; ++j) {
            const float* b = fb + (size_t)j * VO_DESC_LEN;
            float s = 0;
            for (int k = 0; k < VO_DESC_LEN; ++k) { float t = a[k] - b[k]; s += t * t; }
            if (s < best) { second = best; best = s; bidx = j; }
            else if (s < second) second = s;
        }
        if (bidx < 0) continue;
        if (!(best <= T)) continue;
        if (!(best / second <= p->max_ratio)) continue;
        out1[P] = i; out2[P] = bidx; P++;
    }
    free(fa); free(fb);
    return P;
}
#else
/* generic match on gathered rows: F1 rows = A[ia[i]], F2 rows = B[ib[j]] */
static int match_idx(const uint8_t* A, const int* ia, int n1, const uint8_t* B, const int* ib, int n2,
                     const vo_match_params* p, int* out1, int* out2)
{
    float* inb = (float*)malloc(sizeof(float) * (n2 > 0 ? n2 : 1));
    for (int j = 0; j < n2; ++j) inb[j] = inv_norm_u8(B + (size_t)ib[j] * VO_DESC_LEN);
    const float T = p->match_threshold * 0.04f;
    int P = 0;
    for (int i = 0; i < n1; ++i) {
        const uint8_t* a = A + (size_t)ia[i] * VO_DESC_LEN;
        float ina = inv_norm_u8(a);
        float best = INFINITY, second = INFINITY;
        int bidx = -1;
        for (int j = 0; j < n2; ++j) {
            float s = ssd_u8(a, B + (size_t)ib[j] * VO_DESC_LEN, ina, inb[j]);
            if (s < best) { second = best; best = s; bidx = j; }
            else if (s < second) second = s;
        }
        if (bidx < 0) continue;
        if (!(best <= T)) continue;
        float ratio = best / second;
        if (!(ratio <= p->max_ratio)) continue;
        out1[P] = i; out2[P] = bidx; P++;
    }
    free(inb);
    return P;
}
#endif

int oracle_match(const uint8_t* F1, int n1, const uint8_t* F2, int n2, const vo_match_params* p,
                 uint32_t* pairs, int capacity)
{
    int* ia = (int*)malloc(sizeof(int) * (n1 + 1));
    int* ib = (int*)malloc(sizeof(int) * (n2 + 1));
    int* o1 = (int*)malloc(sizeof(int) * (n1 + 1));
    int* o2 = (int*)malloc(sizeof(int) * (n1 + 1));
    for (int i = 0; i < n1; ++i) ia[i] = i;
    for (int j = 0; j < n2; ++j) ib[j] = j;
    int P = match_idx(F1, ia, n1, F2, ib, n2, p, o1, o2);
    for (int k = 0; k < P && k < capacity; ++k) { pairs[2 * k] = (uint32_t)o1[k] + 1; pairs[2 * k + 1] = (uint32_t)o2[k] + 1; }
    free(ia); free(ib); free(o1); free(o2);
    return P;
}

/* matchFeatures on general single-precision features (libvo vo_match_f32 when the rows are not
 * u8-valued): rows normalised to unit L2 (a_k = f_k / sqrtf(fmaf chain of f_k^2), zero rows stay
 * zero), SSD as the fmaf chain of (a_k - b_k)^2 over k = 0..127, then the u8 path's selection
 * (smallest / second smallest, ties to the lowest F2 row; SSD <= 0.04 * MatchThreshold; ratio
 * <= MaxRatio).  Element k of row i: F[col_major ? k * ld + i : i * ld + k]. */
static void norm_rows_f32(const float* F, int n, int ld, int col_major, float* out)
{
    for (int i = 0; i < n; ++i) {
        float n2 = 0.0f;
        for (int k = 0; k < VO_DESC_LEN; ++k) {
            const float v = col_major ? F[(size_t)k * ld + i] : F[(size_t)i * ld + k];
            n2 = fmaf(v, v, n2);
        }
        const float nrm = sqrtf(n2);
        for (int k = 0; k < VO_DESC_LEN; ++k) {
            const float v = col_major ? F[(size_t)k * ld + i] : F[(size_t)i * ld + k];
            out[(size_t)i * VO_DESC_LEN + k] = nrm > 0.0f ? v / nrm : 0.0f;
        }
    }
}

int oracle_match_f32(const float* F1, int n1, int ld1, const float* F2, int n2, int ld2, int col_major,
                     const vo_match_params* p, uint32_t* pairs, int capacity)
{
    float* a = (float*)malloc(sizeof(float) * VO_DESC_LEN * (size_t)(n1 > 0 ? n1 : 1));
    float* b = (float*)malloc(sizeof(float) * VO_DESC_LEN * (size_t)(n2 > 0 ? n2 : 1));
    norm_rows_f32(F1, n1, ld1, col_major, a);
    norm_rows_f32(F2, n2, ld2, col_major, b);
    const float T = p->match_threshold * 0.04f;
    int P = 0;
    for (int i = 0; i < n1; ++i) {
        float best = INFINITY, second = INFINITY;
        int bidx = -1;
        for (int j = 0; j < n2; ++j) {
            float s = 0.0f;
            for (int k = 0; k < VO_DESC_LEN; ++k) {
                const float d = a[(size_t)i * VO_DESC_LEN + k] - b[(size_t)j * VO_DESC_LEN + k];
                s = fmaf(d, d, s);
            }
            if (s < best) { second = best; best = s; bidx = j; }
            else if (s < second) second = s;
        }
        if (bidx < 0 || !(best <= T) || !(best / second <= p->max_ratio)) continue;
        if (P < capacity) { pairs[2 * P] = (uint32_t)i + 1; pairs[2 * P + 1] = (uint32_t)bidx + 1; }
        P++;
    }
    free(a); free(b);
    return P;
}

/* ======================================================================= */
/* find_remaining_points (VO.m:280-334) as index composition                 */
/* ======================================================================= */
int oracle_track(const uint8_t* old_l, const uint8_t* old_r, int n_old,
                 const uint8_t* cur_l, int n_cl, const uint8_t* cur_r, int n_cr,
                 const vo_match_params* p, uint32_t* idx_out, int capacity)
{
    int nmax = n_old + n_cl + n_cr + 1;
    int* old_idx = (int*)malloc(sizeof(int) * nmax);
    int* cl = (int*)malloc(sizeof(int) * nmax);
    int* cr = (int*)malloc(sizeof(int) * nmax);
    int* m1 = (int*)malloc(sizeof(int) * nmax);
    int* m2 = (int*)malloc(sizeof(int) * nmax);
    int* tmp = (int*)malloc(sizeof(int) * nmax);
    int* all = (int*)malloc(sizeof(int) * nmax);
    for (int i = 0; i < nmax; ++i) all[i] = i;
    int n_o = n_old;
    for (int i = 0; i < n_o; ++i) old_idx[i] = i;
    /* lm = matchFeatures(cur.l_desc, old.l_desc)  VO.m:283; old <- old(lm(:,2))  :287-290 */
    int nlm = match_idx(cur_l, all, n_cl, old_l, old_idx, n_o, p, m1, m2);
    for (int k = 0; k < nlm; ++k) tmp[k] = old_idx[m2[k]];
    for (int k = 0; k < nlm; ++k) { old_idx[k] = tmp[k]; cl[k] = m1[k]; }   /* cur.l <- cur.l(lm(:,1)) :305-306 */
    n_o = nlm;
    /* rm = matchFeatures(cur.r_desc, old.r_desc)  VO.m:293; old <- old(rm(:,2))  :297-300 */
    int nrm = match_idx(cur_r, all, n_cr, old_r, old_idx, n_o, p, m1, m2);
    for (int k = 0; k < nrm; ++k) tmp[k] = old_idx[m2[k]];
    for (int k = 0; k < nrm; ++k) { old_idx[k] = tmp[k]; cr[k] = m1[k]; }   /* cur.r <- cur.r(rm(:,1)) :307-308 */
    n_o = nrm;
    /* cm = matchFeatures(cur.l_desc, cur.r_desc)  VO.m:311; gathers :314-317 */
    int ncm = match_idx(cur_l, cl, nlm, cur_r, cr, nrm, p, m1, m2);
    for (int k = 0; k < ncm; ++k) tmp[k] = cl[m1[k]];
    int* cl2 = (int*)malloc(sizeof(int) * nmax);
    int* cr2 = (int*)malloc(sizeof(int) * nmax);
    for (int k = 0; k < ncm; ++k) { cl2[k] = tmp[k]; cr2[k] = cr[m2[k]]; }
    /* last = matchFeatures(cur.l_desc, old.l_desc)  VO.m:323; gathers :326-333 */
    int nlast = match_idx(cur_l, cl2, ncm, old_l, old_idx, n_o, p, m1, m2);
    for (int k = 0; k < nlast && k < capacity; ++k) {
        idx_out[3 * k + 0] = (uint32_t)old_idx[m2[k]] + 1;
        idx_out[3 * k + 1] = (uint32_t)cl2[m1[k]] + 1;
        idx_out[3 * k + 2] = (uint32_t)cr2[m1[k]] + 1;
    }
    free(old_idx); free(cl); free(cr); free(m1); free(m2); free(tmp); free(all); free(cl2); free(cr2);
    return nlast;
}

/* ======================================================================= */
/* triangulate: DLT, null vector by one-sided Jacobi SVD (Hestenes)         */
/* ======================================================================= */
static void dlt_point(float u1f, float v1f, float u2f, float v2f, const double* P1, const double* P2, double X[3])
{
    double u1 = u1f, v1 = v1f, u2 = u2f, v2 = v2f;
    double A[4][4];   /* A[row][col] */
    for (int c = 0; c < 4; ++c) {
        A[0][c] = u1 * P1[8 + c] - P1[c];
        A[1][c] = v1 * P1[8 + c] - P1[4 + c];
        A[2][c] = u2 * P2[8 + c] - P2[c];
        A[3][c] = v2 * P2[8 + c] - P2[4 + c];
    }
    double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    for (int sweep = 0; sweep < 30; ++sweep) {
        int rotated = 0;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) {
                double al = 0, be = 0, ga = 0;
                for (int i = 0; i < 4; ++i) {
                    al = al + A[i][p] * A[i][p];
                    be = be + A[i][q] * A[i][q];
                    ga = ga + A[i][p] * A[i][q];
                }
                if (ga == 0.0 || fabs(ga) <= 1e-15 * sqrt(al * be)) continue;
                rotated = 1;
                double zeta = (be - al) / (2.0 * ga);
                double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                double c = 1.0 / sqrt(1.0 + t * t);
                double s = c * t;
                for (int i = 0; i < 4; ++i) {
                    double ap = A[i][p], aq = A[i][q];
                    A[i][p] = c * ap - s * aq;
                    A[i][q] = s * ap + c * aq;
                    double vp = V[i][p], vq = V[i][q];
                    V[i][p] = c * vp - s * vq;
                    V[i][q] = s * vp + c * vq;
                }
            }
        if (!rotated) break;
    }
    int jmin = 0;
    double nmin = 0;
    for (int j = 0; j < 4; ++j) {
        double nj = 0;
        for (int i = 0; i < 4; ++i) nj = nj + A[i][j] * A[i][j];
        if (j == 0 || nj < nmin) { nmin = nj; jmin = j; }
    }
    double w = V[3][jmin];
    /* MATLAB returns single for single inputs: round through float */
    X[0] = (double)(float)(V[0][jmin] / w);
    X[1] = (double)(float)(V[1][jmin] / w);
    X[2] = (double)(float)(V[2][jmin] / w);
}

void oracle_triangulate(const float* x1, const float* x2, int n, const double P1[12],
                        const double P2[12], double* X)
{
    for (int i = 0; i < n; ++i) dlt_point(x1[2 * i], x1[2 * i + 1], x2[2 * i], x2[2 * i + 1], P1, P2, X + 3 * i);
}

/* ======================================================================= */
/* P3P: Grunert's quartic in v = s3/s1, coefficients by polynomial algebra   */
/* ======================================================================= */
static double peval(const double* a, int deg, double x)
{
    double r = a[deg];
    for (int i = deg - 1; i >= 0; --i) r = r * x + a[i];
    return r;
}

/* real roots of sum a[i] x^i (deg <= 4), ascending; deterministic
 * recursive-derivative bracketing + bisection. */
static int real_roots(const double* a_in, int deg, double* roots)
{
    double a[5];
    for (int i = 0; i <= deg; ++i) a[i] = a_in[i];
    /* drop negligible leading coefficients */
    double amax = 0;
    for (int i = 0; i <= deg; ++i) if (fabs(a[i]) > amax) amax = fabs(a[i]);
    if (amax == 0.0) return 0;
    while (deg > 0 && fabs(a[deg]) <= 1e-14 * amax) deg--;
    if (deg == 0) return 0;
    if (deg == 1) { roots[0] = -a[0] / a[1]; return 1; }
    if (deg == 2) {
        double disc = a[1] * a[1] - 4.0 * a[2] * a[0];
        if (disc < 0) return 0;
        double sq = sqrt(disc);
        double q = -0.5 * (a[1] + (a[1] >= 0 ? sq : -sq));
        double r1 = q / a[2], r2 = (q != 0.0) ? a[0] / q : r1;
        if (r1 <= r2) { roots[0] = r1; roots[1] = r2; } else { roots[0] = r2; roots[1] = r1; }
        return 2;
    }
    double d[4] = {0, 0, 0, 0};
    for (int i = 1; i <= deg; ++i) d[i - 1] = a[i] * (double)i;
    double crit[4];
    int nc = real_roots(d, deg - 1, crit);
    /* Cauchy bound */
    double B = 0;
    for (int i = 0; i < deg; ++i) { double t = fabs(a[i] / a[deg]); if (t > B) B = t; }
    B = B + 1.0;
    double pts[6];
    int np = 0;
    pts[np++] = -B;
    for (int i = 0; i < nc; ++i) if (crit[i] > -B && crit[i] < B) pts[np++] = crit[i];
    pts[np++] = B;
    int nr = 0;
    for (int k = 0; k + 1 < np; ++k) {
        double lo = pts[k], hi = pts[k + 1];
        double flo = peval(a, deg, lo), fhi = peval(a, deg, hi);
        if (flo == 0.0) { if (nr == 0 || roots[nr - 1] != lo) roots[nr++] = lo; continue; }
        if ((flo < 0) == (fhi < 0)) continue;
        for (int it = 0; it < 200; ++it) {
            double mid = 0.5 * (lo + hi);
            if (mid <= lo || mid >= hi) break;
            double fm = peval(a, deg, mid);
            if (fm == 0.0) { lo = hi = mid; break; }
            if ((fm < 0) == (flo < 0)) { lo = mid; flo = fm; } else hi = mid;
        }
        roots[nr++] = 0.5 * (lo + hi);
    }
    return nr;
}

static void pmul(const double* a, int da, const double* b, int db, double* out)
{
    for (int i = 0; i <= da + db; ++i) out[i] = 0.0;
    for (int i = 0; i <= da; ++i)
        for (int j = 0; j <= db; ++j) out[i + j] = out[i + j] + a[i] * b[j];
}

static void bearing(const double K[9], double u, double v, double f[3])
{
    double yn = (v - K[5]) / K[4];
    double xn = (u - K[2] - K[1] * yn) / K[0];
    double n = sqrt(xn * xn + yn * yn + 1.0);
    f[0] = xn / n; f[1] = yn / n; f[2] = 1.0 / n;
}

static void cross3(const double* a, const double* b, double* c)
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

static int normalize3(double* a)
{
    double n = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    if (!(n > 0)) return 0;
    a[0] = a[0] / n; a[1] = a[1] / n; a[2] = a[2] / n;
    return 1;
}

/* rotation R (row-major) and t with Pc = R Pw + t from 3 congruent points */
static int align3(const double Pw[3][3], const double Pc[3][3], double R[9], double t[3])
{
    double ew[3][3], ec[3][3];   /* ew[k] = k-th basis vector */
    double d1[3], d2[3];
    for (int i = 0; i < 3; ++i) { ew[0][i] = Pw[1][i] - Pw[0][i]; d1[i] = Pw[2][i] - Pw[0][i]; }
    if (!normalize3(ew[0])) return 0;
    cross3(ew[0], d1, ew[2]);
    if (!normalize3(ew[2])) return 0;
    cross3(ew[2], ew[0], ew[1]);
    for (int i = 0; i < 3; ++i) { ec[0][i] = Pc[1][i] - Pc[0][i]; d2[i] = Pc[2][i] - Pc[0][i]; }
    if (!normalize3(ec[0])) return 0;
    cross3(ec[0], d2, ec[2]);
    if (!normalize3(ec[2])) return 0;
    cross3(ec[2], ec[0], ec[1]);
    /* R = Ec * Ew^T : R[i][j] = sum_k ec[k][i] * ew[k][j] */
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[3 * i + j] = ec[0][i] * ew[0][j] + ec[1][i] * ew[1][j] + ec[2][i] * ew[2][j];
    double mw[3], mc[3];
    for (int i = 0; i < 3; ++i) {
        mw[i] = (Pw[0][i] + Pw[1][i] + Pw[2][i]) / 3.0;
        mc[i] = (Pc[0][i] + Pc[1][i] + Pc[2][i]) / 3.0;
    }
    for (int i = 0; i < 3; ++i) t[i] = mc[i] - (R[3 * i] * mw[0] + R[3 * i + 1] * mw[1] + R[3 * i + 2] * mw[2]);
    return 1;
}

int oracle_p3p(const double img[3][2], const double world[3][3], const double K[9],
               double Rs[4][9], double ts[4][3])
{
    double j[3][3];
    for (int i = 0; i < 3; ++i) bearing(K, img[i][0], img[i][1], j[i]);
    double dv[3];
    for (int i = 0; i < 3; ++i) dv[i] = world[1][i] - world[2][i];
    double a2 = dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2];
    for (int i = 0; i < 3; ++i) dv[i] = world[0][i] - world[2][i];
    double b2 = dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2];
    for (int i = 0; i < 3; ++i) dv[i] = world[0][i] - world[1][i];
    double c2 = dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2];
    if (!(a2 > 0 && b2 > 0 && c2 > 0)) return 0;
    double ca = j[1][0] * j[2][0] + j[1][1] * j[2][1] + j[1][2] * j[2][2];  /* cos alpha: rays 2,3 */
    double cb = j[0][0] * j[2][0] + j[0][1] * j[2][1] + j[0][2] * j[2][2];  /* cos beta:  rays 1,3 */
    double cg = j[0][0] * j[1][0] + j[0][1] * j[1][1] + j[0][2] * j[1][2];  /* cos gamma: rays 1,2 */
    double Kq = (a2 - c2) / b2, cb2 = c2 / b2;
    /* u = N(v)/D(v); quartic = D^2 + N^2 - 2 cg N D - (c2/b2) Q D^2 */
    double N[3] = {1.0 + Kq, -2.0 * Kq * cb, Kq - 1.0};
    double D[2] = {2.0 * cg, -2.0 * ca};
    double Q[3] = {1.0, -2.0 * cb, 1.0};
    double DD[3], NN[5], ND[4], QDD[5];
    pmul(D, 1, D, 1, DD);
    pmul(N, 2, N, 2, NN);
    pmul(N, 2, D, 1, ND);
    pmul(Q, 2, DD, 2, QDD);
    double P[5];
    for (int i = 0; i < 5; ++i) {
        double v = NN[i] - cb2 * QDD[i];
        if (i < 3) v = v + DD[i];
        if (i < 4) v = v - 2.0 * cg * ND[i];
        P[i] = v;
    }
    double roots[4];
    int nr = real_roots(P, 4, roots);
    int ns = 0;
    for (int k = 0; k < nr; ++k) {
        double v = roots[k];
        if (!(v > 0)) continue;
        double Dv = D[0] + D[1] * v;
        if (Dv == 0.0) continue;
        double u = (N[0] + N[1] * v + N[2] * v * v) / Dv;
        if (!(u > 0)) continue;
        double Qv = Q[0] + Q[1] * v + Q[2] * v * v;
        if (!(Qv > 0)) continue;
        double s1 = sqrt(b2 / Qv), s2 = u * s1, s3 = v * s1;
        double Pc[3][3];
        for (int i = 0; i < 3; ++i) { Pc[0][i] = s1 * j[0][i]; Pc[1][i] = s2 * j[1][i]; Pc[2][i] = s3 * j[2][i]; }
        if (align3(world, Pc, Rs[ns], ts[ns])) ns++;
        if (ns == 4) break;
    }
    return ns;
}

/* ======================================================================= */
/* estworldpose: P3P + MSAC                                 */
/* ======================================================================= */
static double reproj_err2(const double R[9], const double t[3], const double K[9], const double* X, const double* uv)
{
    double xc = R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + t[0];
    double yc = R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + t[1];
    double zc = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + t[2];
    if (!(zc > 0)) return INFINITY;
    double xn = xc / zc, yn = yc / zc;
    double u = K[0] * xn + K[1] * yn + K[2];
    double v = K[4] * yn + K[5];
    double du = u - uv[0], dv = v - uv[1];
    return du * du + dv * dv;
}

/* sample 4 distinct indices for slot s; returns 0 if none found */
static int msac_sample(uint32_t seed, uint32_t frame_key, uint32_t s, uint32_t n, uint32_t idx[4])
{
    for (uint32_t att = 0; att < 16; ++att) {
        vo_u32x4 c = {{s, att, frame_key, 0x5EEDu}};
        vo_u32x4 r = vo_philox4x32_10(c, seed, 0x9E3779B9u);
        for (int q = 0; q < 4; ++q) idx[q] = vo_rand_index(r.v[q], n);
        if (idx[0] != idx[1] && idx[0] != idx[2] && idx[0] != idx[3] && idx[1] != idx[2] && idx[1] != idx[3] && idx[2] != idx[3])
            return 1;
    }
    return 0;
}

/* one hypothesis slot: returns 1 if valid (R,t filled) */
static int msac_hypothesis(const double* img, const double* world, int n, const double K[9], uint32_t seed,
                           uint32_t frame_key, uint32_t s, double R[9], double t[3])
{
    uint32_t idx[4];
    if (!msac_sample(seed, frame_key, s, (uint32_t)n, idx)) return 0;
    double im3[3][2], w3[3][3];
    for (int q = 0; q < 3; ++q) {
        im3[q][0] = img[2 * idx[q]]; im3[q][1] = img[2 * idx[q] + 1];
        for (int i = 0; i < 3; ++i) w3[q][i] = world[3 * idx[q] + i];
    }
    double Rs[4][9], ts[4][3];
    int ns = oracle_p3p(im3, w3, K, Rs, ts);
    int best = -1;
    double be = INFINITY;
    for (int k = 0; k < ns; ++k) {
        double e = reproj_err2(Rs[k], ts[k], K, world + 3 * idx[3], img + 2 * idx[3]);
        if (e < be) { be = e; best = k; }
    }
    if (best < 0) return 0;
    memcpy(R, Rs[best], sizeof(double) * 9);
    memcpy(t, ts[best], sizeof(double) * 3);
    return 1;
}

/* MSAC score: 64 lane-strided partial sums + pairwise tree */
static double msac_score(const double R[9], const double t[3], const double* img, const double* world, int n,
                         const double K[9], double thr, int* n_in)
{
    double part[64];
    int cnt = 0;
    for (int l = 0; l < 64; ++l) part[l] = 0.0;
    for (int k = 0; k < n; ++k) {
        double e = reproj_err2(R, t, K, world + 3 * k, img + 2 * k);
        if (e < thr) cnt++;
        part[k & 63] = part[k & 63] + (e < thr ? e : thr);
    }
    for (int off = 32; off >= 1; off >>= 1)
        for (int l = 0; l < off; ++l) part[l] = part[l] + part[l + off];
    *n_in = cnt;
    return part[0];
}

int msac_trials_needed(int n_in, int n, double conf)
{
    double w = (double)n_in / (double)n;
    double w4 = w * w * w * w;
    if (!(w4 > 1e-300)) return 0x7fffffff;
    double den = vo_log_d(1.0 - w4);
    if (!(den < 0)) return 1;
    double num = vo_log_d(1.0 - conf);
    double N = ceil(num / den);
    if (N > 2147483647.0) return 0x7fffffff;
    if (N < 1.0) return 1;
    return (int)N;
}

int oracle_estworldpose(const double* img, const double* world, int n, const double K[9],
                        const vo_ransac_params* p, uint32_t frame_key, double T[16],
                        uint8_t* inliers, int* n_inliers)
{
    if (n_inliers) *n_inliers = 0;
    if (n < 4) return VO_ERR_TOO_FEW_POINTS;
    const double thr = p->max_reprojection_error * p->max_reprojection_error;
    const double conf = p->confidence / 100.0;
    int num_trials = p->max_num_trials;
    int trials = 0;
    double best_score = INFINITY, bR[9], bt[3];
    int have = 0, best_in = 0;
    for (int s = 0; s < p->max_num_trials && trials < num_trials; ++s) {
        double R[9], t[3];
        if (!msac_hypothesis(img, world, n, K, p->seed, frame_key, (uint32_t)s, R, t)) continue;
        trials++;
        int nin;
        double sc = msac_score(R, t, img, world, n, K, thr, &nin);
        if (sc < best_score) {
            best_score = sc; have = 1; best_in = nin;
            memcpy(bR, R, sizeof(bR)); memcpy(bt, t, sizeof(bt));
            int need = msac_trials_needed(nin, n, conf);
            if (need < num_trials) num_trials = need;
        }
    }
    if (!have || best_in < 4) return VO_ERR_NO_CONSENSUS;
    int cnt = 0;
    for (int k = 0; k < n; ++k) {
        double e = reproj_err2(bR, bt, K, world + 3 * k, img + 2 * k);
        int in = e < thr;
        if (inliers) inliers[k] = (uint8_t)in;
        cnt += in;
    }
    if (n_inliers) *n_inliers = cnt;
    /* camera pose in world: [R^T, -R^T t; 0 0 0 1] */
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) T[4 * i + j] = bR[3 * j + i];
        T[4 * i + 3] = -(bR[i] * bt[0] + bR[3 + i] * bt[1] + bR[6 + i] * bt[2]);
    }
    T[12] = 0; T[13] = 0; T[14] = 0; T[15] = 1;
    return VO_OK;
}

/* ======================================================================= */
/* landmarks: VO.m:145-160 + CreateLandmarksFromFeatures.m                  */
/* ======================================================================= */
/* CreateLandmarksFromFeatures.m:1-16 in the camera frame: X[rows][3] (the triangulated
 * point, single-rounded as dlt_point returns it) and keep[rows] (0 = zero row).  Returns
 * rows; only min(rows, capacity) are written. */
int oracle_landmark_rows(const float* l_pos, const float* r_pos, int S, const float* old_l,
                         const float* old_r, int K, const double P1[12], const double P2[12],
                         float* X_out, uint8_t* keep, int capacity)
{
    int* idx = (int*)malloc(sizeof(int) * (S + 1));
    int M = 0;
    for (int j = 0; j < S; ++j) {
        int hit = 0;
        for (int k = 0; k < K && !hit; ++k)
            if (old_l[2 * k] == l_pos[2 * j] || old_l[2 * k + 1] == l_pos[2 * j + 1]) hit = 1;
        for (int k = 0; k < K && !hit; ++k)
            if (old_r[2 * k] == r_pos[2 * j] || old_r[2 * k + 1] == r_pos[2 * j + 1]) hit = 1;
        if (!hit) idx[M++] = j;
    }
    /* landmarks = zeros(size(features_l,2),3) -> 2 rows; grows to last kept odd i */
    int rows = 2;
    for (int r = 0; r < 2 && r < capacity; ++r) { keep[r] = 0; X_out[3 * r] = X_out[3 * r + 1] = X_out[3 * r + 2] = 0.0f; }
    for (int i = 0; i < M; i += 2) {   /* 1-based odd i <-> 0-based even */
        double X[3];
        dlt_point(l_pos[2 * idx[i]], l_pos[2 * idx[i] + 1], r_pos[2 * idx[i]], r_pos[2 * idx[i] + 1], P1, P2, X);
        if (X[2] < 0) continue;
        if (X[2] > 80) continue;
        for (int r = rows; r < i + 1 && r < capacity; ++r) { keep[r] = 0; X_out[3 * r] = X_out[3 * r + 1] = X_out[3 * r + 2] = 0.0f; }
        if (i + 1 > rows) rows = i + 1;
        if (i < capacity) {
            keep[i] = 1;
            for (int a = 0; a < 3; ++a) X_out[3 * i + a] = (float)X[a];
        }
    }
    free(idx);
    return rows;
}

/* CreateLandmarksFromFeatures.m:17: world = single(pose * [X; 1]) for kept rows. */
void oracle_landmarks_to_world(const double pose[16], const float* X, const uint8_t* keep, int n, double* out)
{
    for (int m = 0; m < n; ++m)
        for (int a = 0; a < 3; ++a) {
            if (!keep[m]) { out[3 * m + a] = 0.0; continue; }
            const double x0 = X[3 * m], x1 = X[3 * m + 1], x2 = X[3 * m + 2];
            double w = pose[4 * a] * x0 + pose[4 * a + 1] * x1 + pose[4 * a + 2] * x2 + pose[4 * a + 3];
            out[3 * m + a] = (double)(float)w;
        }
}

int oracle_landmarks(const float* l_pos, const float* r_pos, int S, const float* old_l,
                     const float* old_r, int K, const double P1[12], const double P2[12],
                     const double pose[16], double* out, int capacity)
{
    int cap = S + 2;
    float* X = (float*)malloc(sizeof(float) * 3 * cap);
    uint8_t* keep = (uint8_t*)malloc(cap);
    int rows = oracle_landmark_rows(l_pos, r_pos, S, old_l, old_r, K, P1, P2, X, keep, cap);
    if (out) oracle_landmarks_to_world(pose, X, keep, rows < capacity ? rows : capacity, out);
    free(X);
    free(keep);
    return rows;
}

/* ======================================================================= */
/* the loop: VO.m:64-232                                                    */
/* ======================================================================= */
static void mat4_mul(const double* A, const double* B, double* C)
{
    double T[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            T[4 * i + j] = A[4 * i] * B[j] + A[4 * i + 1] * B[4 + j] + A[4 * i + 2] * B[8 + j] + A[4 * i + 3] * B[12 + j];
    memcpy(C, T, sizeof(T));
}

static const double I4[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};

long oracle_run_sequence(const uint8_t* lefts, const uint8_t* rights, int F, int rows, int cols,
                         const vo_calib* calib, const vo_sift_params* sp, const vo_match_params* mp,
                         const vo_ransac_params* rp, vo_step_out* outs, double* lm_out, long lm_cap,
                         uint32_t key0, float* lm_cam_X, uint8_t* lm_cam_keep)
{
    int cap = sp->max_keypoints;
    vo_keypoint *kl = malloc(sizeof(vo_keypoint) * cap), *kr = malloc(sizeof(vo_keypoint) * cap);
    uint8_t *dl = malloc((size_t)cap * 128), *dr = malloc((size_t)cap * 128);
    /* features state (stereo subset of previous frame) */
    float *fl_pos = malloc(sizeof(float) * 2 * cap), *fr_pos = malloc(sizeof(float) * 2 * cap);
    uint8_t *fl_desc = malloc((size_t)cap * 128), *fr_desc = malloc((size_t)cap * 128);
    int nf = 0, have_features = 0;
    uint32_t* pairs = malloc(sizeof(uint32_t) * 2 * cap);
    uint32_t* tidx = malloc(sizeof(uint32_t) * 3 * cap);
    double *img = malloc(sizeof(double) * 2 * cap), *wld = malloc(sizeof(double) * 3 * cap);
    float *ol = malloc(sizeof(float) * 2 * cap), *orr = malloc(sizeof(float) * 2 * cap);
    float *sl = malloc(sizeof(float) * 2 * cap), *sr = malloc(sizeof(float) * 2 * cap);
    double pose[16];
    memcpy(pose, I4, sizeof(pose));
    long lm_rows = 0;
    size_t fsz = (size_t)rows * cols;
    for (int f = 0; f < F; ++f) {
        vo_step_out* o = &outs[f];
        memset(o, 0, sizeof(*o));
        int nl = oracle_sift(lefts + f * fsz, rows, cols, cols, sp, kl, dl, cap);
        int nr = oracle_sift(rights + f * fsz, rows, cols, cols, sp, kr, dr, cap);
        if (nl > cap) nl = cap;
        if (nr > cap) nr = cap;
        int S = oracle_match(dl, nl, dr, nr, mp, pairs, cap);
        o->n_left = nl; o->n_right = nr; o->n_stereo = S;
        memcpy(o->rel_pose, I4, sizeof(I4));
        /* stereo subset (VO.m:141-144 / 207-210) */
        for (int k = 0; k < S; ++k) {
            int a = (int)pairs[2 * k] - 1, b = (int)pairs[2 * k + 1] - 1;
            sl[2 * k] = kl[a].x; sl[2 * k + 1] = kl[a].y;
            sr[2 * k] = kr[b].x; sr[2 * k + 1] = kr[b].y;
        }
        if (have_features) {
            int Kt = oracle_track(fl_desc, fr_desc, nf, dl, nl, dr, nr, mp, tidx, cap);
            o->n_tracked = Kt;
            for (int k = 0; k < Kt; ++k) {
                int oi = (int)tidx[3 * k] - 1, ci = (int)tidx[3 * k + 1] - 1;
                ol[2 * k] = fl_pos[2 * oi]; ol[2 * k + 1] = fl_pos[2 * oi + 1];
                orr[2 * k] = fr_pos[2 * oi]; orr[2 * k + 1] = fr_pos[2 * oi + 1];
                img[2 * k] = kl[ci].x; img[2 * k + 1] = kl[ci].y;
            }
            oracle_triangulate(ol, orr, Kt, calib->P1, calib->P2, wld);
            double T[16];
            int nin = 0;
            int st = oracle_estworldpose(img, wld, Kt, calib->K, rp, key0 + (uint32_t)f, T, NULL, &nin);
            o->status = st;
            o->n_inliers = nin;
            if (st == VO_OK) {
                memcpy(o->rel_pose, T, sizeof(T));
                mat4_mul(pose, T, pose);
            }
            long room = lm_cap - lm_rows;
            int room_i = room > 0 ? (int)(room < 0x7fffffff ? room : 0x7fffffff) : 0;
            int rows_added;
            if (lm_cam_X)        /* camera-frame rows for a sharded run (world transform after the chain) */
                rows_added = oracle_landmark_rows(sl, sr, S, ol, orr, Kt, calib->P1, calib->P2,
                                                  lm_cam_X + 3 * lm_rows, lm_cam_keep + lm_rows, room_i);
            else
                rows_added = oracle_landmarks(sl, sr, S, ol, orr, Kt, calib->P1, calib->P2, pose,
                                              lm_out ? lm_out + 3 * lm_rows : NULL, room_i);
            o->n_landmarks = rows_added;
            lm_rows += rows_added;
        }
        memcpy(o->pose, pose, sizeof(pose));
        /* features = stereo subset (VO.m:225-230) */
        for (int k = 0; k < S; ++k) {
            int a = (int)pairs[2 * k] - 1, b = (int)pairs[2 * k + 1] - 1;
            fl_pos[2 * k] = sl[2 * k]; fl_pos[2 * k + 1] = sl[2 * k + 1];
            fr_pos[2 * k] = sr[2 * k]; fr_pos[2 * k + 1] = sr[2 * k + 1];
            memcpy(fl_desc + (size_t)k * 128, dl + (size_t)a * 128, 128);
            memcpy(fr_desc + (size_t)k * 128, dr + (size_t)b * 128, 128);
        }
        nf = S;
        have_features = 1;
    }
    free(kl); free(kr); free(dl); free(dr); free(fl_pos); free(fr_pos); free(fl_desc); free(fr_desc);
    free(pairs); free(tidx); free(img); free(wld); free(ol); free(orr); free(sl); free(sr);
    return lm_rows;
}

int oracle_sift_match_pair(const uint8_t* left, const uint8_t* right, int rows, int cols,
                           const vo_sift_params* sp, const vo_match_params* mp,
                           int* n_left, int* n_right)
{
    int cap = sp->max_keypoints;
    vo_keypoint *kl = malloc(sizeof(vo_keypoint) * cap), *kr = malloc(sizeof(vo_keypoint) * cap);
    uint8_t *dl = malloc((size_t)cap * 128), *dr = malloc((size_t)cap * 128);
    uint32_t* pairs = malloc(sizeof(uint32_t) * 2 * cap);
    int nl = oracle_sift(left, rows, cols, cols, sp, kl, dl, cap);
    int nr = oracle_sift(right, rows, cols, cols, sp, kr, dr, cap);
    if (nl > cap) nl = cap;
    if (nr > cap) nr = cap;
    int S = oracle_match(dl, nl, dr, nr, mp, pairs, cap);
    if (n_left) *n_left = nl;
    if (n_right) *n_right = nr;
    free(kl); free(kr); free(dl); free(dr); free(pairs);
    return S;
}
