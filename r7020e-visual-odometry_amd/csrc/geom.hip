// geom.hip — tracking + geometry stages of the per-frame path (see vo_geom.h).
//
//   find_remaining_points (VO.m:280-334)  four match jobs per frame whose row
//       sets are index lists; k_compose turns each step's (i, j) pairs into the
//       next step's lists, so no descriptor is ever copied.
//   triangulate (VO.m:113-116)            k_gather_tri: one lane per tracked
//       point, linear DLT + one-sided Jacobi SVD in f64 (oracle dlt_point).
//   estworldpose (VO.m:123-127)           k_msac: one block per frame walks the
//       hypothesis slots in chunks of 64 -- a lane per slot (Philox sample,
//       Grunert P3P, 4th-point disambiguation), a wave per slot score
//       (lane-strided partial MSAC sums + fixed shuffle tree), then the
//       sequential adaptive-termination replay of the chunk -- until the replay
//       stops; msac_final: inlier mask + camera pose.  (The eager kernels
//       k_msac_hyp / k_msac_score / k_msac_select score every slot first; they
//       are compiled only into the test build libvo_exp.so, VO_EXPERIMENTAL.)
//   landmarks (VO.m:145-160, CreateLandmarksFromFeatures.m)  k_stereo_pos,
//       k_lm_filter (any-x-or-y equality test, quirk Q3) + block compaction,
//       k_lm_tri (odd rows, z gates).  (One fused block per frame measured
//       3.5x slower: 0.27 vs 0.075 ms per batch for positions + filter.)  The world transform needs the chained pose and runs
//       on the host after the 4x4 chain.
// Float/double expressions mirror oracle/vo_ref.c operation for operation.
#include "vo_geom.h"
#include <cstring>
#include <cstdlib>

namespace vo {

hipError_t geom_alloc(GeomBuffers& g, int max_frames, int kp_cap, int n_hyp)
{
    g.max_frames = max_frames; g.kp_cap = kp_cap; g.n_hyp = n_hyp;
    const size_t F = max_frames, K = kp_cap;
    hipError_t e;
#define GA(ptr, bytes) do { e = hipMalloc((void**)&(ptr), (bytes)); if (e != hipSuccess) return e; } while (0)
    GA(g.lists, sizeof(int) * F * TL_COUNT * K);
    GA(g.list_n, sizeof(int) * F * 4);
    GA(g.step_i, sizeof(int) * 4 * F * K);
    GA(g.step_j, sizeof(int) * 4 * F * K);
    GA(g.step_n, sizeof(int) * 4 * F);
    GA(g.world, sizeof(double) * F * K * 3);
    GA(g.imgpt, sizeof(double) * F * K * 2);
    GA(g.oldpos, sizeof(float) * F * K * 4);
    GA(g.inliers, F * K);
    GA(g.hyp, sizeof(MsacHyp) * F * n_hyp);
    GA(g.fg, sizeof(FrameGeom) * F);
    GA(g.spos, sizeof(float) * F * K * 4);
    GA(g.s_n, sizeof(int) * F);
    GA(g.lm_new, sizeof(int) * F * K);
    GA(g.lm_M, sizeof(int) * F);
    GA(g.lm_X, sizeof(float) * F * K * 3);
    GA(g.lm_keep, F * K);
    GA(g.lm_rows, sizeof(int) * F);
#undef GA
    e = hipMemset(g.step_n, 0, sizeof(int) * 4 * F);
    if (e != hipSuccess) return e;
    return hipMemset(g.list_n, 0, sizeof(int) * 4 * F);
}

void geom_free(GeomBuffers& g)
{
    void* bufs[] = {g.lists, g.list_n, g.step_i, g.step_j, g.step_n, g.world, g.imgpt, g.oldpos, g.inliers, g.hyp,
                    g.fg, g.spos, g.s_n, g.lm_new, g.lm_M, g.lm_X, g.lm_keep, g.lm_rows};
    for (void* p : bufs) (void)hipFree(p);   // teardown: nothing to report to
    g = GeomBuffers();
}

static inline int* glist(const GeomBuffers& g, int f, int l) { return g.lists + ((size_t)f * TL_COUNT + l) * g.kp_cap; }

void geom_fill_track_jobs(const GeomBuffers& g, MatchJob* jobs, int M, int first, const SiftBuffers& sb,
                          int* pair_i, int* pair_j, int* pair_n, int kp_cap)
{
    const size_t ds = (size_t)kp_cap * VO_DESC_LEN;
    auto D = [&](int slot) { return (const uint8_t*)(sb.desc + slot * ds); };
    auto Mt = [&](int slot) { return (const DescMeta*)(sb.meta + (size_t)slot * kp_cap); };
    for (int f = 0; f < M; ++f) {
        const int cl = 2 * f, cr = 2 * f + 1;
        const int pl = f ? 2 * (f - 1) : 2 * M, pr = pl + 1;
        const int pp = f ? f - 1 : M;
        for (int s = 0; s < 4; ++s) {
            MatchJob& J = jobs[first + s * M + f];
            memset(&J, 0, sizeof(J));
            J.out_i = g.step_i + ((size_t)s * M + f) * kp_cap;
            J.out_j = g.step_j + ((size_t)s * M + f) * kp_cap;
            J.out_n = g.step_n + s * M + f;
            J.cap = kp_cap;
        }
        // step 0: lm = matchFeatures(cur.l_desc, old.l_desc)            VO.m:283
        MatchJob& J0 = jobs[first + 0 * M + f];
        J0.d1 = D(cl); J0.m1 = Mt(cl); J0.idx1 = nullptr; J0.n1 = sb.n_kp + cl;
        J0.d2 = D(pl); J0.m2 = Mt(pl); J0.idx2 = pair_i + (size_t)pp * kp_cap; J0.n2 = pair_n + pp;
        // step 1: rm = matchFeatures(cur.r_desc, old.r_desc)            VO.m:293
        MatchJob& J1 = jobs[first + 1 * M + f];
        J1.d1 = D(cr); J1.m1 = Mt(cr); J1.idx1 = nullptr; J1.n1 = sb.n_kp + cr;
        J1.d2 = D(pr); J1.m2 = Mt(pr); J1.idx2 = glist(g, f, TL_OR1); J1.n2 = g.list_n + 4 * f + 0;
        // step 2: cm = matchFeatures(cur.l_desc, cur.r_desc)            VO.m:311
        MatchJob& J2 = jobs[first + 2 * M + f];
        J2.d1 = D(cl); J2.m1 = Mt(cl); J2.idx1 = glist(g, f, TL_CL); J2.n1 = g.list_n + 4 * f + 0;
        J2.d2 = D(cr); J2.m2 = Mt(cr); J2.idx2 = glist(g, f, TL_CR); J2.n2 = g.list_n + 4 * f + 1;
        // step 3: last = matchFeatures(cur.l_desc, old.l_desc)          VO.m:323
        MatchJob& J3 = jobs[first + 3 * M + f];
        J3.d1 = D(cl); J3.m1 = Mt(cl); J3.idx1 = glist(g, f, TL_CL2); J3.n1 = g.list_n + 4 * f + 2;
        J3.d2 = D(pl); J3.m2 = Mt(pl); J3.idx2 = glist(g, f, TL_OL2); J3.n2 = g.list_n + 4 * f + 1;
    }
}

// ---------------------------------------------------------------------------
// index composition after each tracking step (VO.m:287-290,297-300,305-308,
// 314-317,326-333).  grid (blocks, B)
// ---------------------------------------------------------------------------
struct ComposeArgs {
    int* lists; int* list_n; const int* step_i; const int* step_j; const int* step_n;
    const int* pair_i; const int* pair_j; const int* pair_n;
    int M, kp_cap, step;
};

__global__ void k_compose(ComposeArgs a)
{
    const int f = blockIdx.y, K = a.kp_cap, M = a.M;
    const int s = a.step;
    int n = a.step_n[s * M + f];
    if (n > K) n = K;
    if (n < 0) n = 0;
    const int* si = a.step_i + ((size_t)s * M + f) * K;
    const int* sj = a.step_j + ((size_t)s * M + f) * K;
    int* L = a.lists + (size_t)f * TL_COUNT * K;
    const int pp = f ? f - 1 : M;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const int i = si[k], j = sj[k];
        if (s == 0) {
            L[TL_OL1 * K + k] = a.pair_i[(size_t)pp * K + j];
            L[TL_OR1 * K + k] = a.pair_j[(size_t)pp * K + j];
            L[TL_CL * K + k] = i;
        } else if (s == 1) {
            L[TL_OL2 * K + k] = L[TL_OL1 * K + j];
            L[TL_OR2 * K + k] = L[TL_OR1 * K + j];
            L[TL_CR * K + k] = i;
        } else if (s == 2) {
            L[TL_CL2 * K + k] = L[TL_CL * K + i];
            L[TL_CR2 * K + k] = L[TL_CR * K + j];
        } else {
            L[TL_OLF * K + k] = L[TL_OL2 * K + j];
            L[TL_ORF * K + k] = L[TL_OR2 * K + j];
            L[TL_CLF * K + k] = L[TL_CL2 * K + i];
            L[TL_CRF * K + k] = L[TL_CR2 * K + i];
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) a.list_n[4 * f + s] = n;
}

// ---------------------------------------------------------------------------
// DLT triangulation (oracle dlt_point)
// ---------------------------------------------------------------------------
__device__ void dlt_point_dev(float u1f, float v1f, float u2f, float v2f, const double* P1, const double* P2, double X[3])
{
    double u1 = u1f, v1 = v1f, u2 = u2f, v2 = v2f;
    double A[4][4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        A[0][c] = u1 * P1[8 + c] - P1[c];
        A[1][c] = v1 * P1[8 + c] - P1[4 + c];
        A[2][c] = u2 * P2[8 + c] - P2[c];
        A[3][c] = v2 * P2[8 + c] - P2[4 + c];
    }
    double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    for (int sweep = 0; sweep < 30; ++sweep) {
        int rotated = 0;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int q = p + 1; q < 4; ++q) {
                double al = 0, be = 0, ga = 0;
#pragma unroll
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
#pragma unroll
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
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        double nj = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) nj = nj + A[i][j] * A[i][j];
        if (j == 0 || nj < nmin) { nmin = nj; jmin = j; }
    }
    double v0 = 0, v1_ = 0, v2_ = 0, w = 1;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (j == jmin) { v0 = V[0][j]; v1_ = V[1][j]; v2_ = V[2][j]; w = V[3][j]; }
    X[0] = (double)(float)(v0 / w);
    X[1] = (double)(float)(v1_ / w);
    X[2] = (double)(float)(v2_ / w);
}

struct CalibDev { double P1[12], P2[12], K[9]; };

// gather tracked positions and triangulate the old stereo pair. grid (blocks, B)
__global__ void k_gather_tri(const vo_keypoint* __restrict__ kp, int kp_cap, const int* __restrict__ lists,
                             const int* __restrict__ list_n, float* __restrict__ oldpos, double* __restrict__ imgpt,
                             double* __restrict__ world, int M, CalibDev cal)
{
    const int f = blockIdx.y, K = kp_cap;
    int n = list_n[4 * f + 3];
    const int cl = 2 * f;
    const int pl = f ? 2 * (f - 1) : 2 * M, pr = pl + 1;
    const int* L = lists + (size_t)f * TL_COUNT * K;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const vo_keypoint ol = kp[(size_t)pl * K + L[TL_OLF * K + k]];
        const vo_keypoint orr = kp[(size_t)pr * K + L[TL_ORF * K + k]];
        const vo_keypoint cu = kp[(size_t)cl * K + L[TL_CLF * K + k]];
        float* op = oldpos + ((size_t)f * K + k) * 4;
        op[0] = ol.x; op[1] = ol.y; op[2] = orr.x; op[3] = orr.y;
        double* ip = imgpt + ((size_t)f * K + k) * 2;
        ip[0] = cu.x; ip[1] = cu.y;
        double X[3];
        dlt_point_dev(ol.x, ol.y, orr.x, orr.y, cal.P1, cal.P2, X);
        double* w = world + ((size_t)f * K + k) * 3;
        w[0] = X[0]; w[1] = X[1]; w[2] = X[2];
    }
}

// standalone triangulation of position quads (x1, y1, x2, y2)
__global__ void k_tri_list(const float* __restrict__ pos, int n, CalibDev cal, double* __restrict__ X)
{
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        double Y[3];
        dlt_point_dev(pos[4 * k], pos[4 * k + 1], pos[4 * k + 2], pos[4 * k + 3], cal.P1, cal.P2, Y);
        X[3 * k] = Y[0]; X[3 * k + 1] = Y[1]; X[3 * k + 2] = Y[2];
    }
}

// ---------------------------------------------------------------------------
// P3P (oracle_p3p) — Grunert's quartic by polynomial algebra, deterministic
// bracketing/bisection root finder (template recursion = the oracle's).
// ---------------------------------------------------------------------------
// Register-resident form: every array index is a compile-time constant (fixed-degree solvers
// selected by a switch on the trimmed degree, roots appended through select chains), so the
// coefficients, critical points and roots stay in VGPRs -- the dynamically indexed form
// lived in scratch and its bisection loop waited on scratch loads every iteration.  Same
// operations in the same order as the oracle (real_roots, oracle/vo_ref.c:294): the trim
// keeps the largest i >= 1 with !(|a_i| <= 1e-14 amax), Horner as r = r*x + a_i.
template <int D>
__device__ __forceinline__ double peval_fixed(const double* a, double x)
{
    double r = a[D];
#pragma unroll
    for (int i = D - 1; i >= 0; --i) r = r * x + a[i];
    return r;
}

template <int N>
__device__ __forceinline__ void push_root(double* r, int& nr, double v)
{
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (i == nr) r[i] = v;
    nr++;
}

template <int MAXD>
__device__ int real_roots_trim(const double* a, double* roots);

// one bracketed interval: an exact zero at lo, or bisection to adjacent doubles (<= 200 halvings)
template <int D, int N>
__device__ __forceinline__ void bisect_interval(const double* a, double lo, double hi, double* roots, int& nr,
                                                double& last)
{
    double flo = peval_fixed<D>(a, lo), fhi = peval_fixed<D>(a, hi);
    if (flo == 0.0) {
        if (nr == 0 || last != lo) { push_root<N>(roots, nr, lo); last = lo; }
        return;
    }
    if ((flo < 0) == (fhi < 0)) return;
    for (int it = 0; it < 200; ++it) {
        double mid = 0.5 * (lo + hi);
        if (mid <= lo || mid >= hi) break;
        double fm = peval_fixed<D>(a, mid);
        if (fm == 0.0) { lo = hi = mid; break; }
        if ((fm < 0) == (flo < 0)) { lo = mid; flo = fm; } else hi = mid;
    }
    last = 0.5 * (lo + hi);
    push_root<N>(roots, nr, last);
}

// exact degree D >= 3: critical points from the derivative, then one bisection per bracket
template <int D>
__device__ __forceinline__ int real_roots_fixed(const double* a, double* roots)
{
    double d[D];
#pragma unroll
    for (int i = 1; i <= D; ++i) d[i - 1] = a[i] * (double)i;
    double crit[D - 1];
    const int nc = real_roots_trim<D - 1>(d, crit);
    double B = 0;
#pragma unroll
    for (int i = 0; i < D; ++i) { double t = fabs(a[i] / a[D]); if (t > B) B = t; }
    B = B + 1.0;
    int nr = 0;
    double last = 0.0, prev = -B;
#pragma unroll
    for (int k = 0; k < D - 1; ++k) {
        if (k < nc && crit[k] > -B && crit[k] < B) {
            bisect_interval<D, D>(a, prev, crit[k], roots, nr, last);
            prev = crit[k];
        }
    }
    bisect_interval<D, D>(a, prev, B, roots, nr, last);
    return nr;
}

template <int MAXD>
__device__ int real_roots_trim(const double* a, double* roots)
{
    double amax = 0;
#pragma unroll
    for (int i = 0; i <= MAXD; ++i) if (fabs(a[i]) > amax) amax = fabs(a[i]);
    if (amax == 0.0) return 0;
    int deg = 0;
#pragma unroll
    for (int i = 1; i <= MAXD; ++i) if (!(fabs(a[i]) <= 1e-14 * amax)) deg = i;
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
    if constexpr (MAXD >= 4) {
        if (deg == 4) return real_roots_fixed<4>(a, roots);
    }
    if constexpr (MAXD >= 3) {
        return real_roots_fixed<3>(a, roots);
    }
    return 0;
}

__device__ __forceinline__ void pmul_dev(const double* a, int da, const double* b, int db, double* out)
{
    for (int i = 0; i <= da + db; ++i) out[i] = 0.0;
    for (int i = 0; i <= da; ++i)
        for (int j = 0; j <= db; ++j) out[i + j] = out[i + j] + a[i] * b[j];
}

__device__ __forceinline__ void bearing_dev(const double* K, double u, double v, double f[3])
{
    double yn = (v - K[5]) / K[4];
    double xn = (u - K[2] - K[1] * yn) / K[0];
    double n = sqrt(xn * xn + yn * yn + 1.0);
    f[0] = xn / n; f[1] = yn / n; f[2] = 1.0 / n;
}

__device__ __forceinline__ void cross3_dev(const double* a, const double* b, double* c)
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ __forceinline__ int normalize3_dev(double* a)
{
    double n = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    if (!(n > 0)) return 0;
    a[0] = a[0] / n; a[1] = a[1] / n; a[2] = a[2] / n;
    return 1;
}

__device__ int align3_dev(const double Pw[3][3], const double Pc[3][3], double R[9], double t[3])
{
    double ew[3][3], ec[3][3];
    double d1[3], d2[3];
    for (int i = 0; i < 3; ++i) { ew[0][i] = Pw[1][i] - Pw[0][i]; d1[i] = Pw[2][i] - Pw[0][i]; }
    if (!normalize3_dev(ew[0])) return 0;
    cross3_dev(ew[0], d1, ew[2]);
    if (!normalize3_dev(ew[2])) return 0;
    cross3_dev(ew[2], ew[0], ew[1]);
    for (int i = 0; i < 3; ++i) { ec[0][i] = Pc[1][i] - Pc[0][i]; d2[i] = Pc[2][i] - Pc[0][i]; }
    if (!normalize3_dev(ec[0])) return 0;
    cross3_dev(ec[0], d2, ec[2]);
    if (!normalize3_dev(ec[2])) return 0;
    cross3_dev(ec[2], ec[0], ec[1]);
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

__device__ __forceinline__ double reproj_err2_dev(const double R[9], const double t[3], const double* K, const double* X,
                                                  const double* uv)
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

// one P3P + 4th-point selection; returns 1 if valid
__device__ int p3p_hyp_dev(const double im3[3][2], const double w3[3][3], const double* w4, const double* im4,
                           const double* K, double Rb[9], double tb[3])
{
    double j[3][3];
    for (int i = 0; i < 3; ++i) bearing_dev(K, im3[i][0], im3[i][1], j[i]);
    double dv[3];
    for (int i = 0; i < 3; ++i) dv[i] = w3[1][i] - w3[2][i];
    double a2 = dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2];
    for (int i = 0; i < 3; ++i) dv[i] = w3[0][i] - w3[2][i];
    double b2 = dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2];
    for (int i = 0; i < 3; ++i) dv[i] = w3[0][i] - w3[1][i];
    double c2 = dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2];
    if (!(a2 > 0 && b2 > 0 && c2 > 0)) return 0;
    double ca = j[1][0] * j[2][0] + j[1][1] * j[2][1] + j[1][2] * j[2][2];
    double cb = j[0][0] * j[2][0] + j[0][1] * j[2][1] + j[0][2] * j[2][2];
    double cg = j[0][0] * j[1][0] + j[0][1] * j[1][1] + j[0][2] * j[1][2];
    double Kq = (a2 - c2) / b2, cb2 = c2 / b2;
    double N[3] = {1.0 + Kq, -2.0 * Kq * cb, Kq - 1.0};
    double D[2] = {2.0 * cg, -2.0 * ca};
    double Q[3] = {1.0, -2.0 * cb, 1.0};
    double DD[3], NN[5], ND[4], QDD[5];
    pmul_dev(D, 1, D, 1, DD);
    pmul_dev(N, 2, N, 2, NN);
    pmul_dev(N, 2, D, 1, ND);
    pmul_dev(Q, 2, DD, 2, QDD);
    double P[5];
    for (int i = 0; i < 5; ++i) {
        double v = NN[i] - cb2 * QDD[i];
        if (i < 3) v = v + DD[i];
        if (i < 4) v = v - 2.0 * cg * ND[i];
        P[i] = v;
    }
    double roots[4];
    const int nr = real_roots_trim<4>(P, roots);
    int ns = 0, best = -1;
    double be = INFINITY;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k >= nr) break;
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
        double R[9], t[3];
        if (align3_dev(w3, Pc, R, t)) {
            double e = reproj_err2_dev(R, t, K, w4, im4);
            if (e < be) {
                be = e; best = ns;
                for (int q = 0; q < 9; ++q) Rb[q] = R[q];
                for (int q = 0; q < 3; ++q) tb[q] = t[q];
            }
            ns++;
        }
        if (ns == 4) break;
    }
    return best >= 0;
}

struct MsacArgs {
    const double* img; const double* world; const int* n; int n_stride;   // n[f * n_stride]
    MsacHyp* hyp; FrameGeom* fg; uint8_t* inliers;
    int kp_cap, n_hyp, max_trials;
    double thr, conf;
    uint32_t seed;
    uint32_t key0;           // frame key of frame 0 (frame f uses key0 + f)
    double K[9];
};

__device__ __forceinline__ int msac_n(const MsacArgs& a, int f)
{
    int n = a.n[(size_t)f * a.n_stride];
    return n < 0 ? 0 : (n > a.kp_cap ? a.kp_cap : n);
}

// hypothesis slot s of frame f: Philox sample, Grunert P3P, 4th-point disambiguation
__device__ void msac_hyp_slot(const MsacArgs& a, int f, int s, int n)
{
    MsacHyp* h = a.hyp + (size_t)f * a.n_hyp + s;
    h->valid = 0;
    if (n < 4 || s >= a.max_trials) return;
    const double* img = a.img + (size_t)f * a.kp_cap * 2;
    const double* world = a.world + (size_t)f * a.kp_cap * 3;
    uint32_t idx[4];
    bool ok = false;
    for (uint32_t att = 0; att < 16 && !ok; ++att) {
        vo_u32x4 c = {{(uint32_t)s, att, a.key0 + (uint32_t)f, 0x5EEDu}};
        vo_u32x4 r = vo_philox4x32_10(c, a.seed, 0x9E3779B9u);
        for (int q = 0; q < 4; ++q) idx[q] = vo_rand_index(r.v[q], (uint32_t)n);
        ok = idx[0] != idx[1] && idx[0] != idx[2] && idx[0] != idx[3] && idx[1] != idx[2] && idx[1] != idx[3] &&
             idx[2] != idx[3];
    }
    if (!ok) return;
    double im3[3][2], w3[3][3];
    for (int q = 0; q < 3; ++q) {
        im3[q][0] = img[2 * idx[q]]; im3[q][1] = img[2 * idx[q] + 1];
        for (int i = 0; i < 3; ++i) w3[q][i] = world[3 * idx[q] + i];
    }
    double R[9], t[3];
    if (!p3p_hyp_dev(im3, w3, world + 3 * idx[3], img + 2 * idx[3], a.K, R, t)) return;
    for (int q = 0; q < 9; ++q) h->R[q] = R[q];
    for (int q = 0; q < 3; ++q) h->t[q] = t[q];
    h->valid = 1;
}

#if VO_EXPERIMENTAL   // eager MSAC: test build only (libvo_exp.so), the cross-check of k_msac
// one lane per (frame, slot).  grid (ceil(n_hyp/64), B)  (eager form: every slot)
__global__ __launch_bounds__(64) void k_msac_hyp(MsacArgs a)
{
    const int f = blockIdx.y;
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= a.n_hyp) return;
    msac_hyp_slot(a, f, s, msac_n(a, f));
}
#endif  // VO_EXPERIMENTAL

// MSAC score of one valid slot by one wave: 64 lane-strided partials + the fixed shuffle tree
__device__ __forceinline__ void msac_score_slot(const MsacArgs& a, int f, int s, int n, int lane)
{
    MsacHyp* h = a.hyp + (size_t)f * a.n_hyp + s;
    const double* img = a.img + (size_t)f * a.kp_cap * 2;
    const double* world = a.world + (size_t)f * a.kp_cap * 3;
    double R[9], tt[3];
    for (int q = 0; q < 9; ++q) R[q] = h->R[q];
    for (int q = 0; q < 3; ++q) tt[q] = h->t[q];
    double part = 0.0;
    int cnt = 0;
    for (int k = lane; k < n; k += 64) {
        double e = reproj_err2_dev(R, tt, a.K, world + 3 * k, img + 2 * k);
        if (e < a.thr) cnt++;
        part = part + (e < a.thr ? e : a.thr);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        part = part + __shfl_down(part, off);
        cnt += __shfl_xor(cnt, off);
    }
    if (lane == 0) { h->score = part; h->n_in = cnt; }
}

#if VO_EXPERIMENTAL   // eager MSAC: test build only (libvo_exp.so), the cross-check of k_msac
// one wave per (frame, slot): MSAC score = 64 lane-strided partials + tree
__global__ __launch_bounds__(256) void k_msac_score(MsacArgs a, int B)
{
    const int lane = threadIdx.x & 63;
    const long total = (long)B * a.n_hyp;
    for (long t = (long)blockIdx.x * 4 + (threadIdx.x >> 6); t < total; t += (long)gridDim.x * 4) {
        const int f = (int)(t / a.n_hyp), s = (int)(t - (long)f * a.n_hyp);
        if (!a.hyp[(size_t)f * a.n_hyp + s].valid) continue;
        msac_score_slot(a, f, s, msac_n(a, f), lane);
    }
}
#endif  // VO_EXPERIMENTAL

__device__ int msac_trials_needed_dev(int n_in, int n, double conf)
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

__device__ void msac_final(const MsacArgs& a, int f, int n, int best, int status, int lane);

#if VO_EXPERIMENTAL   // eager MSAC: test build only (libvo_exp.so), the cross-check of k_msac
// sequential MSAC replay (adaptive trial count) + final inliers/pose.  block 64 per frame
__global__ __launch_bounds__(64) void k_msac_select(MsacArgs a)
{
    __shared__ int s_best;
    __shared__ int s_status;
    const int f = blockIdx.x, lane = threadIdx.x;
    const int n = msac_n(a, f);
    FrameGeom* g = a.fg + f;
    if (lane == 0) {
        int status = VO_OK, best = -1;
        if (n < 4) status = VO_ERR_TOO_FEW_POINTS;
        else {
            int num_trials = a.max_trials, trials = 0, best_in = 0;
            double best_score = INFINITY;
            for (int s = 0; s < a.max_trials && s < a.n_hyp && trials < num_trials; ++s) {
                const MsacHyp* h = a.hyp + (size_t)f * a.n_hyp + s;
                if (!h->valid) continue;
                trials++;
                if (h->score < best_score) {
                    best_score = h->score; best = s; best_in = h->n_in;
                    int need = msac_trials_needed_dev(h->n_in, n, a.conf);
                    if (need < num_trials) num_trials = need;
                }
            }
            if (best < 0 || best_in < 4) status = VO_ERR_NO_CONSENSUS;
        }
        s_best = best;
        s_status = status;
        g->status = status;
        g->best = best;
        g->n_tracked = n;
    }
    __syncthreads();
    msac_final(a, f, n, s_best, s_status, lane);
}
#endif  // VO_EXPERIMENTAL

// inlier mask + camera pose of the chosen slot (one wave)
__device__ void msac_final(const MsacArgs& a, int f, int n, int best, int status, int lane)
{
    FrameGeom* g = a.fg + f;
    if (status != VO_OK) {
        if (lane == 0) {
            g->n_inliers = 0;
            for (int q = 0; q < 16; ++q) g->T[q] = (q % 5 == 0) ? 1.0 : 0.0;
        }
        return;
    }
    const MsacHyp* h = a.hyp + (size_t)f * a.n_hyp + best;
    double R[9], t[3];
    for (int q = 0; q < 9; ++q) R[q] = h->R[q];
    for (int q = 0; q < 3; ++q) t[q] = h->t[q];
    const double* img = a.img + (size_t)f * a.kp_cap * 2;
    const double* world = a.world + (size_t)f * a.kp_cap * 3;
    int cnt = 0;
    for (int k = lane; k < n; k += 64) {
        const int in = reproj_err2_dev(R, t, a.K, world + 3 * k, img + 2 * k) < a.thr;
        a.inliers[(size_t)f * a.kp_cap + k] = (uint8_t)in;
        cnt += in;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
    if (lane == 0) {
        g->n_inliers = cnt;
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) g->T[4 * i + j] = R[3 * j + i];
            g->T[4 * i + 3] = -(R[i] * t[0] + R[3 + i] * t[1] + R[6 + i] * t[2]);
        }
        g->T[12] = 0; g->T[13] = 0; g->T[14] = 0; g->T[15] = 1;
    }
}

// Lazy MSAC: one 1024-thread block per frame walks the slots in chunks of 64 -- generate the
// chunk's hypotheses (lane per slot), score its valid ones (wave per slot), replay the
// sequential adaptive-termination loop over the chunk (thread 0, state carried across chunks)
// -- and stops at the chunk where the replay stops.  At the ~97 % inlier ratios of the KITTI
// path the replay needs ~3 trials, so one chunk of 64 replaces 2048 eager slots.  Same
// slots, same per-slot arithmetic, same replay: results identical to the eager kernels.
#ifndef VO_MSAC_CHUNK
#define VO_MSAC_CHUNK 64          // slots per chunk after the first (<= 64: one lane per slot)
#endif
#ifndef VO_MSAC_FIRST
#define VO_MSAC_FIRST 64          // slots of the first chunk (<= VO_MSAC_CHUNK)
#endif
#ifndef VO_MSAC_T
#define VO_MSAC_T 1024            // 16 waves: a chunk's 64 slots scored 4 per wave (one block per frame)
#endif
#ifndef VO_MSAC_SPLITGEN
#define VO_MSAC_SPLITGEN 0        // 1: the first chunk's hypotheses come from k_msac_gen (64-lane blocks)
#endif

#if VO_MSAC_SPLITGEN
// first chunk of every frame, one lane per slot: a 64-thread block has the whole register file
// for the P3P root finder that spills at k_msac's 1024-thread bound
__global__ __launch_bounds__(64) void k_msac_gen(MsacArgs a)
{
    const int f = blockIdx.x, s = threadIdx.x;
    const int limit = a.max_trials < a.n_hyp ? a.max_trials : a.n_hyp;
    if (s < VO_MSAC_FIRST && s < limit) msac_hyp_slot(a, f, s, msac_n(a, f));
}
#endif

__global__ __launch_bounds__(VO_MSAC_T) void k_msac(MsacArgs a)
{
    __shared__ int s_best, s_status, s_done;
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = msac_n(a, f);
    const int limit = a.max_trials < a.n_hyp ? a.max_trials : a.n_hyp;
    FrameGeom* g = a.fg + f;
    // replay state (thread 0)
    int num_trials = a.max_trials, trials = 0, best_in = 0, best = -1;
    double best_score = INFINITY;
    if (tid == 0) s_done = n < 4;
    __syncthreads();
    for (int c0 = 0, c1 = min(VO_MSAC_FIRST, limit); !s_done && c0 < limit;
         c0 = c1, c1 = min(c1 + VO_MSAC_CHUNK, limit)) {
        if (tid < c1 - c0 && (!VO_MSAC_SPLITGEN || c0 > 0)) msac_hyp_slot(a, f, c0 + tid, n);
        __syncthreads();                                    // the chunk's slots are written
        for (int s = c0 + wv; s < c1; s += VO_MSAC_T / 64)
            if (a.hyp[(size_t)f * a.n_hyp + s].valid) msac_score_slot(a, f, s, n, lane);
        __syncthreads();                                    // ... and scored
        if (tid == 0) {
            int s = c0;
            for (; s < c1 && trials < num_trials; ++s) {
                const MsacHyp* h = a.hyp + (size_t)f * a.n_hyp + s;
                if (!h->valid) continue;
                trials++;
                if (h->score < best_score) {
                    best_score = h->score; best = s; best_in = h->n_in;
                    int need = msac_trials_needed_dev(h->n_in, n, a.conf);
                    if (need < num_trials) num_trials = need;
                }
            }
            s_done = trials >= num_trials || s >= limit;
        }
        __syncthreads();
    }
    if (tid == 0) {
        int status = VO_OK;
        if (n < 4) status = VO_ERR_TOO_FEW_POINTS;
        else if (best < 0 || best_in < 4) status = VO_ERR_NO_CONSENSUS;
        s_best = best;
        s_status = status;
        g->status = status;
        g->best = best;
        g->n_tracked = n;
    }
    __syncthreads();
    if (wv) return;
    msac_final(a, f, n, s_best, s_status, lane);
}

// ---------------------------------------------------------------------------
// landmarks
// ---------------------------------------------------------------------------
// stereo subset positions of frame f (VO.m:141-142): spos[f][j] = (lx, ly, rx, ry)
__global__ void k_stereo_pos(const vo_keypoint* __restrict__ kp, int kp_cap, const int* __restrict__ pair_i,
                             const int* __restrict__ pair_j, const int* __restrict__ pair_n, float* __restrict__ spos,
                             int* __restrict__ s_n)
{
    const int f = blockIdx.y, K = kp_cap;
    int n = pair_n[f];
    if (n > K) n = K;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const vo_keypoint l = kp[(size_t)(2 * f) * K + pair_i[(size_t)f * K + j]];
        const vo_keypoint r = kp[(size_t)(2 * f + 1) * K + pair_j[(size_t)f * K + j]];
        float* p = spos + ((size_t)f * K + j) * 4;
        p[0] = l.x; p[1] = l.y; p[2] = r.x; p[3] = r.y;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) s_n[f] = n;
}

__device__ __forceinline__ uint32_t block_exscan_1024_g(uint32_t v, uint32_t* sh, uint32_t* total)
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

// new-landmark filter (VO.m:147-154) + compaction.  one block (1024) per frame.
// old positions: oldpos[f][k] (x1, y1, x2, y2) for k < *kn (kn[f * kn_stride]).
// flags: per-frame byte scratch (lm_keep, rewritten later by k_lm_tri).
__global__ __launch_bounds__(1024) void k_lm_filter(const float* __restrict__ spos, const int* __restrict__ s_n,
                                                    const float* __restrict__ oldpos, const int* __restrict__ kn,
                                                    int kn_stride, int kp_cap, uint8_t* __restrict__ flags,
                                                    int* __restrict__ lm_new, int* __restrict__ lm_M,
                                                    int* __restrict__ lm_rows)
{
    // One block per frame.  Stereo matches are taken 1024 at a time (one per thread,
    // rounds keep the ascending order of the compaction); the old points are staged
    // through LDS 1024 at a time and every thread compares its match against all of
    // them (broadcast reads).  hit = any old left x == lx or any old left y == ly, or
    // likewise on the right (VO.m:150-151, exact float equality).
    __shared__ uint32_t sh[32];
    __shared__ float4 so[1024];
    const int f = blockIdx.x, tid = threadIdx.x, K = kp_cap;
    int S = s_n[f];
    if (S > K) S = K;
    int nk = kn[(size_t)f * kn_stride];
    if (nk > K) nk = K;
    if (nk < 0) nk = 0;
    const float4* sp = reinterpret_cast<const float4*>(spos + (size_t)f * K * 4);
    const float4* op = reinterpret_cast<const float4*>(oldpos + (size_t)f * K * 4);
    uint8_t* fl = flags + (size_t)f * K;
    uint32_t done = 0;                                      // new landmarks emitted by earlier rounds
    for (int j0 = 0; j0 < S; j0 += 1024) {
        const int j = j0 + tid;
        const bool valid = j < S;
        const float4 p = valid ? sp[j] : float4{0.0f, 0.0f, 0.0f, 0.0f};
        // one lane-mask accumulator per coordinate (v_cmp + s_or per compare); 8 LDS
        // reads in flight per unrolled step; slots past the chunk end hold NaN (never equal)
        bool hx = false, hy = false, hz = false, hw = false;
        for (int k0 = 0; k0 < nk; k0 += 1024) {
            __syncthreads();
            so[tid] = k0 + tid < nk ? op[k0 + tid] : float4{NAN, NAN, NAN, NAN};
            __syncthreads();
            const int kc = (min(1024, nk - k0) + 7) & ~7;
            for (int k = 0; k < kc; k += 8) {
                float4 o[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) o[u] = so[k + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    hx |= o[u].x == p.x;
                    hy |= o[u].y == p.y;
                    hz |= o[u].z == p.z;
                    hw |= o[u].w == p.w;
                }
            }
        }
        const bool hit = hx || hy || hz || hw;
        const uint32_t isnew = (valid && !hit) ? 1u : 0u;
        if (valid) fl[j] = (uint8_t)isnew;
        uint32_t total;
        const uint32_t pos = block_exscan_1024_g(isnew, sh, &total);
        if (isnew) lm_new[(size_t)f * K + done + pos] = j;
        done += total;
    }
    __syncthreads();
    if (tid == 0) {
        lm_M[f] = (int)done;
        lm_rows[f] = 2;                                     // zeros(size(features_l,2),3): 2 rows
        for (int m = (int)done; m < 2; ++m) fl[m] = 0;      // rows beyond M stay zero rows
    }
}

// CreateLandmarksFromFeatures: odd 1-based rows (even 0-based), triangulate, z gates.  Every
// row up to max(M, 2) is written: the kept point, or a zero row (odd rows, rows failing a z
// gate, and the two preallocated rows of CreateLandmarksFromFeatures.m:2 when M < 2) -- the
// camera-frame rows vo_get_landmark_rows returns equal oracle_landmark_rows', zero rows included.
__global__ void k_lm_tri(const float* __restrict__ spos, const int* __restrict__ lm_new, const int* __restrict__ lm_M,
                         int kp_cap, CalibDev cal, float* __restrict__ lm_X, uint8_t* __restrict__ lm_keep,
                         int* __restrict__ lm_rows)
{
    const int f = blockIdx.y, K = kp_cap;
    const int M = lm_M[f];
    const int n = M > 2 ? M : 2;
    for (int m = blockIdx.x * blockDim.x + threadIdx.x; m < n; m += gridDim.x * blockDim.x) {
        uint8_t keep = 0;
        double X[3] = {0.0, 0.0, 0.0};
        if ((m & 1) == 0 && m < M) {
            const int j = lm_new[(size_t)f * K + m];
            const float* p = spos + ((size_t)f * K + j) * 4;
            dlt_point_dev(p[0], p[1], p[2], p[3], cal.P1, cal.P2, X);
            keep = !(X[2] < 0) && !(X[2] > 80);
            if (keep) atomicMax(lm_rows + f, m + 1);
        }
        float* o = lm_X + ((size_t)f * K + m) * 3;
        o[0] = keep ? (float)X[0] : 0.0f; o[1] = keep ? (float)X[1] : 0.0f; o[2] = keep ? (float)X[2] : 0.0f;
        lm_keep[(size_t)f * K + m] = keep;
    }
}

// ---------------------------------------------------------------------------
// host enqueue
// ---------------------------------------------------------------------------
static CalibDev calib_dev(const vo_calib& c)
{
    CalibDev d;
    memcpy(d.P1, c.P1, sizeof(d.P1));
    memcpy(d.P2, c.P2, sizeof(d.P2));
    memcpy(d.K, c.K, sizeof(d.K));
    return d;
}

static MsacArgs msac_args(GeomBuffers& g, const double* img, const double* world, const int* n, int n_stride,
                          const double K[9], const vo_ransac_params& rp, uint32_t key0)
{
    MsacArgs a;
    a.img = img; a.world = world; a.n = n; a.n_stride = n_stride;
    a.hyp = g.hyp; a.fg = g.fg; a.inliers = g.inliers;
    a.kp_cap = g.kp_cap; a.n_hyp = g.n_hyp; a.max_trials = rp.max_num_trials < g.n_hyp ? rp.max_num_trials : g.n_hyp;
    a.thr = rp.max_reprojection_error * rp.max_reprojection_error;
    a.conf = rp.confidence / 100.0;
    a.seed = rp.seed;
    a.key0 = key0;
    memcpy(a.K, K, sizeof(a.K));
    return a;
}

static void msac_enqueue(const MsacArgs& a, int B, hipStream_t s)
{
#if VO_EXPERIMENTAL
    // test build: the eager form (every slot generated and scored, then the replay) when
    // vo_exp_set selects it -- the cross-check of the lazy kernel (tests/test_gpu_geometry.py)
    if (g_exp_msac_eager) {
        VO_LAUNCH(k_msac_hyp, dim3((a.n_hyp + 63) / 64, B), dim3(64), 0, s, a);
        int blocks = (B * a.n_hyp + 3) / 4;
        if (blocks > 4096) blocks = 4096;
        VO_LAUNCH(k_msac_score, dim3(blocks), dim3(256), 0, s, a, B);
        VO_LAUNCH(k_msac_select, dim3(B), dim3(64), 0, s, a);
        return;
    }
#endif
#if VO_MSAC_SPLITGEN
    VO_LAUNCH(k_msac_gen, dim3(B), dim3(64), 0, s, a);
#endif
    VO_LAUNCH(k_msac, dim3(B), dim3(VO_MSAC_T), 0, s, a);
}

void track_enqueue(GeomBuffers& g, const MatchBuffers& mb, const MatchJob* d_track_jobs, const StepArgs& a,
                   const vo_match_params& mp, hipStream_t s)
{
    const int B = a.B, M = a.max_frames, K = a.kp_cap;
#ifndef VO_MATCH_FINISH
#define VO_MATCH_FINISH 1         // the composition inside match_launch's finishing kernel (csrc/match.hip)
#endif
    if (VO_MATCH_FINISH) {
        for (int step = 0; step < 4; ++step) {
            MatchCompose cp{g.lists, g.list_n, a.pair_i, a.pair_j, M, K, step, 0};
            match_launch(mb, d_track_jobs + step * M, B, mp, s, &cp);
        }
        return;
    }
    ComposeArgs ca;
    ca.lists = g.lists; ca.list_n = g.list_n; ca.step_i = g.step_i; ca.step_j = g.step_j; ca.step_n = g.step_n;
    ca.pair_i = a.pair_i; ca.pair_j = a.pair_j; ca.pair_n = a.pair_n; ca.M = M; ca.kp_cap = K;
    for (int step = 0; step < 4; ++step) {
        match_launch(mb, d_track_jobs + step * M, B, mp, s);
        ca.step = step;
        VO_LAUNCH(k_compose, dim3(16, B), dim3(256), 0, s, ca);
    }
}

void geom_enqueue(GeomBuffers& g, const MatchBuffers& mb, const MatchJob* d_track_jobs, const StepArgs& a,
                  const vo_match_params& mp, hipStream_t s)
{
    const int B = a.B, M = a.max_frames, K = a.kp_cap;
    track_enqueue(g, mb, d_track_jobs, a, mp, s);
    CalibDev cal = calib_dev(a.calib);
    VO_LAUNCH(k_gather_tri, dim3(16, B), dim3(64), 0, s, a.sb->kp, K, g.lists, g.list_n, g.oldpos, g.imgpt, g.world, M, cal);
    MsacArgs ma = msac_args(g, g.imgpt, g.world, g.list_n + 3, 4, a.calib.K, a.rp, (uint32_t)a.frame_index0);
    msac_enqueue(ma, B, s);
    VO_LAUNCH(k_stereo_pos, dim3(16, B), dim3(256), 0, s, a.sb->kp, K, a.pair_i, a.pair_j, a.pair_n, g.spos, g.s_n);
    VO_LAUNCH(k_lm_filter, dim3(B), dim3(1024), 0, s, g.spos, g.s_n, g.oldpos, g.list_n + 3, 4, K, g.lm_keep, g.lm_new,
              g.lm_M, g.lm_rows);
    VO_LAUNCH(k_lm_tri, dim3(16, B), dim3(64), 0, s, g.spos, g.lm_new, g.lm_M, K, cal, g.lm_X, g.lm_keep, g.lm_rows);
}

// block f: its offset is the sum of the earlier frames' row counts (B <= 128), then a plain copy
__global__ __launch_bounds__(256) void k_lm_pack(const float* __restrict__ lm_X, const uint8_t* __restrict__ lm_keep,
                                                 const int* __restrict__ lm_rows, int kp_cap, float* __restrict__ pX,
                                                 uint8_t* __restrict__ pkeep)
{
    const int f = blockIdx.x, tid = threadIdx.x;
    __shared__ int off;
    if (tid < 64) {
        int v = 0;
        for (int g2 = tid; g2 < f; g2 += 64) v += min(lm_rows[g2], kp_cap);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
        if (tid == 0) off = v;
    }
    __syncthreads();
    const int n = min(lm_rows[f], kp_cap);
    const float* X = lm_X + (size_t)f * kp_cap * 3;
    for (int e = tid; e < 3 * n; e += 256) pX[(size_t)off * 3 + e] = X[e];
    for (int e = tid; e < n; e += 256) pkeep[off + e] = lm_keep[(size_t)f * kp_cap + e];
}

void lm_pack_launch(GeomBuffers& g, int B, float* pX, uint8_t* pkeep, hipStream_t s)
{
    VO_LAUNCH(k_lm_pack, dim3(B), dim3(256), 0, s, g.lm_X, g.lm_keep, g.lm_rows, g.kp_cap, pX, pkeep);
}

// block f: frame f's rows, one thread per row.  The f64 products and sums are those of the host
// lm_world (vo_api.hip) in the same order (no contraction: -ffp-contract=off), so the single-rounded
// world rows equal a single-process run's bit for bit.
__global__ __launch_bounds__(256) void k_lm_world(const double* __restrict__ poses, const long long* __restrict__ off,
                                                  const float* __restrict__ X, const uint8_t* __restrict__ keep,
                                                  float* __restrict__ out)
{
    const int f = blockIdx.x;
    const long long a = off[f], b = off[f + 1];
    double P[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) P[k] = poses[(size_t)16 * f + k];
    for (long long r = a + threadIdx.x; r < b; r += 256) {
        float w[3] = {0.0f, 0.0f, 0.0f};
        if (keep[r]) {
            const double x0 = X[3 * r], x1 = X[3 * r + 1], x2 = X[3 * r + 2];
#pragma unroll
            for (int i = 0; i < 3; ++i) w[i] = (float)(P[4 * i] * x0 + P[4 * i + 1] * x1 + P[4 * i + 2] * x2 + P[4 * i + 3]);
        }
        out[3 * r] = w[0]; out[3 * r + 1] = w[1]; out[3 * r + 2] = w[2];
    }
}

void lm_world_launch(const double* poses, const long long* off, int n_frames, const float* X, const uint8_t* keep,
                     float* out, hipStream_t s)
{
    if (n_frames <= 0) return;
    VO_LAUNCH(k_lm_world, dim3(n_frames), dim3(256), 0, s, poses, off, X, keep, out);
}

void triangulate_launch(const float* pos, int n, const vo_calib& c, double* X, hipStream_t s)
{
    if (n <= 0) return;
    int blocks = (n + 63) / 64;
    if (blocks > 1024) blocks = 1024;
    VO_LAUNCH(k_tri_list, dim3(blocks), dim3(64), 0, s, pos, n, calib_dev(c), X);
}

void estworldpose_launch(GeomBuffers& g, const double* img, const double* world, const int* n, const double K[9],
                         const vo_ransac_params& rp, uint32_t frame_key, hipStream_t s)
{
    MsacArgs ma = msac_args(g, img, world, n, 0, K, rp, frame_key);
    msac_enqueue(ma, 1, s);
}

void landmarks_launch(GeomBuffers& g, const int* kn, const vo_calib& c, hipStream_t s)
{
    CalibDev cal = calib_dev(c);
    VO_LAUNCH(k_lm_filter, dim3(1), dim3(1024), 0, s, g.spos, g.s_n, g.oldpos, kn, 0, g.kp_cap, g.lm_keep, g.lm_new, g.lm_M,
              g.lm_rows);
    VO_LAUNCH(k_lm_tri, dim3(16, 1), dim3(64), 0, s, g.spos, g.lm_new, g.lm_M, g.kp_cap, cal, g.lm_X, g.lm_keep, g.lm_rows);
}

}  // namespace vo
