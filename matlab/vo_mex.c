/*
 * vo_mex.c — MATLAB MEX gateway of libvo: the reference-side binding of the drop-in boundary.
 *
 * VO.m calls Computer Vision Toolbox functions; MATLAB resolves a name to the first match on
 * its path, so the `.m` files next to this gateway (detectSIFTFeatures.m, extractFeatures.m,
 * matchFeatures.m, triangulate.m, estworldpose.m, CreateLandmarksFromFeatures.m) shadow the
 * toolbox and the reference's own CreateLandmarksFromFeatures.m without editing VO.m.  Each
 * calls this one gateway with a command string:
 *
 *   [loc, scale, ori, metric, desc, octave, layer] = vo_mex('sift', I)
 *        detectSIFTFeatures + extractFeatures(..,"Method","SIFT")        VO.m:79-84
 *   indexPairs = vo_mex('match', F1, F2)
 *        matchFeatures(F1, F2)                                   VO.m:87,283,293,311,323
 *   X = vo_mex('triangulate', x1, x2, P1, P2)
 *        triangulate                              VO.m:113-116, CreateLandmarksFromFeatures.m:7
 *   [A, inliers, status] = vo_mex('estworldpose', imagePoints, worldPoints, K, opts)
 *        estworldpose (P3P + MSAC)                                       VO.m:123-127
 *   rows = vo_mex('landmarks', features_l, features_r, P1, P2, A)
 *        CreateLandmarksFromFeatures.m:2-18 (the rows before the :20 append)
 *   [rel_A, A, status, nLandmarks] = vo_mex('step', Il, Ir, P1, P2)
 *        the whole loop body VO.m:70-161, `features` kept on the device
 *   L = vo_mex('landmarks_all'); vo_mex('reset'); vo_mex('close')
 *
 * Storage: MATLAB arrays are column-major and are handed to libvo as they lie wherever the
 * C-ABI takes a storage-order flag (images: vo_sift_ex / vo_step_batch_ex with col_major = 1,
 * ld = rows; N x 128 single descriptors: vo_match_f32 with col_major = 1, ld = N).  Small
 * matrices (points, 3x4 / 3x3 / 4x4) are transposed here into the ABI's row-major form.
 *
 * Errors: every libvo status becomes mexErrMsgIdAndTxt (which does not return); estworldpose's
 * two failures carry MATLAB-style identifiers, or come back as `status` (1 = not enough points,
 * 2 = not enough inliers: estworldpose's own codes) when the caller asks for that output.
 * One libvo context per MATLAB session (device 0), released by mexAtExit.
 *
 * Build in MATLAB:  mex -R2018a vo_mex.c -I<repo>/include -L<repo>/r7020e-visual-odometry_amd/lib -lvo
 * (tests/mex_shim builds this same file against a minimal mx-API for the test suite).
 */
#include "mex.h"
#include "vo.h"
#include <stdint.h>
#include <string.h>

#define VO_MEX_CAPACITY 16384            /* vo_sift_params.max_keypoints default */

static vo_ctx* g_ctx = NULL;
static int g_rows = 0, g_cols = 0;

static void cleanup(void)
{
    if (g_ctx) vo_destroy(g_ctx);
    g_ctx = NULL;
    g_rows = g_cols = 0;
}

static void check(int rc)
{
    if (rc == VO_OK) return;
    if (rc == VO_ERR_TOO_FEW_POINTS)
        mexErrMsgIdAndTxt("vision:estworldpose:notEnoughPoints", "%s", vo_last_error(g_ctx));
    if (rc == VO_ERR_NO_CONSENSUS)
        mexErrMsgIdAndTxt("vision:estworldpose:notEnoughInliers", "%s", vo_last_error(g_ctx));
    if (rc == VO_ERR_ARG) mexErrMsgIdAndTxt("vo:badArgument", "%s", vo_last_error(g_ctx));
    if (rc == VO_ERR_CAPACITY) mexErrMsgIdAndTxt("vo:capacity", "%s", vo_last_error(g_ctx));
    mexErrMsgIdAndTxt("vo:error", "%s", vo_last_error(g_ctx));
}

/* The session's context.  Image commands need one of their image size (a new size replaces
 * the context and its loop state); the others run on whatever context exists. */
static void need_ctx(int rows, int cols)
{
    if (g_ctx && rows > 0 && (rows != g_rows || cols != g_cols)) cleanup();
    if (!g_ctx) {
        if (rows <= 0) { rows = 64; cols = 64; }          /* size-independent commands */
        g_ctx = vo_create(0, rows, cols, 1, NULL, NULL, NULL, NULL);   /* defaults = VO.m's (1000 MSAC trials) */
        if (!g_ctx) mexErrMsgIdAndTxt("vo:create", "%s", vo_last_error(NULL));
        g_rows = rows;
        g_cols = cols;
        mexAtExit(cleanup);
    }
}

static void need_args(int nrhs, int want, const char* cmd)
{
    if (nrhs != want) mexErrMsgIdAndTxt("vo:nargin", "vo_mex('%s', ...) takes %d arguments, got %d", cmd, want - 1, nrhs - 1);
}

static void need_real(const mxArray* a, mxClassID cls, long rows, long cols, const char* what)
{
    if (mxGetClassID(a) != cls || mxIsComplex(a) || mxGetNumberOfDimensions(a) != 2)
        mexErrMsgIdAndTxt("vo:badArgument", "%s: wrong class or dimensions", what);
    if ((rows >= 0 && (long)mxGetM(a) != rows) || (cols >= 0 && (long)mxGetN(a) != cols))
        mexErrMsgIdAndTxt("vo:badArgument", "%s must be %ld x %ld", what, rows, cols);
}

/* r x c double matrix (column-major) -> row-major */
static void to_row_major(const mxArray* a, double* out, int r, int c, const char* what)
{
    need_real(a, mxDOUBLE_CLASS, r, c, what);
    const double* p = mxGetDoubles(a);
    for (int i = 0; i < r; ++i)
        for (int j = 0; j < c; ++j) out[i * c + j] = p[(size_t)j * r + i];
}

/* row-major 4x4 -> new MATLAB 4x4 double */
static mxArray* mat4_to_mx(const double* T)
{
    mxArray* m = mxCreateDoubleMatrix(4, 4, mxREAL);
    double* o = mxGetDoubles(m);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) o[j * 4 + i] = T[4 * i + j];
    return m;
}

/* n x k points, single or double, column-major -> row-major float (MATLAB Location is single) */
static float* points_f32(const mxArray* a, int k, int* n, const char* what)
{
    if ((!mxIsSingle(a) && !mxIsDouble(a)) || mxIsComplex(a) || mxGetNumberOfDimensions(a) != 2 ||
        ((int)mxGetN(a) != k && mxGetM(a) > 0))
        mexErrMsgIdAndTxt("vo:badArgument", "%s must be an N x %d single or double matrix", what, k);
    const int m = (int)mxGetM(a);
    float* v = (float*)mxMalloc(sizeof(float) * ((size_t)m * k + 1));
    if (mxIsSingle(a)) {
        const float* p = mxGetSingles(a);
        for (int i = 0; i < m; ++i) for (int j = 0; j < k; ++j) v[(size_t)i * k + j] = p[(size_t)j * m + i];
    } else {
        const double* p = mxGetDoubles(a);
        for (int i = 0; i < m; ++i) for (int j = 0; j < k; ++j) v[(size_t)i * k + j] = (float)p[(size_t)j * m + i];
    }
    *n = m;
    return v;
}

/* n x k double points, column-major -> row-major double */
static double* points_f64(const mxArray* a, int k, int n, const char* what)
{
    need_real(a, mxDOUBLE_CLASS, n, k, what);
    const double* p = mxGetDoubles(a);
    double* v = (double*)mxMalloc(sizeof(double) * ((size_t)n * k + 1));
    for (int i = 0; i < n; ++i) for (int j = 0; j < k; ++j) v[(size_t)i * k + j] = p[(size_t)j * n + i];
    return v;
}

/* calibration from the two 3x4 camera matrices VO.m:27-32 builds (K = P1(:, 1:3)) */
static vo_calib calib_from(const mxArray* P1, const mxArray* P2)
{
    vo_calib cal;
    to_row_major(P1, cal.P1, 3, 4, "P1");
    to_row_major(P2, cal.P2, 3, 4, "P2");
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) cal.K[3 * i + j] = cal.P1[4 * i + j];
    return cal;
}

static void cmd_sift(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[])
{
    need_args(nrhs, 2, "sift");
    const mxArray* I = prhs[1];                       /* uint8 rows x cols, column-major */
    need_real(I, mxUINT8_CLASS, -1, -1, "I");
    const int rows = (int)mxGetM(I), cols = (int)mxGetN(I);
    need_ctx(rows, cols);
    const int cap = VO_MEX_CAPACITY;
    int n = 0;
    vo_keypoint* kp = (vo_keypoint*)mxMalloc(sizeof(vo_keypoint) * cap);
    uint8_t* d = (uint8_t*)mxMalloc((size_t)cap * VO_DESC_LEN);
    check(vo_sift_ex(g_ctx, mxGetUint8s(I), rows, cols, rows, 1, kp, d, cap, &n));
    plhs[0] = mxCreateNumericMatrix(n, 2, mxSINGLE_CLASS, mxREAL);      /* Location, 1-based [x y] */
    float* loc = mxGetSingles(plhs[0]);
    for (int i = 0; i < n; ++i) { loc[i] = kp[i].x; loc[(size_t)n + i] = kp[i].y; }
    if (nlhs > 1) {
        plhs[1] = mxCreateNumericMatrix(n, 1, mxSINGLE_CLASS, mxREAL);  /* Scale */
        for (int i = 0; i < n; ++i) mxGetSingles(plhs[1])[i] = kp[i].scale;
    }
    if (nlhs > 2) {
        plhs[2] = mxCreateNumericMatrix(n, 1, mxSINGLE_CLASS, mxREAL);  /* Orientation: radians */
        for (int i = 0; i < n; ++i) mxGetSingles(plhs[2])[i] = (float)((double)kp[i].angle * (3.14159265358979323846 / 180.0));
    }
    if (nlhs > 3) {
        plhs[3] = mxCreateNumericMatrix(n, 1, mxSINGLE_CLASS, mxREAL);  /* Metric */
        for (int i = 0; i < n; ++i) mxGetSingles(plhs[3])[i] = kp[i].response;
    }
    if (nlhs > 4) {
        plhs[4] = mxCreateNumericMatrix(n, VO_DESC_LEN, mxSINGLE_CLASS, mxREAL);   /* N x 128 single */
        float* D = mxGetSingles(plhs[4]);
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < VO_DESC_LEN; ++k) D[(size_t)k * n + i] = (float)d[(size_t)i * VO_DESC_LEN + k];
    }
    if (nlhs > 5) {
        plhs[5] = mxCreateNumericMatrix(n, 1, mxINT32_CLASS, mxREAL);   /* Octave */
        for (int i = 0; i < n; ++i) mxGetInt32s(plhs[5])[i] = kp[i].octave;
    }
    if (nlhs > 6) {
        plhs[6] = mxCreateNumericMatrix(n, 1, mxINT32_CLASS, mxREAL);   /* Layer */
        for (int i = 0; i < n; ++i) mxGetInt32s(plhs[6])[i] = kp[i].layer;
    }
    mxFree(kp);
    mxFree(d);
}

static void cmd_match(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[])
{
    (void)nlhs;
    need_args(nrhs, 3, "match");
    for (int k = 1; k <= 2; ++k)
        if (mxGetM(prhs[k]) > 0) need_real(prhs[k], mxSINGLE_CLASS, -1, VO_DESC_LEN, k == 1 ? "features1" : "features2");
    need_ctx(0, 0);
    const int n1 = (int)mxGetM(prhs[1]), n2 = (int)mxGetM(prhs[2]);
    int P = 0;
    uint32_t* pr = (uint32_t*)mxMalloc(sizeof(uint32_t) * 2 * ((size_t)n1 + 1));
    /* N x 128 single exactly as extractFeatures returned it: col_major = 1, ld = N */
    check(vo_match_f32(g_ctx, n1 ? mxGetSingles(prhs[1]) : NULL, n1, n1 ? n1 : 1, n2 ? mxGetSingles(prhs[2]) : NULL, n2,
                       n2 ? n2 : 1, 1, pr, n1 + 1, &P));
    plhs[0] = mxCreateNumericMatrix(P, 2, mxUINT32_CLASS, mxREAL);
    uint32_t* o = mxGetUint32s(plhs[0]);
    for (int i = 0; i < P; ++i) { o[i] = pr[2 * i]; o[(size_t)P + i] = pr[2 * i + 1]; }
    mxFree(pr);
}

static void cmd_triangulate(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[])
{
    (void)nlhs;
    need_args(nrhs, 5, "triangulate");
    int n = 0, n2 = 0;
    float* x1 = points_f32(prhs[1], 2, &n, "matchedPoints1");
    float* x2 = points_f32(prhs[2], 2, &n2, "matchedPoints2");
    if (n != n2) mexErrMsgIdAndTxt("vo:badArgument", "matchedPoints1 and matchedPoints2 differ in length");
    double P1[12], P2[12];
    to_row_major(prhs[3], P1, 3, 4, "cameraMatrix1");
    to_row_major(prhs[4], P2, 3, 4, "cameraMatrix2");
    need_ctx(0, 0);
    double* X = (double*)mxMalloc(sizeof(double) * 3 * ((size_t)n + 1));
    check(vo_triangulate(g_ctx, x1, x2, n, P1, P2, X));
    plhs[0] = mxCreateNumericMatrix(n, 3, mxSINGLE_CLASS, mxREAL);     /* single, as for single inputs */
    float* o = mxGetSingles(plhs[0]);
    for (int i = 0; i < n; ++i) for (int a = 0; a < 3; ++a) o[(size_t)a * n + i] = (float)X[3 * i + a];
    mxFree(x1);
    mxFree(x2);
    mxFree(X);
}

/* opts (optional 5th argument): [MaxNumTrials Confidence MaxReprojectionError] double */
static void cmd_estworldpose(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[])
{
    if (nrhs != 4 && nrhs != 5) need_args(nrhs, 4, "estworldpose");
    const int n = (int)mxGetM(prhs[1]);
    double* img = points_f64(prhs[1], 2, n, "imagePoints");
    double* wld = points_f64(prhs[2], 3, n, "worldPoints");
    double K[9], T[16];
    to_row_major(prhs[3], K, 3, 3, "intrinsics.K");
    need_ctx(0, 0);
    vo_ransac_params rp;
    vo_default_ransac_params(&rp);
    if (nrhs == 5) {
        need_real(prhs[4], mxDOUBLE_CLASS, 1, 3, "opts");
        const double* o = mxGetDoubles(prhs[4]);
        rp.max_num_trials = (int32_t)o[0];
        rp.confidence = o[1];
        rp.max_reprojection_error = o[2];
    }
    uint8_t* inl = (uint8_t*)mxMalloc((size_t)n + 1);
    int nin = 0;
    memset(inl, 0, (size_t)n + 1);
    for (int k = 0; k < 16; ++k) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
    const int rc = vo_estworldpose(g_ctx, img, wld, n, K, &rp, 0, T, inl, &nin);
    if (nlhs > 2 && (rc == VO_ERR_TOO_FEW_POINTS || rc == VO_ERR_NO_CONSENSUS)) {
        /* estworldpose's status output: 1 = not enough points, 2 = not enough inliers */
        plhs[2] = mxCreateDoubleScalar(rc == VO_ERR_TOO_FEW_POINTS ? 1.0 : 2.0);
        for (int k = 0; k < 16; ++k) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
        memset(inl, 0, (size_t)n + 1);
    } else {
        check(rc);
        if (nlhs > 2) plhs[2] = mxCreateDoubleScalar(0.0);
    }
    plhs[0] = mat4_to_mx(T);
    if (nlhs > 1) {
        plhs[1] = mxCreateLogicalMatrix(n, 1);
        mxLogical* L = mxGetLogicals(plhs[1]);
        for (int i = 0; i < n; ++i) L[i] = inl[i] != 0;
    }
    mxFree(img);
    mxFree(wld);
    mxFree(inl);
}

/* CreateLandmarksFromFeatures(features_l, features_r, P1, P2, pose, ~) rows (:2-18): VO.m:145-158
 * has already filtered the points, so libvo's own filter runs against no old points (K = 0). */
static void cmd_landmarks(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[])
{
    (void)nlhs;
    need_args(nrhs, 6, "landmarks");
    int S = 0, S2 = 0;
    float* l = points_f32(prhs[1], 2, &S, "features_l");
    float* r = points_f32(prhs[2], 2, &S2, "features_r");
    if (S != S2) mexErrMsgIdAndTxt("vo:badArgument", "features_l and features_r differ in length");
    const vo_calib cal = calib_from(prhs[3], prhs[4]);
    double A[16];
    to_row_major(prhs[5], A, 4, 4, "pose.A");
    need_ctx(0, 0);
    check(vo_set_calib(g_ctx, &cal));
    int rows = 0;
    const int cap = S + 2;                             /* max(2, last kept odd row) <= S + 2 */
    double* out = (double*)mxMalloc(sizeof(double) * 3 * (size_t)cap);
    check(vo_landmarks(g_ctx, l, r, S, NULL, NULL, 0, A, out, cap, &rows));
    plhs[0] = mxCreateDoubleMatrix(rows, 3, mxREAL);
    double* o = mxGetDoubles(plhs[0]);
    for (int i = 0; i < rows; ++i) for (int a = 0; a < 3; ++a) o[(size_t)a * rows + i] = out[3 * i + a];
    mxFree(l);
    mxFree(r);
    mxFree(out);
}

static void cmd_step(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[])
{
    need_args(nrhs, 5, "step");
    const mxArray* Il = prhs[1];
    need_real(Il, mxUINT8_CLASS, -1, -1, "Il");
    const int rows = (int)mxGetM(Il), cols = (int)mxGetN(Il);
    need_real(prhs[2], mxUINT8_CLASS, rows, cols, "Ir");
    const vo_calib cal = calib_from(prhs[3], prhs[4]);
    need_ctx(rows, cols);
    check(vo_set_calib(g_ctx, &cal));
    vo_step_out o;
    check(vo_step_batch_ex(g_ctx, mxGetUint8s(Il), mxGetUint8s(prhs[2]), rows, 1, 1, &o));
    plhs[0] = mat4_to_mx(o.rel_pose);
    if (nlhs > 1) plhs[1] = mat4_to_mx(o.pose);
    if (nlhs > 2) plhs[2] = mxCreateDoubleScalar((double)o.status);
    if (nlhs > 3) plhs[3] = mxCreateDoubleScalar((double)o.n_landmarks);
}

static void cmd_landmarks_all(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[])
{
    (void)nlhs;
    (void)prhs;
    need_args(nrhs, 1, "landmarks_all");
    int rows = 0;
    if (g_ctx) check(vo_get_landmarks(g_ctx, NULL, 0, &rows));
    double* out = (double*)mxMalloc(sizeof(double) * 3 * ((size_t)rows + 1));
    if (rows) check(vo_get_landmarks(g_ctx, out, rows, &rows));
    plhs[0] = mxCreateDoubleMatrix(rows, 3, mxREAL);
    double* o = mxGetDoubles(plhs[0]);
    for (int i = 0; i < rows; ++i) for (int a = 0; a < 3; ++a) o[(size_t)a * rows + i] = out[3 * i + a];
    mxFree(out);
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[])
{
    char cmd[32];
    if (nrhs < 1 || !mxIsChar(prhs[0]) || mxGetString(prhs[0], cmd, sizeof cmd))
        mexErrMsgIdAndTxt("vo:nargin", "vo_mex(command, ...): first argument must be a command string");
    if (!strcmp(cmd, "sift")) cmd_sift(nlhs, plhs, nrhs, prhs);
    else if (!strcmp(cmd, "match")) cmd_match(nlhs, plhs, nrhs, prhs);
    else if (!strcmp(cmd, "triangulate")) cmd_triangulate(nlhs, plhs, nrhs, prhs);
    else if (!strcmp(cmd, "estworldpose")) cmd_estworldpose(nlhs, plhs, nrhs, prhs);
    else if (!strcmp(cmd, "landmarks")) cmd_landmarks(nlhs, plhs, nrhs, prhs);
    else if (!strcmp(cmd, "step")) cmd_step(nlhs, plhs, nrhs, prhs);
    else if (!strcmp(cmd, "landmarks_all")) cmd_landmarks_all(nlhs, plhs, nrhs, prhs);
    else if (!strcmp(cmd, "reset")) { if (g_ctx) check(vo_reset(g_ctx)); }
    else if (!strcmp(cmd, "close")) cleanup();
    else mexErrMsgIdAndTxt("vo:cmd", "vo_mex: unknown command '%s'", cmd);
}
