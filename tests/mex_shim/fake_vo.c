/* fake_vo.c — a recording stand-in for libvo (test infrastructure only).
 *
 * Linked into the MEX gateway instead of the real libvo, so the CPU test suite can check the
 * gateway's own work -- argument validation, MATLAB column-major <-> the C-ABI's row-major
 * forms, 1-based index pairs, degrees -> radians, 4x4 transposes, status mapping -- without a
 * GPU.  Each entry point records what it received (images re-read through the ld / col_major
 * the gateway passed) and returns outputs that are simple known functions of its inputs.
 * The GPU test (tests/test_gpu_mex.py) links the same gateway against the real libvo. */
#include "vo.h"
#include <stdlib.h>
#include <string.h>

struct vo_ctx { int rows, cols; vo_calib calib; int has_calib; };

#define CAP (1 << 20)
static struct {
    int creates, destroys, resets, rows, cols, ld, col_major, n1, ld1, n2, ld2, n, S, K, B, capacity, trials;
    double conf, err, P1[12], P2[12], K9[9], pose[16];
    uint8_t img[2][CAP];
    float f1[CAP / 4], f2[CAP / 4];
    double d1[CAP / 8], d2[CAP / 8];
} R;

int fake_int(const char* k)
{
#define F(name) if (!strcmp(k, #name)) return R.name;
    F(creates) F(destroys) F(resets) F(rows) F(cols) F(ld) F(col_major) F(n1) F(ld1) F(n2) F(ld2) F(n) F(S) F(K) F(B)
    F(capacity) F(trials)
#undef F
    return -999;
}
double fake_dbl(const char* k, int i)
{
    if (!strcmp(k, "conf")) return R.conf;
    if (!strcmp(k, "err")) return R.err;
    if (!strcmp(k, "P1")) return R.P1[i];
    if (!strcmp(k, "P2")) return R.P2[i];
    if (!strcmp(k, "K9")) return R.K9[i];
    if (!strcmp(k, "pose")) return R.pose[i];
    if (!strcmp(k, "d1")) return R.d1[i];
    if (!strcmp(k, "d2")) return R.d2[i];
    if (!strcmp(k, "f1")) return R.f1[i];
    if (!strcmp(k, "f2")) return R.f2[i];
    return -999.0;
}
const uint8_t* fake_img(int which) { return R.img[which]; }
void fake_clear(void) { memset(&R, 0, sizeof(R)); }

static const char* g_err = "fake libvo";
const char* vo_last_error(const vo_ctx* c) { (void)c; return g_err; }
void vo_default_ransac_params(vo_ransac_params* p) { p->max_num_trials = 1000; p->confidence = 99.0; p->max_reprojection_error = 1.0; p->seed = 0x5EED; }

vo_ctx* vo_create(int device, int rows, int cols, int max_batch, const vo_calib* calib, const vo_sift_params* sift,
                  const vo_match_params* match, const vo_ransac_params* ransac)
{
    (void)device; (void)max_batch; (void)sift; (void)match; (void)ransac;
    if (rows < 16 || cols < 16) return NULL;
    vo_ctx* c = (vo_ctx*)calloc(1, sizeof(vo_ctx));
    c->rows = rows; c->cols = cols;
    if (calib) { c->calib = *calib; c->has_calib = 1; }
    R.creates++;
    return c;
}
void vo_destroy(vo_ctx* c) { if (c) { R.destroys++; free(c); } }
int vo_set_calib(vo_ctx* c, const vo_calib* cal)
{
    c->calib = *cal; c->has_calib = 1;
    memcpy(R.P1, cal->P1, sizeof(R.P1)); memcpy(R.P2, cal->P2, sizeof(R.P2)); memcpy(R.K9, cal->K, sizeof(R.K9));
    return VO_OK;
}
int vo_reset(vo_ctx* c) { (void)c; R.resets++; return VO_OK; }

/* image as the C-ABI reads it: col_major = 1 -> pixel (r, c) at img[c * ld + r] */
static void grab(int which, const uint8_t* img, int rows, int cols, int ld, int col_major)
{
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols && r * cols + c < CAP; ++c)
            R.img[which][r * cols + c] = col_major ? img[(size_t)c * ld + r] : img[(size_t)r * ld + c];
}

int vo_sift_ex(vo_ctx* c, const uint8_t* img, int rows, int cols, int ld, int col_major, vo_keypoint* kps, uint8_t* desc,
               int capacity, int* n_out)
{
    if (rows != c->rows || cols != c->cols) return VO_ERR_ARG;
    R.rows = rows; R.cols = cols; R.ld = ld; R.col_major = col_major; R.capacity = capacity;
    grab(0, img, rows, cols, ld, col_major);
    const int n = 5;
    *n_out = n;
    if (capacity < n) return VO_ERR_CAPACITY;
    for (int i = 0; i < n; ++i) {
        vo_keypoint k = {1.5f + i, 2.25f + 3 * i, 2.2f * i, 45.0f * i, 0.01f * i, i - 1, 1 + i % 3, 1.1f * i};
        kps[i] = k;
        for (int j = 0; j < VO_DESC_LEN; ++j) desc[i * VO_DESC_LEN + j] = (uint8_t)((i * 31 + j * 7) & 255);
    }
    return VO_OK;
}

int vo_match_f32(vo_ctx* c, const float* F1, int n1, int ld1, const float* F2, int n2, int ld2, int col_major,
                 uint32_t* pairs, int capacity, int* n_pairs)
{
    (void)c;
    R.n1 = n1; R.ld1 = ld1; R.n2 = n2; R.ld2 = ld2; R.col_major = col_major; R.capacity = capacity;
    for (int i = 0; i < n1; ++i) for (int k = 0; k < VO_DESC_LEN; ++k)   /* row-major view of what arrived */
        R.f1[i * VO_DESC_LEN + k] = col_major ? F1[i + (size_t)k * ld1] : F1[(size_t)i * ld1 + k];
    for (int i = 0; i < n2; ++i) for (int k = 0; k < VO_DESC_LEN; ++k)
        R.f2[i * VO_DESC_LEN + k] = col_major ? F2[i + (size_t)k * ld2] : F2[(size_t)i * ld2 + k];
    int P = 0;
    for (int i = 0; i < n1 && i < n2; i += 2) {
        if (P < capacity) { pairs[2 * P] = (uint32_t)i + 1; pairs[2 * P + 1] = (uint32_t)(n2 - i); }
        ++P;
    }
    *n_pairs = P;
    return P > capacity ? VO_ERR_CAPACITY : VO_OK;
}

int vo_triangulate(vo_ctx* c, const float* x1, const float* x2, int n, const double P1[12], const double P2[12], double* X)
{
    (void)c;
    R.n = n;
    memcpy(R.P1, P1, sizeof(R.P1)); memcpy(R.P2, P2, sizeof(R.P2));
    for (int i = 0; i < 2 * n; ++i) { R.f1[i] = x1[i]; R.f2[i] = x2[i]; }
    for (int i = 0; i < n; ++i) {
        X[3 * i] = x1[2 * i];
        X[3 * i + 1] = x2[2 * i + 1];
        X[3 * i + 2] = P1[3] + P2[7] + i;
    }
    return VO_OK;
}

int vo_estworldpose(vo_ctx* c, const double* img, const double* world, int n, const double K[9],
                    const vo_ransac_params* params, uint32_t frame_key, double T[16], uint8_t* inliers, int* n_inliers)
{
    (void)c; (void)frame_key;
    R.n = n;
    memcpy(R.K9, K, sizeof(R.K9));
    R.trials = params ? params->max_num_trials : -1;
    R.conf = params ? params->confidence : -1;
    R.err = params ? params->max_reprojection_error : -1;
    for (int i = 0; i < 2 * n; ++i) R.d1[i] = img[i];
    for (int i = 0; i < 3 * n; ++i) R.d2[i] = world[i];
    if (n < 4) return VO_ERR_TOO_FEW_POINTS;
    if (n == 5) return VO_ERR_NO_CONSENSUS;
    int m = 0;
    for (int k = 0; k < 16; ++k) T[k] = k + 1.5;
    for (int i = 0; i < n; ++i) { inliers[i] = (uint8_t)(i % 2); m += i % 2; }
    *n_inliers = m;
    return VO_OK;
}

int vo_landmarks(vo_ctx* c, const float* l_pos, const float* r_pos, int S, const float* old_l, const float* old_r, int K,
                 const double pose[16], double* out, int capacity, int* rows_out)
{
    (void)old_l; (void)old_r;
    if (!c->has_calib) return VO_ERR_STATE;
    R.S = S; R.K = K; R.capacity = capacity;
    memcpy(R.pose, pose, sizeof(R.pose));
    for (int i = 0; i < 2 * S; ++i) { R.f1[i] = l_pos[i]; R.f2[i] = r_pos[i]; }
    const int rows = S + 2;
    *rows_out = rows;
    if (rows > capacity) return VO_ERR_CAPACITY;
    for (int m = 0; m < rows; ++m)
        for (int a = 0; a < 3; ++a) out[3 * m + a] = (m < S ? l_pos[2 * m + (a % 2)] : 0.0) + pose[4 * a + 3];
    return VO_OK;
}

int vo_step_batch_ex(vo_ctx* c, const uint8_t* lefts, const uint8_t* rights, int ld, int col_major, int B, vo_step_out* outs)
{
    if (!c->has_calib) return VO_ERR_STATE;
    R.ld = ld; R.col_major = col_major; R.B = B; R.rows = c->rows; R.cols = c->cols;
    grab(0, lefts, c->rows, c->cols, ld, col_major);
    grab(1, rights, c->rows, c->cols, ld, col_major);
    for (int f = 0; f < B; ++f) {
        memset(&outs[f], 0, sizeof(outs[f]));
        for (int k = 0; k < 16; ++k) { outs[f].rel_pose[k] = k; outs[f].pose[k] = 100 + k; }
        outs[f].status = VO_OK;
        outs[f].n_landmarks = 7;
    }
    return VO_OK;
}

int vo_get_landmarks(vo_ctx* c, double* out, int capacity, int* rows)
{
    (void)c;
    *rows = 3;
    if (out) for (int k = 0; k < 9 && k < 3 * capacity; ++k) out[k] = 0.5 * k;
    return VO_OK;
}
