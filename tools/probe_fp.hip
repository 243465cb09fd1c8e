// Probe: are the arithmetic primitives the spec relies on bit-identical
// between gfx950 and the x86 host?  Also discovers the i8 MFMA lane maps.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../include probe_fp.hip -o probe_fp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>
#include <random>
#include "vo_spec.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_f32(const float* a, const float* b, float* o, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = a[i], y = b[i];
    o[i * 8 + 0] = x / y;
    o[i * 8 + 1] = sqrtf(fabsf(x));
    o[i * 8 + 2] = vo_expf(-fabsf(x) * 0.01f);
    o[i * 8 + 3] = vo_atan2_deg(x, y);
    float s, c; vo_sincos_deg(x * 0.001f, &s, &c);
    o[i * 8 + 4] = s; o[i * 8 + 5] = c;
    o[i * 8 + 6] = fmaf(x, y, x);
    o[i * 8 + 7] = (float)rintf(x * 0.37f) + floorf(y * 0.11f);
}
__global__ void k_f64(const double* a, const double* b, double* o, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x = a[i], y = b[i];
    o[i * 5 + 0] = x / y;
    o[i * 5 + 1] = sqrt(fabs(x));
    o[i * 5 + 2] = vo_exp_d(-fabs(x) * 1e-3);
    o[i * 5 + 3] = vo_log_d(fabs(x) + 1e-300);
    o[i * 5 + 4] = (double)(float)(x * y);
}

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__global__ void k_mfma(const v4i* a, const v4i* b, v16i* c32, v4i* c16) {
    int l = threadIdx.x;
    v16i acc = {0};
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[l], b[l], acc, 0, 0, 0);
    c32[l] = acc;
    v4i acc2 = {0, 0, 0, 0};
    acc2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[l], b[l], acc2, 0, 0, 0);
    c16[l] = acc2;
}

static int kmap32(int hyp, int l, int j) { int h = l >> 5; return hyp == 0 ? 16 * h + j : (j < 8 ? 8 * h + j : 16 + 8 * h + (j - 8)); }
static int kmap16(int hyp, int l, int j) { int h = l >> 4; return hyp == 0 ? 16 * h + j : (j < 8 ? 8 * h + j : 32 + 8 * h + (j - 8)); }

int main() {
    const int n = 1 << 20;
    std::mt19937 rng(123);
    std::vector<float> a(n), b(n), o(n * 8);
    for (int i = 0; i < n; ++i) {
        uint32_t ua = rng(), ub = rng();
        // mix of "interesting" and random-bit floats
        a[i] = (i & 1) ? vo_u32_as_f32((ua & 0x807fffffu) | ((100u + (ua >> 24) % 60u) << 23)) : (float)((int)(ua % 20001) - 10000) * 0.0173f;
        b[i] = (i & 2) ? vo_u32_as_f32((ub & 0x807fffffu) | ((100u + (ub >> 24) % 60u) << 23)) : (float)((int)(ub % 20001) - 10000) * 0.0311f + 0.5f;
    }
    float *da, *db, *dout;
    CK(hipMalloc(&da, n * 4)); CK(hipMalloc(&db, n * 4)); CK(hipMalloc(&dout, n * 32));
    CK(hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice));
    k_f32<<<n / 256, 256>>>(da, db, dout, n);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o.data(), dout, n * 32, hipMemcpyDeviceToHost));
    long bad[8] = {0};
    for (int i = 0; i < n; ++i) {
        float x = a[i], y = b[i];
        float r[8];
        r[0] = x / y; r[1] = sqrtf(fabsf(x)); r[2] = vo_expf(-fabsf(x) * 0.01f); r[3] = vo_atan2_deg(x, y);
        vo_sincos_deg(x * 0.001f, &r[4], &r[5]); r[6] = fmaf(x, y, x); r[7] = (float)rintf(x * 0.37f) + floorf(y * 0.11f);
        for (int k = 0; k < 8; ++k) {
            uint32_t u1 = vo_f32_as_u32(r[k]), u2 = vo_f32_as_u32(o[i * 8 + k]);
            if (u1 != u2 && !(std::isnan(r[k]) && std::isnan(o[i * 8 + k]))) { if (bad[k] < 3) printf("f32 op%d mismatch x=%a y=%a host=%a dev=%a\n", k, x, y, r[k], o[i*8+k]); bad[k]++; }
        }
    }
    printf("F32 mismatches: div=%ld sqrt=%ld vo_expf=%ld vo_atan2=%ld sin=%ld cos=%ld fmaf=%ld rint/floor=%ld\n", bad[0], bad[1], bad[2], bad[3], bad[4], bad[5], bad[6], bad[7]);

    std::vector<double> ad(n), bd(n), od(n * 5);
    for (int i = 0; i < n; ++i) {
        uint64_t ua = ((uint64_t)rng() << 32) | rng(), ub = ((uint64_t)rng() << 32) | rng();
        ad[i] = vo_u64_as_f64((ua & 0x800fffffffffffffULL) | ((uint64_t)(900 + (ua >> 52) % 250) << 52));
        bd[i] = vo_u64_as_f64((ub & 0x800fffffffffffffULL) | ((uint64_t)(900 + (ub >> 52) % 250) << 52));
    }
    double *dad, *dbd, *dod;
    CK(hipMalloc(&dad, n * 8)); CK(hipMalloc(&dbd, n * 8)); CK(hipMalloc(&dod, n * 40));
    CK(hipMemcpy(dad, ad.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dbd, bd.data(), n * 8, hipMemcpyHostToDevice));
    k_f64<<<n / 256, 256>>>(dad, dbd, dod, n);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(od.data(), dod, n * 40, hipMemcpyDeviceToHost));
    long badd[5] = {0};
    for (int i = 0; i < n; ++i) {
        double x = ad[i], y = bd[i];
        double r[5] = {x / y, sqrt(fabs(x)), vo_exp_d(-fabs(x) * 1e-3), vo_log_d(fabs(x) + 1e-300), (double)(float)(x * y)};
        for (int k = 0; k < 5; ++k)
            if (vo_f64_as_u64(r[k]) != vo_f64_as_u64(od[i * 5 + k])) { if (badd[k] < 3) printf("f64 op%d mismatch x=%a y=%a host=%a dev=%a\n", k, x, y, r[k], od[i*5+k]); badd[k]++; }
    }
    printf("F64 mismatches: div=%ld sqrt=%ld vo_exp_d=%ld vo_log_d=%ld cvt=%ld\n", badd[0], badd[1], badd[2], badd[3], badd[4]);

    // MFMA i8 lane map discovery
    int8_t A[32][64], B[64][32];
    for (int r = 0; r < 32; ++r) for (int k = 0; k < 64; ++k) A[r][k] = (int8_t)(rng() % 255 - 127);
    for (int k = 0; k < 64; ++k) for (int c = 0; c < 32; ++c) B[k][c] = (int8_t)(rng() % 255 - 127);
    for (int hyp = 0; hyp < 2; ++hyp) {
        std::vector<v4i> ha(64), hb(64);
        std::vector<v16i> hc(64); std::vector<v4i> hc16(64);
        for (int l = 0; l < 64; ++l) {
            int8_t ab[16], bb[16];
            for (int j = 0; j < 16; ++j) { ab[j] = A[l & 31][kmap32(hyp, l, j)]; bb[j] = B[kmap32(hyp, l, j)][l & 31]; }
            memcpy(&ha[l], ab, 16); memcpy(&hb[l], bb, 16);
        }
        v4i *dA, *dB, *dC16; v16i* dC;
        CK(hipMalloc(&dA, 64 * 16)); CK(hipMalloc(&dB, 64 * 16)); CK(hipMalloc(&dC, 64 * 64)); CK(hipMalloc(&dC16, 64 * 16));
        CK(hipMemcpy(dA, ha.data(), 64 * 16, hipMemcpyHostToDevice));
        CK(hipMemcpy(dB, hb.data(), 64 * 16, hipMemcpyHostToDevice));
        k_mfma<<<1, 64>>>(dA, dB, dC, dC16);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hc.data(), dC, 64 * 64, hipMemcpyDeviceToHost));
        int err = 0;
        for (int l = 0; l < 64; ++l) for (int reg = 0; reg < 16; ++reg) {
            int col = l & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (l >> 5);
            int ref = 0; for (int k = 0; k < 32; ++k) ref += A[row][k] * B[k][col];
            if (ref != hc[l][reg]) err++;
        }
        printf("mfma_i32_32x32x32_i8 hyp%d: %d mismatches of 1024\n", hyp, err);
        // 16x16x64
        for (int l = 0; l < 64; ++l) {
            int8_t ab[16], bb[16];
            for (int j = 0; j < 16; ++j) { ab[j] = A[l & 15][kmap16(hyp, l, j)]; bb[j] = B[kmap16(hyp, l, j)][l & 15]; }
            memcpy(&ha[l], ab, 16); memcpy(&hb[l], bb, 16);
        }
        CK(hipMemcpy(dA, ha.data(), 64 * 16, hipMemcpyHostToDevice));
        CK(hipMemcpy(dB, hb.data(), 64 * 16, hipMemcpyHostToDevice));
        k_mfma<<<1, 64>>>(dA, dB, dC, dC16);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hc16.data(), dC16, 64 * 16, hipMemcpyDeviceToHost));
        err = 0;
        for (int l = 0; l < 64; ++l) for (int reg = 0; reg < 4; ++reg) {
            int col = l & 15, row = (l >> 4) * 4 + reg;
            int ref = 0; for (int k = 0; k < 64; ++k) ref += A[row][k] * B[k][col];
            if (ref != hc16[l][reg]) err++;
        }
        printf("mfma_i32_16x16x64_i8 hyp%d: %d mismatches of 256\n", hyp, err);
    }
    hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
    printf("device %s arch %s CUs %d\n", p.name, p.gcnArchName, p.multiProcessorCount);
    return 0;
}
