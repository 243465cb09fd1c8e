/*
 * spec_eval.c — exports the vo_spec.h primitives so the KATs can pin them
 * against numpy/libm (tests/test_spec_math.py).  TEST INFRASTRUCTURE ONLY.
 */
#include <stdint.h>
#include "vo_spec.h"

/* fn: 0 expf, 1 atan2_deg(y=in[2i], x=in[2i+1]), 2 sin_deg, 3 cos_deg, 4 exp_d, 5 log_d,
 *     6 rcp_nr, 7 sift_wt(s=in[2i], k=in[2i+1]) */
void oracle_spec_eval(int fn, const double* in, double* out, int n)
{
    for (int i = 0; i < n; ++i) {
        switch (fn) {
        case 0: out[i] = vo_expf((float)in[i]); break;
        case 1: out[i] = vo_atan2_deg((float)in[2 * i], (float)in[2 * i + 1]); break;
        case 2: { float s, c; vo_sincos_deg((float)in[i], &s, &c); out[i] = s; break; }
        case 3: { float s, c; vo_sincos_deg((float)in[i], &s, &c); out[i] = c; break; }
        case 4: out[i] = vo_exp_d(in[i]); break;
        case 5: out[i] = vo_log_d(in[i]); break;
        case 6: out[i] = vo_rcp_nr((float)in[i]); break;
        case 7: out[i] = vo_sift_wt((float)in[2 * i], (int)in[2 * i + 1]); break;
        default: out[i] = 0; break;
        }
    }
}

void oracle_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t* out)
{
    vo_u32x4 c = {{c0, c1, c2, c3}};
    vo_u32x4 r = vo_philox4x32_10(c, k0, k1);
    for (int i = 0; i < 4; ++i) out[i] = r.v[i];
}

int oracle_gauss_radius(double sigma)
{
    float k[VO_SIFT_MAX_RADIUS + 1];
    return vo_gauss_kernel(sigma, k, VO_SIFT_MAX_RADIUS + 1);
}

/* number of floats x in [-87, 0] (every bit pattern, -0 included) where the specialised window
 * exponential differs from vo_expf in any bit */
long oracle_spec_check_expf_nonpos(void)
{
    long bad = 0;
    const uint32_t lo = vo_f32_as_u32(-0.0f), hi = vo_f32_as_u32(-87.0f);
    for (uint32_t u = lo; u <= hi; ++u) {
        const float x = vo_u32_as_f32(u);
        if (vo_f32_as_u32(vo_expf_nonpos(x)) != vo_f32_as_u32(vo_expf(x))) ++bad;
    }
    if (vo_f32_as_u32(vo_expf_nonpos(0.0f)) != vo_f32_as_u32(vo_expf(0.0f))) ++bad;
    return bad;
}
