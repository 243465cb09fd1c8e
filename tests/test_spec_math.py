"""Pins the deterministic spec primitives of include/vo_spec.h (shared by the
oracle and the HIP path) against numpy/libm, with stated tolerances.  The GPU
evaluates the same recipes bit for bit (tools/probe_fp.hip on MI355X)."""
import math

import numpy as np


def test_expf_accuracy(oracle):
    x = np.concatenate([np.linspace(-87, 0, 20001), np.linspace(-5, 5, 2001)])
    got = oracle.spec_eval("expf", x)
    ref = np.exp(x.astype(np.float32).astype(np.float64))
    rel = np.abs(got - ref) / np.maximum(ref, 1e-38)
    assert rel.max() < 5e-7           # ~4 ulp of float
    assert oracle.spec_eval("expf", np.array([-100.0]))[0] == 0.0


def test_expf_nonpos_equals_expf_exhaustively(oracle):
    # the HIP window weights (k_orient, k_desc) use the ldexp form on [-87, 0]
    assert oracle.spec_check_expf_nonpos() == 0


def test_rcp_nr_accuracy(oracle):
    """vo_rcp_nr (integer seed + 3 Newton steps, the reciprocal inside vo_atan2_deg) is within
    2 ulp of 1/d over the range atan2 feeds it (denominators of gradient components, clamped to
    >= 1e-30) and well beyond."""
    rng = np.random.default_rng(3)
    d = np.concatenate([np.exp2(rng.uniform(-100, 100, 200000)), [1e-30, 1.0, 2.0, 0.75, 510.0, 1024.0]])
    d = d.astype(np.float32)
    got = oracle.spec_eval("rcp_nr", d.astype(np.float64)).astype(np.float32)
    ref = (1.0 / d.astype(np.float64)).astype(np.float32)
    ulp = np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    assert ulp.max() <= 2, ulp.max()
    assert (ulp == 0).mean() > 0.5


def test_sift_wt_is_the_separable_window_weight(oracle):
    """vo_sift_wt(s, |i|) * vo_sift_wt(s, |j|) (the k_desc window weight, s = -1/8 / hist_width^2)
    agrees with OpenCV's exp((i^2 + j^2) s) to float rounding over the descriptor window."""
    hw = np.float32(3.0 * 3.2)
    s = np.float32(np.float32(-0.125) / (hw * hw))
    k = np.arange(0, 35)
    wk = oracle.spec_eval("sift_wt", np.stack([np.full(len(k), s, np.float64), k], 1).reshape(-1))
    i, j = np.meshgrid(k, k)
    w = (wk[i].astype(np.float32) * wk[j].astype(np.float32)).astype(np.float64)
    ref = np.exp((i * i + j * j) * np.float64(s))
    assert np.max(np.abs(w - ref) / ref) < 4e-7


def _cv_fast_atan2(y, x):
    """OpenCV's fastAtan2 (cv::hal, degrees) in float32 numpy: the formula the spec restates."""
    f = np.float32
    p1, p3 = f(0.9997878412794807) * f(57.29577951308232), f(-0.3258083974640975) * f(57.29577951308232)
    p5, p7 = f(0.1555786518463281) * f(57.29577951308232), f(-0.04432655554792128) * f(57.29577951308232)
    ax, ay = np.abs(x), np.abs(y)
    sw = ay > ax
    lo, hi = np.where(sw, ax, ay), np.where(sw, ay, ax)
    c = (lo / (hi + f(2.220446049250313e-16))).astype(f)
    c2 = c * c
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c
    a = np.where(sw, f(90) - a, a)
    a = np.where(x < 0, f(180) - a, a)
    return np.where(y < 0, f(360) - a, a).astype(np.float64)


def test_atan2_deg_is_opencv_fast_atan2(oracle):
    """vo_atan2_deg restates OpenCV's fastAtan2 (its quotient by vo_rcp_nr, Horner by fmaf): equal
    to the float formula within 1e-4 deg, and like it within 0.01 deg of the true atan2."""
    rng = np.random.default_rng(0)
    y = rng.uniform(-300, 300, 20000)
    x = rng.uniform(-300, 300, 20000)
    yx = np.stack([y, x], 1).astype(np.float32).astype(np.float64)
    got = oracle.spec_eval("atan2_deg", yx.reshape(-1))
    for ref, tol in ((_cv_fast_atan2(yx[:, 0].astype(np.float32), yx[:, 1].astype(np.float32)), 1e-4),
                     (np.degrees(np.arctan2(yx[:, 0], yx[:, 1])) % 360.0, 1e-2)):
        d = np.abs(got - ref)
        d = np.minimum(d, 360 - d)
        assert d.max() < tol, (d.max(), tol)
    assert np.all((got >= 0) & (got < 360))
    # axes and the origin (OpenCV fastAtan2 conventions)
    pts = np.array([[0, 1], [1, 0], [0, -1], [-1, 0], [0, 0]], np.float64)
    assert np.allclose(oracle.spec_eval("atan2_deg", pts.reshape(-1)), [0, 90, 180, 270, 0], atol=1e-5)


def test_sincos_deg_accuracy(oracle):
    d = np.linspace(-720, 720, 40001)
    s = oracle.spec_eval("sin_deg", d)
    c = oracle.spec_eval("cos_deg", d)
    r = np.radians(d.astype(np.float32).astype(np.float64))
    assert np.abs(s - np.sin(r)).max() < 3e-7
    assert np.abs(c - np.cos(r)).max() < 3e-7


def test_exp_log_double(oracle):
    x = np.linspace(-700, 700, 10001)
    assert np.max(np.abs(oracle.spec_eval("exp_d", x) / np.exp(x) - 1)) < 1e-15
    y = np.exp(np.linspace(-700, 700, 10001))
    assert np.max(np.abs(oracle.spec_eval("log_d", y) - np.log(y))) < 4e-13
    assert oracle.spec_eval("log_d", np.array([0.0]))[0] < -1e307


def test_philox_known_answer(oracle):
    # Random123 Philox4x32-10 known-answer vectors (kat_vectors: philox4x32 10)
    assert oracle.philox((0, 0, 0, 0), (0, 0)).tolist() == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert oracle.philox((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF)).tolist() == \
        [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert oracle.philox((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0)).tolist() == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_gauss_kernel_matches_formula(oracle):
    for sigma in (1.2489995996796797, 1.2262735, 1.5450077, 1.9465878, 2.4525151, 3.0900650):
        k = oracle.gauss_kernel(sigma)
        r = len(k) - 1
        assert r == (int(round(sigma * 8 + 1)) | 1) // 2
        x = np.arange(-r, r + 1)
        g = np.exp(-x * x / (2 * sigma * sigma))
        g /= g.sum()
        assert np.allclose(k, g[r:], rtol=1e-6, atol=1e-9)
        assert abs(k[0] + 2 * k[1:].sum() - 1) < 1e-6
