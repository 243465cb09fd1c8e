"""ctypes wrapper of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker.  The product package never
imports this module (tests/test_abi.py asserts that).

Parity status vs the MATLAB reference: "parity unpinned" (see oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "liboracle.so"
# the same sources built with -DVO_CV_LITERAL: OpenCV-literal float SIFT + MATLAB-literal
# float matcher (the reference implementations the spec's deterministic choices depart from)
LIB_CV = HERE / "build" / "liboracle_cv.so"


class SiftParams(C.Structure):
    _fields_ = [("n_octave_layers", C.c_int32), ("sigma", C.c_float), ("contrast_threshold", C.c_float),
                ("edge_threshold", C.c_float), ("upsample", C.c_int32), ("max_keypoints", C.c_int32)]


class MatchParams(C.Structure):
    _fields_ = [("match_threshold", C.c_float), ("max_ratio", C.c_float)]


class RansacParams(C.Structure):
    _fields_ = [("max_num_trials", C.c_int32), ("confidence", C.c_double),
                ("max_reprojection_error", C.c_double), ("seed", C.c_uint32)]


class Calib(C.Structure):
    _fields_ = [("P1", C.c_double * 12), ("P2", C.c_double * 12), ("K", C.c_double * 9)]


class Keypoint(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("layer", C.c_int32), ("scale", C.c_float)]


class StepOut(C.Structure):
    _fields_ = [("status", C.c_int32), ("n_left", C.c_int32), ("n_right", C.c_int32),
                ("n_stereo", C.c_int32), ("n_tracked", C.c_int32), ("n_inliers", C.c_int32),
                ("n_landmarks", C.c_int32), ("flags", C.c_int32),
                ("rel_pose", C.c_double * 16), ("pose", C.c_double * 16)]


KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4"), ("layer", "<i4"), ("scale", "<f4")])


def sift_params(max_keypoints: int = 16384) -> SiftParams:
    return SiftParams(3, 1.6, 0.04, 10.0, 1, max_keypoints)


def match_params() -> MatchParams:
    return MatchParams(1.0, 0.6)


def ransac_params(trials: int = 1000, seed: int = 0x5EED) -> RansacParams:
    """estworldpose defaults as VO.m:123-127 calls it (MaxNumTrials 1000); the BASELINE
    configs[2] bench uses trials=2048."""
    return RansacParams(trials, 99.0, 1.0, seed)


def calib_from(P1: np.ndarray, P2: np.ndarray) -> Calib:
    c = Calib()
    c.P1[:] = [float(v) for v in np.asarray(P1, np.float64).reshape(-1)]
    c.P2[:] = [float(v) for v in np.asarray(P2, np.float64).reshape(-1)]
    K = np.asarray(P1, np.float64)[:, :3]
    c.K[:] = [float(v) for v in K.reshape(-1)]
    return c


_libs: dict = {}


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib(cv: bool = False):
    path = LIB_CV if cv else LIB
    if path not in _libs:
        if not path.exists():
            build()
        L = C.CDLL(str(path))
        P = C.POINTER
        L.oracle_sift.argtypes = [P(C.c_uint8), C.c_int, C.c_int, C.c_int, P(SiftParams), P(Keypoint), P(C.c_uint8), C.c_int]
        L.oracle_sift.restype = C.c_int
        L.oracle_gauss_kernel.argtypes = [C.c_double, P(C.c_float), C.c_int]
        L.oracle_gauss_kernel.restype = C.c_int
        L.oracle_blur.argtypes = [P(C.c_float), P(C.c_float), C.c_int, C.c_int, P(C.c_float), C.c_int]
        L.oracle_upsample.argtypes = [P(C.c_uint8), C.c_int, C.c_int, C.c_int, P(C.c_float)]
        L.oracle_num_octaves.argtypes = [C.c_int, C.c_int, C.c_int]
        L.oracle_pyramid.argtypes = [P(C.c_uint8), C.c_int, C.c_int, C.c_int, P(SiftParams), P(C.c_float)]
        L.oracle_pyramid.restype = C.c_long
        L.oracle_match.argtypes = [P(C.c_uint8), C.c_int, P(C.c_uint8), C.c_int, P(MatchParams), P(C.c_uint32), C.c_int]
        L.oracle_match_f32.argtypes = [P(C.c_float), C.c_int, C.c_int, P(C.c_float), C.c_int, C.c_int, C.c_int,
                                       P(MatchParams), P(C.c_uint32), C.c_int]
        L.oracle_track.argtypes = [P(C.c_uint8), P(C.c_uint8), C.c_int, P(C.c_uint8), C.c_int, P(C.c_uint8), C.c_int,
                                   P(MatchParams), P(C.c_uint32), C.c_int]
        L.oracle_triangulate.argtypes = [P(C.c_float), P(C.c_float), C.c_int, P(C.c_double), P(C.c_double), P(C.c_double)]
        L.oracle_triangulate.restype = None
        L.oracle_p3p.argtypes = [P(C.c_double), P(C.c_double), P(C.c_double), P(C.c_double), P(C.c_double)]
        L.oracle_estworldpose.argtypes = [P(C.c_double), P(C.c_double), C.c_int, P(C.c_double), P(RansacParams), C.c_uint32,
                                          P(C.c_double), P(C.c_uint8), P(C.c_int)]
        L.oracle_landmarks.argtypes = [P(C.c_float), P(C.c_float), C.c_int, P(C.c_float), P(C.c_float), C.c_int,
                                       P(C.c_double), P(C.c_double), P(C.c_double), P(C.c_double), C.c_int]
        L.oracle_run_sequence.argtypes = [P(C.c_uint8), P(C.c_uint8), C.c_int, C.c_int, C.c_int, P(Calib), P(SiftParams),
                                          P(MatchParams), P(RansacParams), P(StepOut), P(C.c_double), C.c_long,
                                          C.c_uint32, P(C.c_float), P(C.c_uint8)]
        L.oracle_landmarks_to_world.argtypes = [P(C.c_double), P(C.c_float), P(C.c_uint8), C.c_int, P(C.c_double)]
        L.oracle_landmarks_to_world.restype = None
        L.oracle_spec_eval.argtypes = [C.c_int, P(C.c_double), P(C.c_double), C.c_int]
        L.oracle_spec_eval.restype = None
        L.oracle_philox.argtypes = [C.c_uint32] * 6 + [P(C.c_uint32)]
        L.oracle_spec_check_expf_nonpos.argtypes = []
        L.oracle_spec_check_expf_nonpos.restype = C.c_long
        L.oracle_philox.restype = None
        L.oracle_gauss_radius.argtypes = [C.c_double]
        L.oracle_run_sequence.restype = C.c_long
        L.oracle_sift_match_pair.argtypes = [P(C.c_uint8), P(C.c_uint8), C.c_int, C.c_int, P(SiftParams), P(MatchParams),
                                             P(C.c_int), P(C.c_int)]
        _libs[path] = L
    return _libs[path]


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def sift(img: np.ndarray, params: SiftParams | None = None, cv: bool = False):
    """-> (keypoints structured array, descriptors [n,128] u8)"""
    img = np.ascontiguousarray(img, np.uint8)
    p = params or sift_params()
    cap = p.max_keypoints
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 128), np.uint8)
    n = lib(cv).oracle_sift(_p(img, C.c_uint8), img.shape[0], img.shape[1], img.shape[1], C.byref(p),
                          kps.ctypes.data_as(C.POINTER(Keypoint)), _p(desc, C.c_uint8), cap)
    n = min(n, cap)
    return kps[:n].copy(), desc[:n].copy()


def gauss_kernel(sigma: float) -> np.ndarray:
    k = np.zeros(64, np.float32)
    r = lib().oracle_gauss_kernel(sigma, _p(k, C.c_float), 64)
    return k[: r + 1].copy()


def blur(img: np.ndarray, sigma: float) -> np.ndarray:
    img = np.ascontiguousarray(img, np.float32)
    k = gauss_kernel(sigma)
    out = np.empty_like(img)
    lib().oracle_blur(_p(img, C.c_float), _p(out, C.c_float), img.shape[0], img.shape[1], _p(k, C.c_float), len(k) - 1)
    return out


def upsample(img: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    out = np.empty((img.shape[0] * 2, img.shape[1] * 2), np.float32)
    lib().oracle_upsample(_p(img, C.c_uint8), img.shape[0], img.shape[1], img.shape[1], _p(out, C.c_float))
    return out


def pyramid(img: np.ndarray, params: SiftParams | None = None) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    p = params or sift_params()
    n = lib().oracle_pyramid(_p(img, C.c_uint8), img.shape[0], img.shape[1], img.shape[1], C.byref(p), None)
    out = np.empty(n, np.float32)
    lib().oracle_pyramid(_p(img, C.c_uint8), img.shape[0], img.shape[1], img.shape[1], C.byref(p), _p(out, C.c_float))
    return out


def match(F1: np.ndarray, F2: np.ndarray, params: MatchParams | None = None, cv: bool = False) -> np.ndarray:
    F1 = np.ascontiguousarray(F1, np.uint8)
    F2 = np.ascontiguousarray(F2, np.uint8)
    cap = max(F1.shape[0], 1)
    pairs = np.zeros((cap, 2), np.uint32)
    n = lib(cv).oracle_match(_p(F1, C.c_uint8), F1.shape[0], _p(F2, C.c_uint8), F2.shape[0],
                           C.byref(params or match_params()), _p(pairs, C.c_uint32), cap)
    return pairs[:n].copy()


def match_f32(F1: np.ndarray, F2: np.ndarray, params: MatchParams | None = None) -> np.ndarray:
    """matchFeatures on general single features (the float spec of libvo vo_match_f32):
    1-based uint32 (P, 2).  Rows are passed row-major (ld = 128)."""
    F1 = np.ascontiguousarray(F1, np.float32).reshape(-1, 128)
    F2 = np.ascontiguousarray(F2, np.float32).reshape(-1, 128)
    cap = max(F1.shape[0], 1)
    pairs = np.zeros((cap, 2), np.uint32)
    n = lib().oracle_match_f32(_p(F1, C.c_float), F1.shape[0], 128, _p(F2, C.c_float), F2.shape[0], 128, 0,
                               C.byref(params or match_params()), _p(pairs, C.c_uint32), cap)
    return pairs[:n].copy()


def track(old_l, old_r, cur_l, cur_r, params: MatchParams | None = None) -> np.ndarray:
    arrs = [np.ascontiguousarray(a, np.uint8) for a in (old_l, old_r, cur_l, cur_r)]
    cap = max(a.shape[0] for a in arrs) + 1
    idx = np.zeros((cap, 3), np.uint32)
    n = lib().oracle_track(_p(arrs[0], C.c_uint8), _p(arrs[1], C.c_uint8), arrs[0].shape[0],
                           _p(arrs[2], C.c_uint8), arrs[2].shape[0], _p(arrs[3], C.c_uint8), arrs[3].shape[0],
                           C.byref(params or match_params()), _p(idx, C.c_uint32), cap)
    return idx[:n].copy()


def triangulate(x1, x2, P1, P2) -> np.ndarray:
    x1 = np.ascontiguousarray(x1, np.float32).reshape(-1, 2)
    x2 = np.ascontiguousarray(x2, np.float32).reshape(-1, 2)
    P1 = np.ascontiguousarray(P1, np.float64)
    P2 = np.ascontiguousarray(P2, np.float64)
    X = np.zeros((x1.shape[0], 3))
    lib().oracle_triangulate(_p(x1, C.c_float), _p(x2, C.c_float), x1.shape[0], _p(P1, C.c_double),
                             _p(P2, C.c_double), _p(X, C.c_double))
    return X


def p3p(img3, world3, K):
    img3 = np.ascontiguousarray(img3, np.float64)
    world3 = np.ascontiguousarray(world3, np.float64)
    K = np.ascontiguousarray(K, np.float64)
    Rs = np.zeros((4, 9))
    ts = np.zeros((4, 3))
    n = lib().oracle_p3p(_p(img3, C.c_double), _p(world3, C.c_double), _p(K, C.c_double), _p(Rs, C.c_double),
                         _p(ts, C.c_double))
    return Rs[:n].reshape(-1, 3, 3), ts[:n]


def estworldpose(img, world, K, params: RansacParams | None = None, frame_key: int = 0):
    img = np.ascontiguousarray(img, np.float64)
    world = np.ascontiguousarray(world, np.float64)
    K = np.ascontiguousarray(K, np.float64)
    T = np.zeros(16)
    inl = np.zeros(max(img.shape[0], 1), np.uint8)
    nin = C.c_int(0)
    st = lib().oracle_estworldpose(_p(img, C.c_double), _p(world, C.c_double), img.shape[0], _p(K, C.c_double),
                                   C.byref(params or ransac_params()), frame_key, _p(T, C.c_double),
                                   _p(inl, C.c_uint8), C.byref(nin))
    return st, T.reshape(4, 4), inl[: img.shape[0]].astype(bool), nin.value


def landmarks(l_pos, r_pos, old_l, old_r, P1, P2, pose):
    a = [np.ascontiguousarray(x, np.float32).reshape(-1, 2) for x in (l_pos, r_pos, old_l, old_r)]
    P1 = np.ascontiguousarray(P1, np.float64)
    P2 = np.ascontiguousarray(P2, np.float64)
    pose = np.ascontiguousarray(pose, np.float64)
    cap = a[0].shape[0] + 2
    out = np.zeros((cap, 3))
    rows = lib().oracle_landmarks(_p(a[0], C.c_float), _p(a[1], C.c_float), a[0].shape[0], _p(a[2], C.c_float),
                                  _p(a[3], C.c_float), a[2].shape[0], _p(P1, C.c_double), _p(P2, C.c_double),
                                  _p(pose, C.c_double), _p(out, C.c_double), cap)
    return out[:rows].copy()


STEP_DTYPE = np.dtype([("status", "<i4"), ("n_left", "<i4"), ("n_right", "<i4"), ("n_stereo", "<i4"),
                       ("n_tracked", "<i4"), ("n_inliers", "<i4"), ("n_landmarks", "<i4"), ("flags", "<i4"),
                       ("rel_pose", "<f8", (4, 4)), ("pose", "<f8", (4, 4))])


def run_sequence(L, R, P1, P2, sp=None, mp=None, rp=None, lm_cap: int = 1 << 20, key0: int = 0,
                 camera_rows: bool = False, cv: bool = False):
    """VO.m loop -> (outs, landmarks [L, 3] world); with camera_rows=True the landmark rows
    stay in the camera frame: (outs, (X [L, 3] float32, keep [L] bool))."""
    L = np.ascontiguousarray(L, np.uint8)
    R = np.ascontiguousarray(R, np.uint8)
    F, rows, cols = L.shape
    outs = np.zeros(F, STEP_DTYPE)
    lm = np.zeros((lm_cap, 3))
    cal = calib_from(P1, P2)
    X = np.zeros((lm_cap, 3), np.float32) if camera_rows else None
    keep = np.zeros(lm_cap, np.uint8) if camera_rows else None
    n = lib(cv).oracle_run_sequence(_p(L, C.c_uint8), _p(R, C.c_uint8), F, rows, cols, C.byref(cal),
                                  C.byref(sp or sift_params()), C.byref(mp or match_params()),
                                  C.byref(rp or ransac_params()), outs.ctypes.data_as(C.POINTER(StepOut)),
                                  _p(lm, C.c_double), lm_cap, key0,
                                  _p(X, C.c_float) if camera_rows else None,
                                  _p(keep, C.c_uint8) if camera_rows else None)
    if camera_rows:
        return outs, (X[:n].copy(), keep[:n].astype(bool))
    return outs, lm[:n].copy()


def landmarks_to_world(pose, X, keep) -> np.ndarray:
    """CreateLandmarksFromFeatures.m:17 on camera-frame rows (keep=False: zero row)."""
    pose = np.ascontiguousarray(pose, np.float64).reshape(4, 4)
    X = np.ascontiguousarray(X, np.float32).reshape(-1, 3)
    k = np.ascontiguousarray(keep, np.uint8).reshape(-1)
    out = np.zeros((X.shape[0], 3))
    lib().oracle_landmarks_to_world(_p(pose, C.c_double), _p(X, C.c_float), _p(k, C.c_uint8), X.shape[0],
                                    _p(out, C.c_double))
    return out


def sift_match_pair(left, right, sp=None, mp=None):
    left = np.ascontiguousarray(left, np.uint8)
    right = np.ascontiguousarray(right, np.uint8)
    nl, nr = C.c_int(0), C.c_int(0)
    S = lib().oracle_sift_match_pair(_p(left, C.c_uint8), _p(right, C.c_uint8), left.shape[0], left.shape[1],
                                     C.byref(sp or sift_params()), C.byref(mp or match_params()),
                                     C.byref(nl), C.byref(nr))
    return S, nl.value, nr.value


SPEC_FN = {"expf": 0, "atan2_deg": 1, "sin_deg": 2, "cos_deg": 3, "exp_d": 4, "log_d": 5, "rcp_nr": 6, "sift_wt": 7}


def spec_check_expf_nonpos() -> int:
    """Mismatching floats of vo_expf_nonpos vs vo_expf over every float in [-87, 0]."""
    return int(lib().oracle_spec_check_expf_nonpos())


def spec_eval(fn: str, x) -> np.ndarray:
    """Evaluate a vo_spec.h primitive (float ones are computed in float)."""
    x = np.ascontiguousarray(x, np.float64).reshape(-1)
    n = x.shape[0] // 2 if fn in ("atan2_deg", "sift_wt") else x.shape[0]   # atan2: (y, x) pairs; sift_wt: (s, k)
    out = np.zeros(n)
    lib().oracle_spec_eval(SPEC_FN[fn], _p(x, C.c_double), _p(out, C.c_double), n)
    return out


def philox(ctr, key) -> np.ndarray:
    out = np.zeros(4, np.uint32)
    lib().oracle_philox(*[int(v) for v in ctr], int(key[0]), int(key[1]), _p(out, C.c_uint32))
    return out
