"""Python host mirror of the reference's per-frame call surface, over the
libvo C-ABI (include/vo.h).

The reference (VO.m) calls MathWorks toolbox functions; this module exposes
the same names with the same argument meaning and error behaviour, each
running on the MI355X through libvo.so:

    detectSIFTFeatures / extractFeatures   VO.m:79-84
    matchFeatures                          VO.m:87,283,293,311,323
    find_remaining_points                  VO.m:280-334
    triangulate                            VO.m:113-116
    estworldpose                           VO.m:123-127
    CreateLandmarksFromFeatures            CreateLandmarksFromFeatures.m:1-21
    VisualOdometry.step                    the VO.m loop body (VO.m:70-161)

Coordinates are MATLAB 1-based.  Index pairs are 1-based uint32 (P x 2).
There is no CPU fallback: if libvo.so cannot be loaded or no GPU is present,
every call raises VOError.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG = Path(__file__).resolve().parent
LIBPATH = PKG / "lib" / "libvo.so"

VO_OK = 0
VO_ERR_ARG = -1
VO_ERR_HIP = -2
VO_ERR_TOO_FEW_POINTS = -3
VO_ERR_NO_CONSENSUS = -4
VO_ERR_CAPACITY = -5
VO_ERR_STATE = -6
STEP_DEPTH = 3            # VO_STEP_DEPTH: batches vo_step_submit_dev keeps in flight


class VOError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libvo error {code}: {msg}")
        self.code = code


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


class PairStats(C.Structure):
    _fields_ = [("n_left", C.c_int32), ("n_right", C.c_int32), ("n_stereo", C.c_int32), ("flags", C.c_int32)]


KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4"), ("layer", "<i4"), ("scale", "<f4")])
STEP_DTYPE = np.dtype([("status", "<i4"), ("n_left", "<i4"), ("n_right", "<i4"), ("n_stereo", "<i4"),
                       ("n_tracked", "<i4"), ("n_inliers", "<i4"), ("n_landmarks", "<i4"), ("flags", "<i4"),
                       ("rel_pose", "<f8", (4, 4)), ("pose", "<f8", (4, 4))])

# exported symbols (tests check the library exports every one)
EXPORTS = [
    "vo_default_sift_params", "vo_default_match_params", "vo_default_ransac_params", "vo_create", "vo_destroy",
    "vo_set_calib", "vo_last_error", "vo_sift", "vo_match", "vo_track", "vo_triangulate", "vo_estworldpose",
    "vo_landmarks", "vo_step", "vo_step_batch", "vo_step_batch_dev", "vo_step_submit_dev", "vo_step_collect",
    "vo_steps_pending", "vo_fetch_tracks", "vo_get_landmarks", "vo_reset",
    "vo_sift_match_batch_dev", "vo_fetch_keypoints", "vo_fetch_stereo_pairs", "vo_fetch_gaussian", "vo_stream", "vo_set_profiling",
    "vo_kernel_times", "vo_set_frame_index", "vo_set_concurrency",
    "vo_set_landmark_frame", "vo_get_landmark_rows", "vo_landmarks_to_world", "vo_match_f32",
    "vo_sift_ex", "vo_step_batch_ex", "vo_chain_poses", "vo_landmarks_to_world_frames", "vo_landmarks_world_dev",
    "vo_fetch_candidate_counts",
]

# the test build (csrc `make exp`, -DVO_EXPERIMENTAL=1): libvo plus the experimental kernels kept
# as cross-checks (fused octave, eager MSAC), selected by its extra export vo_exp_set.  Only the
# parity tests load it (load_experimental_library); the product path never does.
EXP_LIBPATH = PKG / "lib" / "libvo_exp.so"

_libs: dict = {}


def load_library(path: str | os.PathLike | None = None):
    """Load libvo.so (built in-tree by __graft_entry__.build()).  Raises if absent.  One handle
    per path (the default path, or $VO_LIBPATH, unless `path` is given)."""
    p = Path(path) if path else Path(os.environ.get("VO_LIBPATH", LIBPATH))
    key = str(p.resolve()) if p.exists() else str(p)
    if key in _libs:
        return _libs[key]
    if not p.exists():
        raise VOError(VO_ERR_STATE, f"{p} not built; run __graft_entry__.build() (make -C csrc)")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same
    # soname as /opt/rocm's).  Loading torch first makes libvo bind to that
    # runtime, so device pointers from torch tensors and torch.distributed
    # (RCCL) share one runtime with libvo.  Without torch, libvo uses /opt/rocm.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(str(p))
    P = C.POINTER
    vp = C.c_void_p
    L.vo_default_sift_params.argtypes = [P(SiftParams)]
    L.vo_default_match_params.argtypes = [P(MatchParams)]
    L.vo_default_ransac_params.argtypes = [P(RansacParams)]
    L.vo_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, P(Calib), P(SiftParams), P(MatchParams), P(RansacParams)]
    L.vo_create.restype = vp
    L.vo_destroy.argtypes = [vp]
    L.vo_destroy.restype = None
    L.vo_set_calib.argtypes = [vp, P(Calib)]
    L.vo_last_error.argtypes = [vp]
    L.vo_last_error.restype = C.c_char_p
    L.vo_sift.argtypes = [vp, P(C.c_uint8), C.c_int, C.c_int, C.c_int, P(Keypoint), P(C.c_uint8), C.c_int, P(C.c_int)]
    L.vo_match.argtypes = [vp, P(C.c_uint8), C.c_int, P(C.c_uint8), C.c_int, P(C.c_uint32), C.c_int, P(C.c_int)]
    L.vo_sift_ex.argtypes = [vp, P(C.c_uint8), C.c_int, C.c_int, C.c_int, C.c_int, P(Keypoint), P(C.c_uint8), C.c_int,
                             P(C.c_int)]
    L.vo_step_batch_ex.argtypes = [vp, P(C.c_uint8), P(C.c_uint8), C.c_int, C.c_int, C.c_int, P(StepOut)]
    L.vo_match_f32.argtypes = [vp, P(C.c_float), C.c_int, C.c_int, P(C.c_float), C.c_int, C.c_int, C.c_int,
                               P(C.c_uint32), C.c_int, P(C.c_int)]
    L.vo_track.argtypes = [vp, P(C.c_uint8), P(C.c_uint8), C.c_int, P(C.c_uint8), C.c_int, P(C.c_uint8), C.c_int,
                           P(C.c_uint32), C.c_int, P(C.c_int)]
    L.vo_triangulate.argtypes = [vp, P(C.c_float), P(C.c_float), C.c_int, P(C.c_double), P(C.c_double), P(C.c_double)]
    L.vo_estworldpose.argtypes = [vp, P(C.c_double), P(C.c_double), C.c_int, P(C.c_double), P(RansacParams),
                                  C.c_uint32, P(C.c_double), P(C.c_uint8), P(C.c_int)]
    L.vo_landmarks.argtypes = [vp, P(C.c_float), P(C.c_float), C.c_int, P(C.c_float), P(C.c_float), C.c_int,
                               P(C.c_double), P(C.c_double), C.c_int, P(C.c_int)]
    L.vo_step.argtypes = [vp, P(C.c_uint8), P(C.c_uint8), C.c_int, P(StepOut)]
    L.vo_step_batch.argtypes = [vp, P(C.c_uint8), P(C.c_uint8), C.c_int, C.c_int, P(StepOut)]
    L.vo_step_batch_dev.argtypes = [vp, vp, vp, C.c_int, P(StepOut)]
    L.vo_step_submit_dev.argtypes = [vp, vp, vp, C.c_int]
    L.vo_step_collect.argtypes = [vp, P(StepOut), C.c_int, P(C.c_int)]
    L.vo_steps_pending.argtypes = [vp]
    L.vo_fetch_tracks.argtypes = [vp, C.c_int, P(C.c_float), P(C.c_float), P(C.c_double), P(C.c_float), C.c_int,
                                  P(C.c_int), P(C.c_int)]
    L.vo_get_landmarks.argtypes = [vp, P(C.c_double), C.c_int, P(C.c_int)]
    L.vo_reset.argtypes = [vp]
    L.vo_set_frame_index.argtypes = [vp, C.c_long]
    L.vo_sift_match_batch_dev.argtypes = [vp, vp, vp, C.c_int, P(PairStats)]
    L.vo_fetch_keypoints.argtypes = [vp, C.c_int, P(Keypoint), P(C.c_uint8), C.c_int, P(C.c_int)]
    L.vo_fetch_stereo_pairs.argtypes = [vp, C.c_int, P(C.c_uint32), C.c_int, P(C.c_int)]
    L.vo_fetch_candidate_counts.argtypes = [vp, C.c_int, P(C.c_int), P(C.c_int)]
    L.vo_fetch_gaussian.argtypes = [vp, C.c_int, C.c_int, C.c_int, P(C.c_float), C.c_int, P(C.c_int), P(C.c_int)]
    L.vo_stream.argtypes = [vp]
    L.vo_stream.restype = vp
    L.vo_set_profiling.argtypes = [vp, C.c_int]
    L.vo_set_concurrency.argtypes = [vp, C.c_int]
    L.vo_set_landmark_frame.argtypes = [vp, C.c_int]
    L.vo_get_landmark_rows.argtypes = [vp, P(C.c_float), P(C.c_uint8), C.c_int, P(C.c_int)]
    L.vo_landmarks_to_world.argtypes = [P(C.c_double), P(C.c_float), P(C.c_uint8), C.c_int, P(C.c_double)]
    L.vo_landmarks_to_world_frames.argtypes = [P(C.c_double), P(C.c_int32), C.c_int, P(C.c_float), P(C.c_uint8), C.c_long,
                                               P(C.c_double)]
    L.vo_chain_poses.argtypes = [P(C.c_double), P(C.c_int32), C.c_int, P(C.c_double), P(C.c_double)]
    L.vo_landmarks_world_dev.argtypes = [vp, P(C.c_double), C.c_int, vp, C.c_long, P(C.c_long)]
    L.vo_kernel_times.argtypes = [vp, P(C.c_char_p), P(C.c_double), P(C.c_int), C.c_int, P(C.c_int)]
    _libs[key] = L
    return L


def experimental_library_path() -> Path:
    """libvo_exp.so beside the product library in use: the in-tree test build, or -- when
    $VO_LIBPATH points at another libvo.so (a variant build) -- the libvo_exp.so next to it, so an
    experimental cross-check compares a build with its own test build."""
    lp = os.environ.get("VO_LIBPATH")
    return Path(lp).resolve().parent / "libvo_exp.so" if lp else EXP_LIBPATH


def load_experimental_library():
    """The test build libvo_exp.so (experimental_library_path()) with `vo_exp_set(fused_octave,
    msac_eager)` bound; pass it to Context(lib=...).  Raises VOError if it is not built."""
    L = load_library(experimental_library_path())
    if not hasattr(L, "vo_exp_set"):
        raise VOError(VO_ERR_STATE, f"{experimental_library_path()} lacks vo_exp_set (not a VO_EXPERIMENTAL build)")
    L.vo_exp_set.argtypes = [C.c_int, C.c_int]
    return L


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def default_sift_params(max_keypoints: int = 16384) -> SiftParams:
    p = SiftParams()
    load_library().vo_default_sift_params(C.byref(p))
    p.max_keypoints = max_keypoints
    return p


def default_match_params() -> MatchParams:
    p = MatchParams()
    load_library().vo_default_match_params(C.byref(p))
    return p


def default_ransac_params() -> RansacParams:
    p = RansacParams()
    load_library().vo_default_ransac_params(C.byref(p))
    return p


def calib_from(P1, P2, K=None) -> Calib:
    c = Calib()
    c.P1[:] = [float(v) for v in np.asarray(P1, np.float64).reshape(-1)]
    c.P2[:] = [float(v) for v in np.asarray(P2, np.float64).reshape(-1)]
    K = np.asarray(P1, np.float64)[:, :3] if K is None else np.asarray(K, np.float64)
    c.K[:] = [float(v) for v in K.reshape(-1)]
    return c


class Context:
    """One libvo context (one HIP device, fixed image size, up to max_batch frames per call)."""

    def __init__(self, rows: int = 375, cols: int = 1242, max_batch: int = 1, device: int = 0, calib: Calib | None = None,
                 sift: SiftParams | None = None, match: MatchParams | None = None, ransac: RansacParams | None = None,
                 lib=None):
        self.lib = lib if lib is not None else load_library()
        self.rows, self.cols, self.max_batch = rows, cols, max_batch
        self.sift_params = sift or default_sift_params()
        self.match_params = match or default_match_params()
        self.ransac_params = ransac or default_ransac_params()
        h = self.lib.vo_create(device, rows, cols, max_batch, C.byref(calib) if calib else None,
                               C.byref(self.sift_params), C.byref(self.match_params), C.byref(self.ransac_params))
        if not h:
            raise VOError(VO_ERR_HIP, self.lib.vo_last_error(None).decode())
        self.h = C.c_void_p(h)

    def close(self):
        if getattr(self, "h", None):
            self.lib.vo_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, allow=()):
        if rc != VO_OK and rc not in allow:
            raise VOError(rc, self.lib.vo_last_error(self.h).decode())
        return rc

    # ---- detectSIFTFeatures + extractFeatures ----
    def sift(self, img: np.ndarray):
        """A Fortran-ordered image (MATLAB's layout) goes to vo_sift_ex untransposed."""
        img = np.asarray(img, np.uint8)
        if img.ndim != 2:
            raise VOError(VO_ERR_ARG, "sift: a 2-D uint8 image")
        rows, cols = img.shape
        # zero-copy only for positive strides the ABI can express (ld >= rows column-major,
        # ld >= cols row-major); flipped or otherwise strided views are packed first
        if rows > 1 and img.strides[0] == 1 and img.strides[1] >= rows:
            col_major, ld = 1, img.strides[1]
        elif img.strides[1] == 1 and img.strides[0] >= cols:
            col_major, ld = 0, img.strides[0]
        else:
            img = np.ascontiguousarray(img)
            col_major, ld = 0, cols
        cap = self.sift_params.max_keypoints
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 128), np.uint8)
        n = C.c_int(0)
        self._check(self.lib.vo_sift_ex(self.h, _p(img, C.c_uint8), img.shape[0], img.shape[1], ld, col_major,
                                        kps.ctypes.data_as(C.POINTER(Keypoint)), _p(desc, C.c_uint8), cap, C.byref(n)))
        return kps[: n.value].copy(), desc[: n.value].copy()

    # ---- matchFeatures ----
    def match(self, F1: np.ndarray, F2: np.ndarray) -> np.ndarray:
        F1 = np.ascontiguousarray(F1, np.uint8)
        F2 = np.ascontiguousarray(F2, np.uint8)
        cap = max(F1.shape[0], 1)
        pairs = np.zeros((cap, 2), np.uint32)
        n = C.c_int(0)
        self._check(self.lib.vo_match(self.h, _p(F1, C.c_uint8), F1.shape[0], _p(F2, C.c_uint8), F2.shape[0],
                                      _p(pairs, C.c_uint32), cap, C.byref(n)))
        return pairs[: n.value].copy()

    def match_f32(self, F1: np.ndarray, F2: np.ndarray) -> np.ndarray:
        """matchFeatures on single-precision n x 128 matrices in their own storage order
        (vo_match_f32): a Fortran-ordered array (MATLAB's layout) goes through without a
        transpose, a C-ordered one (any row stride) likewise."""
        def view(F):
            F = np.asarray(F)
            if F.dtype != np.float32 or F.ndim != 2 or F.shape[1] != 128:
                raise VOError(VO_ERR_ARG, "match_f32: n x 128 float32 matrices")
            if F.strides[0] == 4 and F.strides[1] % 4 == 0 and F.shape[0] > 0:       # column-major
                return F, F.strides[1] // 4, 1
            if F.strides[1] == 4 and F.strides[0] % 4 == 0:
                return F, max(F.strides[0] // 4, 128), 0
            F = np.ascontiguousarray(F)
            return F, 128, 0
        (A, la, ca), (B, lb, cb) = view(F1), view(F2)
        if A.shape[0] and B.shape[0] and ca != cb:
            B, lb, cb = (np.asfortranarray(B), B.shape[0], 1) if ca else (np.ascontiguousarray(B), 128, 0)
        order = ca if A.shape[0] else cb
        cap = max(A.shape[0], 1)
        pairs = np.zeros((cap, 2), np.uint32)
        n = C.c_int(0)
        pa = A.ctypes.data_as(C.POINTER(C.c_float)) if A.shape[0] else None
        pb = B.ctypes.data_as(C.POINTER(C.c_float)) if B.shape[0] else None
        self._check(self.lib.vo_match_f32(self.h, pa, A.shape[0], la, pb, B.shape[0], lb, order,
                                          _p(pairs, C.c_uint32), cap, C.byref(n)))
        return pairs[: n.value].copy()

    # ---- benchmark workload: SIFT + stereo match of B pairs resident on device ----
    def sift_match_batch_dev(self, d_lefts: int, d_rights: int, B: int, stats: bool = True):
        st = (PairStats * B)() if stats else None
        self._check(self.lib.vo_sift_match_batch_dev(self.h, C.c_void_p(d_lefts), C.c_void_p(d_rights), B, st))
        if stats:
            return [(s.n_left, s.n_right, s.n_stereo, s.flags) for s in st]
        return None

    def fetch_keypoints(self, image: int, descriptors: bool = True):
        """(keypoints, descriptors) of `image` in the last batched call; descriptors=False
        skips the descriptor copy (returns None for them)."""
        cap = self.sift_params.max_keypoints
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 128), np.uint8) if descriptors else None
        n = C.c_int(0)
        self._check(self.lib.vo_fetch_keypoints(self.h, image, kps.ctypes.data_as(C.POINTER(Keypoint)),
                                                _p(desc, C.c_uint8) if descriptors else None, cap, C.byref(n)))
        m = min(n.value, cap)
        return kps[:m].copy(), (desc[:m].copy() if descriptors else None)

    def fetch_candidate_counts(self, image: int) -> tuple[int, int]:
        """(extremum candidates, candidates accepted by the refinement) of `image` in the last
        batched call (vo_fetch_candidate_counts)."""
        nc, na = C.c_int(0), C.c_int(0)
        self._check(self.lib.vo_fetch_candidate_counts(self.h, image, C.byref(nc), C.byref(na)))
        return nc.value, na.value

    def fetch_stereo_pairs(self, frame: int) -> np.ndarray:
        cap = self.sift_params.max_keypoints
        pairs = np.zeros((cap, 2), np.uint32)
        n = C.c_int(0)
        self._check(self.lib.vo_fetch_stereo_pairs(self.h, frame, _p(pairs, C.c_uint32), cap, C.byref(n)))
        return pairs[: min(n.value, cap)].copy()

    def fetch_gaussian(self, image: int, octave: int, level: int) -> np.ndarray:
        """Gaussian level G(octave, level) of image `image` of the last batched call (diagnostic)."""
        r, c = C.c_int(0), C.c_int(0)
        self._check(self.lib.vo_fetch_gaussian(self.h, image, octave, level, None, 0, C.byref(r), C.byref(c)))
        out = np.empty((r.value, c.value), np.float32)
        self._check(self.lib.vo_fetch_gaussian(self.h, image, octave, level, _p(out, C.c_float), out.size, None, None))
        return out

    # ---- find_remaining_points ----
    def track(self, old_l, old_r, cur_l, cur_r) -> np.ndarray:
        """-> idx [K, 3] 1-based rows {old_row, cur_left_row, cur_right_row}."""
        a = [np.ascontiguousarray(x, np.uint8).reshape(-1, 128) for x in (old_l, old_r, cur_l, cur_r)]
        cap = max(x.shape[0] for x in a) + 1
        idx = np.zeros((cap, 3), np.uint32)
        n = C.c_int(0)
        self._check(self.lib.vo_track(self.h, _p(a[0], C.c_uint8), _p(a[1], C.c_uint8), a[0].shape[0],
                                      _p(a[2], C.c_uint8), a[2].shape[0], _p(a[3], C.c_uint8), a[3].shape[0],
                                      _p(idx, C.c_uint32), cap, C.byref(n)))
        return idx[: n.value].copy()

    # ---- triangulate ----
    def triangulate(self, x1, x2, P1, P2) -> np.ndarray:
        x1 = np.ascontiguousarray(x1, np.float32).reshape(-1, 2)
        x2 = np.ascontiguousarray(x2, np.float32).reshape(-1, 2)
        P1 = np.ascontiguousarray(P1, np.float64)
        P2 = np.ascontiguousarray(P2, np.float64)
        X = np.zeros((x1.shape[0], 3))
        self._check(self.lib.vo_triangulate(self.h, _p(x1, C.c_float), _p(x2, C.c_float), x1.shape[0],
                                            _p(P1, C.c_double), _p(P2, C.c_double), _p(X, C.c_double)))
        return X

    # ---- estworldpose ----
    def estworldpose(self, imagePoints, worldPoints, K, params: RansacParams | None = None, frame_key: int = 0,
                     raise_on_failure: bool = True):
        """-> (status, T 4x4 camera pose in world, inlier mask, n_inliers).  Like MATLAB,
        raises on < 4 points / no consensus unless raise_on_failure=False."""
        img = np.ascontiguousarray(imagePoints, np.float64).reshape(-1, 2)
        world = np.ascontiguousarray(worldPoints, np.float64).reshape(-1, 3)
        K = np.ascontiguousarray(K, np.float64)
        T = np.zeros(16)
        inl = np.zeros(max(img.shape[0], 1), np.uint8)
        nin = C.c_int(0)
        rc = self.lib.vo_estworldpose(self.h, _p(img, C.c_double), _p(world, C.c_double), img.shape[0], _p(K, C.c_double),
                                      C.byref(params) if params else None, frame_key, _p(T, C.c_double),
                                      _p(inl, C.c_uint8), C.byref(nin))
        if raise_on_failure:
            self._check(rc)
        else:
            self._check(rc, allow=(VO_ERR_TOO_FEW_POINTS, VO_ERR_NO_CONSENSUS))
        return rc, T.reshape(4, 4), inl[: img.shape[0]].astype(bool), nin.value

    # ---- new-landmark filter + CreateLandmarksFromFeatures ----
    def landmarks(self, l_pos, r_pos, old_l, old_r, pose) -> np.ndarray:
        a = [np.ascontiguousarray(x, np.float32).reshape(-1, 2) for x in (l_pos, r_pos, old_l, old_r)]
        pose = np.ascontiguousarray(pose, np.float64)
        cap = a[0].shape[0] + 2
        out = np.zeros((cap, 3))
        rows = C.c_int(0)
        self._check(self.lib.vo_landmarks(self.h, _p(a[0], C.c_float), _p(a[1], C.c_float), a[0].shape[0],
                                          _p(a[2], C.c_float), _p(a[3], C.c_float), a[2].shape[0],
                                          _p(pose, C.c_double), _p(out, C.c_double), cap, C.byref(rows)))
        return out[: rows.value].copy()

    # ---- the VO.m loop body ----
    def step_batch(self, lefts: np.ndarray, rights: np.ndarray, col_major: bool = False) -> np.ndarray:
        """B frames [B, rows, cols]; with col_major the frames are handed over in MATLAB's
        storage (each frame column-major: pixel (r, c) at c * rows + r)."""
        L, R = np.asarray(lefts, np.uint8), np.asarray(rights, np.uint8)
        B = L.shape[0]
        if col_major:
            L = np.ascontiguousarray(np.swapaxes(L, 1, 2))       # [B, cols, rows] = B column-major frames
            R = np.ascontiguousarray(np.swapaxes(R, 1, 2))
            ld = L.shape[2]
        else:
            L, R = np.ascontiguousarray(L), np.ascontiguousarray(R)
            ld = L.shape[2]
        outs = np.zeros(B, STEP_DTYPE)
        self._check(self.lib.vo_step_batch_ex(self.h, _p(L, C.c_uint8), _p(R, C.c_uint8), ld, 1 if col_major else 0, B,
                                              outs.ctypes.data_as(C.POINTER(StepOut))))
        return outs

    def step_batch_dev(self, d_lefts: int, d_rights: int, B: int) -> np.ndarray:
        outs = np.zeros(B, STEP_DTYPE)
        self._check(self.lib.vo_step_batch_dev(self.h, C.c_void_p(d_lefts), C.c_void_p(d_rights), B,
                                               outs.ctypes.data_as(C.POINTER(StepOut))))
        return outs

    def step_submit_dev(self, d_lefts: int, d_rights: int, B: int) -> None:
        """Pipelined step_batch_dev, device half (vo_step_submit_dev): returns at once."""
        self._check(self.lib.vo_step_submit_dev(self.h, C.c_void_p(d_lefts), C.c_void_p(d_rights), B))

    def step_collect(self) -> np.ndarray:
        """Outputs of the oldest submitted batch (vo_step_collect)."""
        outs = np.zeros(self.max_batch, STEP_DTYPE)
        n = C.c_int(0)
        self._check(self.lib.vo_step_collect(self.h, outs.ctypes.data_as(C.POINTER(StepOut)), self.max_batch, C.byref(n)))
        return outs[: n.value].copy()

    def steps_pending(self) -> int:
        return int(self.lib.vo_steps_pending(self.h))

    def fetch_tracks(self, frame: int) -> dict:
        """Visualisation data of `frame` of the last collected batch (vo_fetch_tracks):
        old_l / cur_l [K, 2] (1-based), world [K, 3], det [N, 2] (all current left detections)."""
        nt, nd = C.c_int(0), C.c_int(0)
        self._check(self.lib.vo_fetch_tracks(self.h, frame, None, None, None, None, 0, C.byref(nt), C.byref(nd)))
        cap = max(nt.value, nd.value, 1)
        old = np.zeros((cap, 2), np.float32)
        cur = np.zeros((cap, 2), np.float32)
        world = np.zeros((cap, 3))
        det = np.zeros((cap, 2), np.float32)
        self._check(self.lib.vo_fetch_tracks(self.h, frame, _p(old, C.c_float), _p(cur, C.c_float), _p(world, C.c_double),
                                             _p(det, C.c_float), cap, C.byref(nt), C.byref(nd)))
        k, n = nt.value, nd.value
        return {"old_l": old[:k].copy(), "cur_l": cur[:k].copy(), "world": world[:k].copy(), "det": det[:n].copy()}

    def step(self, left: np.ndarray, right: np.ndarray):
        return self.step_batch(left[None], right[None])[0]

    def get_landmarks(self) -> np.ndarray:
        rows = C.c_int(0)
        self._check(self.lib.vo_get_landmarks(self.h, None, 0, C.byref(rows)))
        out = np.zeros((max(rows.value, 1), 3))
        self._check(self.lib.vo_get_landmarks(self.h, _p(out, C.c_double), rows.value, C.byref(rows)))
        return out[: rows.value].copy()

    def set_landmark_frame(self, camera: bool):
        """Keep landmark rows in the camera frame (sharded sequences) instead of the world."""
        self._check(self.lib.vo_set_landmark_frame(self.h, 1 if camera else 0))

    def get_landmark_rows(self):
        """Camera-frame landmark rows appended so far -> (X [L, 3] float32, keep [L] bool)."""
        rows = C.c_int(0)
        self._check(self.lib.vo_get_landmark_rows(self.h, None, None, 0, C.byref(rows)))
        X = np.zeros((max(rows.value, 1), 3), np.float32)
        keep = np.zeros(max(rows.value, 1), np.uint8)
        self._check(self.lib.vo_get_landmark_rows(self.h, _p(X, C.c_float), _p(keep, C.c_uint8), rows.value,
                                                  C.byref(rows)))
        return X[: rows.value].copy(), keep[: rows.value].astype(bool)

    def landmark_row_count(self) -> int:
        """Camera-frame landmark rows held on the device (vo_set_landmark_frame(ctx, 1))."""
        rows = C.c_int(0)
        self._check(self.lib.vo_get_landmark_rows(self.h, None, None, 0, C.byref(rows)))
        return rows.value

    def landmarks_world_dev(self, poses, d_out: int, capacity: int) -> int:
        """CreateLandmarksFromFeatures.m:17 on the device (vo_landmarks_world_dev): the context's
        camera-frame rows moved to the world with poses[f], the chained world pose of its f-th
        collected frame, written as float32 [rows, 3] to device memory at d_out (e.g. a torch
        tensor's data_ptr(), `capacity` rows).  Returns the row count; d_out is ready on return."""
        P = np.ascontiguousarray(poses, np.float64).reshape(-1, 16)
        rows = C.c_long(0)
        self._check(self.lib.vo_landmarks_world_dev(self.h, _p(P, C.c_double), P.shape[0], C.c_void_p(d_out or None),
                                                    int(capacity), C.byref(rows)))
        return rows.value

    def reset(self):
        self._check(self.lib.vo_reset(self.h))

    def set_frame_index(self, idx: int):
        self._check(self.lib.vo_set_frame_index(self.h, idx))

    def set_calib(self, calib: Calib):
        self._check(self.lib.vo_set_calib(self.h, C.byref(calib)))

    # ---- profiling ----
    def set_profiling(self, on: bool):
        self._check(self.lib.vo_set_profiling(self.h, 1 if on else 0))

    def set_concurrency(self, n_streams: int):
        """Split each batch into n parts (1..4) pipelined over the scale-space and feature streams; results unchanged."""
        self._check(self.lib.vo_set_concurrency(self.h, int(n_streams)))

    def kernel_times(self) -> dict:
        n = C.c_int(0)
        self._check(self.lib.vo_kernel_times(self.h, None, None, None, 0, C.byref(n)))
        m = n.value
        names = (C.c_char_p * m)()
        ms = (C.c_double * m)()
        calls = (C.c_int * m)()
        self._check(self.lib.vo_kernel_times(self.h, names, ms, calls, m, C.byref(n)))
        return {names[i].decode(): (ms[i], calls[i]) for i in range(m)}

    def stream(self) -> int:
        return self.lib.vo_stream(self.h) or 0


def landmarks_to_world(pose, X, keep) -> np.ndarray:
    """CreateLandmarksFromFeatures.m:17 on camera-frame rows (vo_landmarks_to_world): rows with
    keep=False stay the reference's zero rows."""
    pose = np.ascontiguousarray(pose, np.float64).reshape(4, 4)
    X = np.ascontiguousarray(X, np.float32).reshape(-1, 3)
    k = np.ascontiguousarray(keep, np.uint8).reshape(-1)
    out = np.zeros((X.shape[0], 3))
    rc = load_library().vo_landmarks_to_world(_p(pose, C.c_double), _p(X, C.c_float), _p(k, C.c_uint8), X.shape[0],
                                               _p(out, C.c_double))
    if rc != VO_OK:
        raise VOError(rc, "vo_landmarks_to_world: bad arguments")
    return out


def chain_poses(rel, status=None, pose0=None) -> np.ndarray:
    """VO.m:130 world-pose chain (vo_chain_poses): frames with status != 0 hold the pose."""
    rel = np.ascontiguousarray(rel, np.float64).reshape(-1, 16)
    st = None if status is None else np.ascontiguousarray(status, np.int32).reshape(-1)
    p0 = None if pose0 is None else np.ascontiguousarray(pose0, np.float64).reshape(16)
    out = np.zeros((rel.shape[0], 16))
    rc = load_library().vo_chain_poses(_p(rel, C.c_double), None if st is None else _p(st, C.c_int32), rel.shape[0],
                                       None if p0 is None else _p(p0, C.c_double), _p(out, C.c_double))
    if rc != VO_OK:
        raise VOError(rc, "vo_chain_poses: bad arguments")
    return out.reshape(-1, 4, 4)


def landmarks_to_world_frames(poses, rows_per_frame, X, keep) -> np.ndarray:
    """CreateLandmarksFromFeatures.m:17 for a whole gathered sequence (vo_landmarks_to_world_frames)."""
    poses = np.ascontiguousarray(poses, np.float64).reshape(-1, 16)
    n = np.ascontiguousarray(rows_per_frame, np.int32).reshape(-1)
    X = np.ascontiguousarray(X, np.float32).reshape(-1, 3)
    k = np.ascontiguousarray(keep, np.uint8).reshape(-1)
    out = np.zeros((X.shape[0], 3))
    rc = load_library().vo_landmarks_to_world_frames(_p(poses, C.c_double), _p(n, C.c_int32), poses.shape[0],
                                                     _p(X, C.c_float), _p(k, C.c_uint8), X.shape[0], _p(out, C.c_double))
    if rc != VO_OK:
        raise VOError(rc, "vo_landmarks_to_world_frames: rows and per-frame counts disagree")
    return out


# ---------------------------------------------------------------------------
# MATLAB-named functional API (one shared default context per image size)
# ---------------------------------------------------------------------------
_ctx_cache: dict = {}


def _default_ctx(rows: int, cols: int) -> Context:
    key = (rows, cols)
    if key not in _ctx_cache:
        _ctx_cache[key] = Context(rows, cols, 1)
    return _ctx_cache[key]


def detectSIFTFeatures(I: np.ndarray):
    """detectSIFTFeatures(I) (VO.m:79-80) fused with its descriptor pass: returns
    (points, descriptors) where points is a structured array with MATLAB
    1-based Location (x, y), Scale, Orientation (angle), Metric (response)."""
    return _default_ctx(*I.shape).sift(I)


def extractFeatures(I: np.ndarray, points=None, Method: str = "SIFT"):
    """extractFeatures(I, points, "Method", "SIFT") (VO.m:83-84) -> (features, validPoints).
    SIFT descriptors are computed in the same device pass as detection; all
    points are valid."""
    if Method != "SIFT":
        raise VOError(VO_ERR_ARG, "only Method 'SIFT' is on the hot path")
    kps, desc = _default_ctx(*I.shape).sift(I)
    return desc, kps


def matchFeatures(features1: np.ndarray, features2: np.ndarray) -> np.ndarray:
    """matchFeatures defaults (Exhaustive, SSD, MatchThreshold 1, MaxRatio 0.6)."""
    return _default_ctx(375, 1242).match(features1, features2)
