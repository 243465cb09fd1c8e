"""The MATLAB MEX gateway (matlab/vo_mex.c) on the CPU: built against the minimal mx-API of
tests/mex_shim and a recording fake of libvo, so what is checked here is the gateway's own
work -- MATLAB's column-major storage handed to the C-ABI (images and N x 128 descriptors as they
lie, with the right ld / col_major), points and 3x4 / 3x3 / 4x4 matrices transposed, 1-based
index pairs, SIFTPoints Orientation in radians, estworldpose's status output, argument
validation and errors -- call by call as VO.m:79-87,113-127,160 make them.  tests/test_gpu_mex.py
runs the same gateway against the real libvo on the GPU."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

import mexshim

ROOT = Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module")
def mex():
    mexshim.build()
    m = mexshim.Mex(mexshim.FAKE)
    L = m.L
    L.fake_int.argtypes = [C.c_char_p]
    L.fake_dbl.argtypes = [C.c_char_p, C.c_int]
    L.fake_dbl.restype = C.c_double
    L.fake_img.argtypes = [C.c_int]
    L.fake_img.restype = C.c_void_p
    m.i = lambda k: L.fake_int(k.encode())
    m.d = lambda k, n: np.array([L.fake_dbl(k.encode(), j) for j in range(n)])
    m.img = lambda w, r, c: np.frombuffer(bytes((C.c_char * (r * c)).from_address(L.fake_img(w))), np.uint8).reshape(r, c)
    yield m
    m.at_exit()


def _P(seed):
    return np.random.default_rng(seed).normal(size=(3, 4))


def test_sift_hands_over_column_major_image(mex):
    I = np.random.default_rng(1).integers(0, 256, (20, 30), dtype=np.uint8)
    loc, scale, ori, metric, desc, octave, layer = mex.call("sift", I, nout=7)
    assert mex.i("ld") == 20 and mex.i("col_major") == 1            # ld = rows, MATLAB storage, no host transpose
    assert np.array_equal(mex.img(0, 20, 30), I)                      # pixel (r, c) read where MATLAB keeps it
    i = np.arange(5)
    assert loc.dtype == np.float32 and loc.shape == (5, 2)
    assert np.array_equal(loc[:, 0], (1.5 + i).astype(np.float32)) and np.array_equal(loc[:, 1], (2.25 + 3 * i).astype(np.float32))
    assert np.array_equal(scale[:, 0], np.float32(1.1) * i.astype(np.float32))
    # Orientation in radians: the keypoint's degrees (single) times pi/180 in double, then single
    assert np.array_equal(ori[:, 0], ((45.0 * i).astype(np.float32).astype(np.float64) * (np.pi / 180)).astype(np.float32))
    assert np.array_equal(metric[:, 0], np.float32(0.01) * i.astype(np.float32))
    assert desc.dtype == np.float32 and desc.shape == (5, 128)
    j = np.arange(128)
    assert np.array_equal(desc, ((i[:, None] * 31 + j[None] * 7) & 255).astype(np.float32))
    assert octave.dtype == np.int32 and np.array_equal(octave[:, 0], i - 1)
    assert np.array_equal(layer[:, 0], 1 + i % 3)
    # fewer outputs requested: only those are created (no leak, checked by the driver)
    assert mex.call("sift", I, nout=1).shape == (5, 2)


def test_sift_new_size_replaces_context(mex):
    mex.call("sift", np.zeros((20, 30), np.uint8))      # a context of another size exists first
    c0, d0 = mex.i("creates"), mex.i("destroys")
    mex.call("sift", np.zeros((24, 30), np.uint8))
    assert mex.i("creates") == c0 + 1 and mex.i("destroys") == d0 + 1
    mex.call("sift", np.zeros((24, 30), np.uint8))
    assert mex.i("creates") == c0 + 1


def test_match_passes_descriptors_as_they_lie(mex):
    rng = np.random.default_rng(2)
    F1 = rng.integers(0, 256, (7, 128)).astype(np.float32)
    F2 = rng.integers(0, 256, (6, 128)).astype(np.float32)
    pairs = mex.call("match", F1, F2)
    assert (mex.i("n1"), mex.i("ld1"), mex.i("n2"), mex.i("ld2"), mex.i("col_major")) == (7, 7, 6, 6, 1)
    assert np.array_equal(mex.d("f1", 7 * 128).reshape(7, 128), F1)
    assert np.array_equal(mex.d("f2", 6 * 128).reshape(6, 128), F2)
    assert pairs.dtype == np.uint32 and np.array_equal(pairs, [[1, 6], [3, 4], [5, 2]])
    assert mex.call("match", np.zeros((0, 128), np.float32), F2).shape == (0, 2)


def test_triangulate_points_and_camera_matrices(mex):
    rng = np.random.default_rng(3)
    x1 = rng.uniform(0, 1000, (4, 2)).astype(np.float32)
    x2 = rng.uniform(0, 1000, (4, 2)).astype(np.float32)
    P1, P2 = _P(4), _P(5)
    X = mex.call("triangulate", x1, x2, P1, P2)
    assert mex.i("n") == 4
    assert np.array_equal(mex.d("f1", 8), x1.reshape(-1)) and np.array_equal(mex.d("f2", 8), x2.reshape(-1))
    assert np.array_equal(mex.d("P1", 12), P1.reshape(-1)) and np.array_equal(mex.d("P2", 12), P2.reshape(-1))
    assert X.dtype == np.float32 and X.shape == (4, 3)
    exp = np.stack([x1[:, 0], x2[:, 1], P1[0, 3] + P2[1, 3] + np.arange(4)], 1).astype(np.float32)
    assert np.array_equal(X, exp)
    # double points (MATLAB's double Location) are accepted and rounded to single
    X2 = mex.call("triangulate", x1.astype(np.float64), x2, P1, P2)
    assert np.array_equal(X2, X)
    with pytest.raises(mexshim.MexError, match="vo:badArgument"):
        mex.call("triangulate", x1, x2[:3], P1, P2)
    with pytest.raises(mexshim.MexError, match="vo:badArgument"):
        mex.call("triangulate", x1, x2, P1[:, :3], P2)


def test_estworldpose_transposes_and_status(mex):
    rng = np.random.default_rng(6)
    img = rng.uniform(0, 1000, (6, 2))
    world = rng.normal(size=(6, 3))
    K = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1]])
    A, inl, st = mex.call("estworldpose", img, world, K, nout=3)
    assert np.array_equal(mex.d("d1", 12), img.reshape(-1)) and np.array_equal(mex.d("d2", 18), world.reshape(-1))
    assert np.array_equal(mex.d("K9", 9), K.reshape(-1))
    assert (mex.i("trials"), mex.d("conf", 1)[0], mex.d("err", 1)[0]) == (1000, 99.0, 1.0)   # VO.m:123 defaults
    assert np.array_equal(A, (np.arange(16) + 1.5).reshape(4, 4))    # A(i, j) = T[4 i + j]
    assert inl.dtype == np.bool_ and np.array_equal(inl[:, 0], np.arange(6) % 2 == 1)
    assert st[0, 0] == 0
    mex.call("estworldpose", img, world, K, np.array([[500.0, 95.0, 2.0]]))
    assert (mex.i("trials"), mex.d("conf", 1)[0], mex.d("err", 1)[0]) == (500, 95.0, 2.0)
    # failures: thrown like the toolbox function, or returned as estworldpose's status codes
    with pytest.raises(mexshim.MexError, match="vision:estworldpose:notEnoughPoints"):
        mex.call("estworldpose", img[:3], world[:3], K)
    with pytest.raises(mexshim.MexError, match="vision:estworldpose:notEnoughInliers"):
        mex.call("estworldpose", img[:5], world[:5], K, nout=2)
    A, inl, st = mex.call("estworldpose", img[:3], world[:3], K, nout=3)
    assert st[0, 0] == 1 and np.array_equal(A, np.eye(4)) and not inl.any()
    A, inl, st = mex.call("estworldpose", img[:5], world[:5], K, nout=3)
    assert st[0, 0] == 2 and np.array_equal(A, np.eye(4))


def test_landmarks_reference_signature(mex):
    """CreateLandmarksFromFeatures(features_l, features_r, p1, p2, pose, ~): VO.m:145-158 has
    filtered already, so the gateway runs libvo's filter against no old points (K = 0)."""
    rng = np.random.default_rng(7)
    fl = rng.uniform(0, 1000, (5, 2)).astype(np.float32)
    fr = rng.uniform(0, 1000, (5, 2)).astype(np.float32)
    P1, P2 = _P(8), _P(9)
    A = np.eye(4)
    A[:3, 3] = [1.0, 2.0, 3.0]
    A[0, 1] = 0.25
    rows = mex.call("landmarks", fl, fr, P1, P2, A)
    assert (mex.i("S"), mex.i("K")) == (5, 0)
    assert np.array_equal(mex.d("pose", 16), A.reshape(-1))
    assert np.array_equal(mex.d("P1", 12), P1.reshape(-1)) and np.array_equal(mex.d("K9", 9), P1[:, :3].reshape(-1))
    assert np.array_equal(mex.d("f1", 10), fl.reshape(-1)) and np.array_equal(mex.d("f2", 10), fr.reshape(-1))
    assert rows.dtype == np.float64 and rows.shape == (7, 3)
    exp = np.zeros((7, 3))
    for m in range(7):
        for a in range(3):
            exp[m, a] = (float(fl[m, a % 2]) if m < 5 else 0.0) + A[a, 3]
    assert np.array_equal(rows, exp)


def test_step_and_loop_commands(mex):
    rng = np.random.default_rng(10)
    Il = rng.integers(0, 256, (20, 30), dtype=np.uint8)
    Ir = rng.integers(0, 256, (20, 30), dtype=np.uint8)
    rel, A, st, nl = mex.call("step", Il, Ir, _P(11), _P(12), nout=4)
    assert (mex.i("ld"), mex.i("col_major"), mex.i("B")) == (20, 1, 1)
    assert np.array_equal(mex.img(0, 20, 30), Il) and np.array_equal(mex.img(1, 20, 30), Ir)
    assert np.array_equal(rel, np.arange(16.0).reshape(4, 4)) and np.array_equal(A, 100 + np.arange(16.0).reshape(4, 4))
    assert st[0, 0] == 0 and nl[0, 0] == 7
    L = mex.call("landmarks_all")
    assert np.array_equal(L, 0.5 * np.arange(9.0).reshape(3, 3))
    r0 = mex.i("resets")
    mex.call("reset", nout=0)
    assert mex.i("resets") == r0 + 1
    with pytest.raises(mexshim.MexError, match="vo:badArgument"):
        mex.call("step", Il, Ir[:, :29], _P(11), _P(12))


def test_argument_errors(mex):
    with pytest.raises(mexshim.MexError, match="vo:cmd"):
        mex.call("nope")
    with pytest.raises(mexshim.MexError, match="vo:nargin"):
        mex.call("sift")
    with pytest.raises(mexshim.MexError, match="vo:badArgument"):
        mex.call("sift", np.zeros((20, 30)))                         # double image
    with pytest.raises(mexshim.MexError, match="vo:badArgument"):
        mex.call("match", np.zeros((3, 64), np.float32), np.zeros((3, 128), np.float32))
    with pytest.raises(mexshim.MexError, match="vo:create"):
        mex.call("sift", np.zeros((8, 8), np.uint8))                 # libvo refuses the size


def test_close_releases_context(mex):
    mex.call("sift", np.zeros((20, 30), np.uint8))
    d0 = mex.i("destroys")
    mex.call("close", nout=0)
    assert mex.i("destroys") == d0 + 1


def test_integration_doc_carries_the_tree_wrappers():
    """INTEGRATION.md shows the path-shadow wrappers exactly as they are in matlab/."""
    doc = (ROOT / "INTEGRATION.md").read_text()
    for m in sorted((ROOT / "matlab").glob("*.m")):
        assert m.read_text().strip() in doc, f"INTEGRATION.md does not carry matlab/{m.name} as it is in the tree"
    assert "matlab/vo_mex.c" in doc
    # the CreateLandmarksFromFeatures shadow keeps the reference signature (CreateLandmarksFromFeatures.m:1)
    src = (ROOT / "matlab" / "CreateLandmarksFromFeatures.m").read_text()
    assert re.search(r"function landmarks = CreateLandmarksFromFeatures\(features_l, features_r, intrinsics_l, "
                     r"intrinsics_r, pose, current_landmarks\)", src)
