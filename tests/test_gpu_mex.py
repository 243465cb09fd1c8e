"""The MATLAB MEX gateway (matlab/vo_mex.c, built against tests/mex_shim's mx-API) linked to the
real libvo on the GPU: every command driven with MATLAB column-major inputs, as the path-shadow
wrappers of matlab/ call it from an unedited VO.m, against the CPU oracle and the ctypes
mirror (vo.py) -- bit for bit.  Reference call sites: VO.m:79-87 (sift, match), :113-116
(triangulate), :123-127 (estworldpose), :160 + CreateLandmarksFromFeatures.m:1-21 (landmarks),
the whole loop body VO.m:70-161 (step)."""
import numpy as np
import pytest

import mexshim

pytestmark = pytest.mark.gpu

K_L = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1.0]])


@pytest.fixture(scope="module")
def mex(vo):
    vo.load_library()                    # torch, then libvo: one HIP runtime in the process
    m = mexshim.Mex(mexshim.REAL)
    yield m
    m.at_exit()


@pytest.fixture(scope="module")
def pair(syn):
    return syn.stereo_pair(syn.SEED_BASE + 3)


def _kp_outputs(kps, desc):
    loc = np.stack([kps["x"], kps["y"]], 1)
    ori = (kps["angle"].astype(np.float64) * (np.pi / 180)).astype(np.float32)
    return loc, kps["scale"], ori, kps["response"], desc.astype(np.float32), kps["octave"], kps["layer"]


def test_mex_sift_and_match(mex, vo, oracle, pair):
    L, R = pair
    got = {}
    for side, img in (("l", L), ("r", R)):
        out = mex.call("sift", img, nout=7)          # F-ordered: vo_sift_ex(col_major = 1, ld = rows)
        kps, desc = oracle.sift(img)
        assert len(kps) > 1000
        exp = _kp_outputs(kps, desc)
        for g, e in zip(out, exp):
            assert np.array_equal(g.reshape(e.shape), e)
        ck, cd = vo.Context(375, 1242, 1).sift(img)  # the ctypes path (row-major) agrees too
        assert np.array_equal(ck, kps) and np.array_equal(cd, desc)
        got[side] = (out[4], desc)
    pairs = mex.call("match", got["l"][0], got["r"][0])
    ref = oracle.match(got["l"][1], got["r"][1])
    assert pairs.dtype == np.uint32 and len(ref) > 300
    assert np.array_equal(pairs, ref)


def _pose_problem(rng, n=500, outlier_frac=0.2, noise=0.3):
    Xw = np.stack([rng.uniform(-15, 15, n), rng.uniform(-2, 2, n), rng.uniform(5, 60, n)], 1)
    a = np.deg2rad(0.4)
    Rcw = np.array([[np.cos(a), 0, -np.sin(a)], [0, 1, 0], [np.sin(a), 0, np.cos(a)]])
    tcw = np.array([0.02, -0.01, -0.95])
    Xc = Xw @ Rcw.T + tcw
    uv = Xc @ K_L.T
    uv = uv[:, :2] / uv[:, 2:] + 1.0 + rng.normal(0, noise, (n, 2))
    bad = rng.random(n) < outlier_frac
    uv[bad] += rng.uniform(-40, 40, (bad.sum(), 2))
    return uv, Xw


def test_mex_triangulate_estworldpose(mex, vo, oracle, syn):
    rng = np.random.default_rng(21)
    n = 700
    X = np.stack([rng.uniform(-20, 20, n), rng.uniform(-3, 3, n), rng.uniform(4, 90, n)], 1)
    P1, P2 = syn.KITTI00_P0, syn.KITTI00_P1

    def proj(P):
        h = np.c_[X, np.ones(n)] @ P.T
        return (h[:, :2] / h[:, 2:]) + 1.0 + rng.normal(0, 0.3, (n, 2))
    x1, x2 = proj(P1).astype(np.float32), proj(P2).astype(np.float32)
    Xm = mex.call("triangulate", x1, x2, P1, P2)
    assert Xm.dtype == np.float32
    assert np.array_equal(Xm, oracle.triangulate(x1, x2, P1, P2).astype(np.float32))
    img, world = _pose_problem(rng)
    A, inl, st = mex.call("estworldpose", img, world, K_L, nout=3)
    rc, T, cin, _ = vo.Context(375, 1242, 1).estworldpose(img, world, K_L, frame_key=0)
    ost, oT, oin, _ = oracle.estworldpose(img, world, K_L)          # MaxNumTrials 1000, frame key 0
    assert rc == 0 and ost == 0 and st[0, 0] == 0
    assert np.array_equal(A, T) and np.array_equal(A, oT)
    assert np.array_equal(inl[:, 0], cin) and np.array_equal(inl[:, 0], oin)
    # too few points: thrown like the toolbox, or the status output
    with pytest.raises(mexshim.MexError, match="notEnoughPoints"):
        mex.call("estworldpose", img[:3], world[:3], K_L)
    A, inl, st = mex.call("estworldpose", img[:3], world[:3], K_L, nout=3)
    assert st[0, 0] == 1 and np.array_equal(A, np.eye(4))


def _create_landmarks_restated(oracle, fl, fr, P1, P2, A):
    """CreateLandmarksFromFeatures.m:2-18 read literally (odd 1-based rows, z gates, zero rows,
    zeros(size(features_l, 2), 3) = 2 rows preallocated), with the oracle's triangulate and
    world transform (rounded through single)."""
    rows = np.zeros((2, 3))
    for i in range(0, len(fl), 2):                   # i = 1:2:end, 0-based here
        X = oracle.triangulate(fl[i:i + 1], fr[i:i + 1], P1, P2)[0].astype(np.float32)
        if X[2] < 0 or X[2] > 80:
            continue
        if rows.shape[0] < i + 1:
            rows = np.vstack([rows, np.zeros((i + 1 - rows.shape[0], 3))])
        rows[i] = oracle.landmarks_to_world(A, X[None], np.ones(1, bool))[0]
    return rows


def test_mex_create_landmarks_reference_signature(mex, vo, oracle, syn, pair):
    L, R = pair
    kl, dl = oracle.sift(L)
    kr, dr = oracle.sift(R)
    m = oracle.match(dl, dr)
    fl = np.stack([kl["x"], kl["y"]], 1)[m[:, 0] - 1]
    fr = np.stack([kr["x"], kr["y"]], 1)[m[:, 1] - 1]
    P1, P2 = syn.KITTI00_P0, syn.KITTI00_P1
    A = np.eye(4)
    c, s = np.cos(0.3), np.sin(0.3)
    A[:3, :3] = [[c, 0, s], [0, 1, 0], [-s, 0, c]]
    A[:3, 3] = [12.5, -0.25, 301.0]
    rows = mex.call("landmarks", fl, fr, P1, P2, A)
    exp = _create_landmarks_restated(oracle, fl, fr, P1, P2, A)
    assert rows.shape == exp.shape and rows.shape[0] > 100
    assert np.array_equal(rows, exp)
    ctx = vo.Context(375, 1242, 1, calib=vo.calib_from(P1, P2))
    assert np.array_equal(rows, ctx.landmarks(fl, fr, np.zeros((0, 2)), np.zeros((0, 2)), A))
    # the degenerate inputs of the reference: no points -> its two preallocated zero rows
    assert np.array_equal(mex.call("landmarks", np.zeros((0, 2), np.float32), np.zeros((0, 2), np.float32), P1, P2, A),
                          np.zeros((2, 3)))


def test_mex_step_loop(mex, oracle, syn):
    L, R, _ = syn.sequence(4)
    P1, P2 = syn.KITTI00_P0, syn.KITTI00_P1
    ref, lm = oracle.run_sequence(L, R, P1, P2)
    mex.call("reset", nout=0)
    for f in range(len(L)):
        rel, A, st, nl = mex.call("step", L[f], R[f], P1, P2, nout=4)
        assert st[0, 0] == ref["status"][f]
        assert np.array_equal(rel, ref["rel_pose"][f]) and np.array_equal(A, ref["pose"][f])
        assert nl[0, 0] == ref["n_landmarks"][f]
    assert np.array_equal(mex.call("landmarks_all"), lm)
