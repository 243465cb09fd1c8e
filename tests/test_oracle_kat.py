"""Known-answer tests that pin the CPU oracle (the parity anchor) to analytic
truth and to independent numpy restatements.  The reference has no tests or
golden vectors of its own, so these are the oracle's pins."""
import math

import numpy as np
import pytest

P1 = np.array([[718.856, 0.0, 607.1928, 0.0], [0.0, 718.856, 185.2157, 0.0], [0.0, 0.0, 1.0, 0.0]])
P2 = np.array([[718.856, 0.0, 607.1928, -386.1448], [0.0, 718.856, 185.2157, 0.0], [0.0, 0.0, 1.0, 0.0]])
K = P1[:, :3]


# ----------------------------------------------------------------- scale space
def test_upsample_exact(oracle):
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (23, 37)).astype(np.uint8)
    up = oracle.upsample(img)
    H, W = img.shape
    f = img.astype(np.float64)
    ref = np.zeros((2 * H, 2 * W))
    for y in range(2 * H):
        ya, yb = y // 2, (min(y // 2 + 1, H - 1) if y & 1 else max(y // 2 - 1, 0))
        for x in range(2 * W):
            xa, xb = x // 2, (min(x // 2 + 1, W - 1) if x & 1 else max(x // 2 - 1, 0))
            ref[y, x] = 0.75 * (0.75 * f[ya, xa] + 0.25 * f[ya, xb]) + 0.25 * (0.75 * f[yb, xa] + 0.25 * f[yb, xb])
    assert np.array_equal(up, ref.astype(np.float32))


def test_blur_matches_float64_convolution(oracle):
    rng = np.random.default_rng(2)
    img = (rng.random((41, 67)) * 255).astype(np.float32)
    for sigma in (1.249, 3.09):
        out = oracle.blur(img, sigma)
        k = oracle.gauss_kernel(sigma).astype(np.float64)
        r = len(k) - 1
        kk = np.concatenate([k[::-1], k[1:]])
        pad = np.pad(img.astype(np.float64), r, mode="reflect")   # numpy 'reflect' == BORDER_REFLECT_101
        h = np.stack([np.convolve(row, kk, mode="valid") for row in pad[r:-r]])
        hp = np.pad(h, ((r, r), (0, 0)), mode="reflect")
        ref = np.stack([np.convolve(col, kk, mode="valid") for col in hp.T]).T
        assert np.abs(out - ref).max() < 2e-4


def test_pyramid_structure(oracle):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (40, 64)).astype(np.uint8)
    p = oracle.sift_params()
    flat = oracle.pyramid(img, p)
    L = p.n_octave_layers
    dims = []
    R, C = 80, 128
    n_oct = oracle.lib().oracle_num_octaves(40, 64, 1)
    assert n_oct == int(round(math.log2(80) - 2)) + 1
    off = 0
    levels = []
    for o in range(n_oct):
        if o:
            R, C = R // 2, C // 2
        G = [flat[off + i * R * C: off + (i + 1) * R * C].reshape(R, C) for i in range(L + 3)]
        off += (L + 3) * R * C
        D = [flat[off + i * R * C: off + (i + 1) * R * C].reshape(R, C) for i in range(L + 2)]
        off += (L + 2) * R * C
        for i in range(L + 2):
            assert np.array_equal(D[i], G[i + 1] - G[i])
        if o:
            assert np.array_equal(G[0], levels[-1][L][: 2 * R: 2, : 2 * C: 2])
        levels.append(G)
    assert off == flat.size


def _blob_image(H, W, cx, cy, s, dark=True):
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    g = np.exp(-((x - cx) ** 2 + (y - cy) ** 2) / (2 * s * s))
    img = 200 - 150 * g if dark else 50 + 150 * g
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("cx,cy,s", [(40.0, 30.0, 3.0), (70.5, 41.25, 5.0)])
def test_sift_finds_blob(oracle, cx, cy, s):
    img = _blob_image(80, 120, cx, cy, s)
    k, d = oracle.sift(img)
    assert len(k) >= 1
    dist = np.hypot(k["x"] - (cx + 1), k["y"] - (cy + 1))    # MATLAB 1-based Location
    j = np.argmin(dist)
    assert dist[j] < 0.3
    # a Gaussian blob of sigma s is a DoG extremum at scale ~ s*sqrt(2); size = 2*scale
    assert 0.6 * s * math.sqrt(2) < k["scale"][j] < 1.6 * s * math.sqrt(2)
    assert d.shape == (len(k), 128) and d[j].max() > 0


def test_sift_rotation_90_invariance(oracle, syn):
    L, _ = syn.stereo_pair(syn.SEED_BASE + 3, rows=120, cols=160)
    rot = np.ascontiguousarray(np.rot90(L))        # 90 deg counter-clockwise
    k0, d0 = oracle.sift(L)
    k1, d1 = oracle.sift(rot)
    m = oracle.match(d0, d1)
    assert len(m) > 0.5 * len(k0)
    # (x, y) 1-based -> rotated image: x' = y, y' = W + 1 - x
    W = L.shape[1]
    a, b = k0[m[:, 0] - 1], k1[m[:, 1] - 1]
    err = np.hypot(b["x"] - a["y"], b["y"] - (W + 1 - a["x"]))
    assert np.mean(err < 0.5) > 0.9


# ----------------------------------------------------------------- matching
def _np_match(F1, F2, thr=0.04, ratio=0.6):
    """independent numpy float32 restatement of the match spec"""
    a, b = F1.astype(np.int64), F2.astype(np.int64)
    if len(a) == 0 or len(b) == 0:
        return np.zeros((0, 2), np.uint32)
    f32 = np.float32

    def inv(x):
        s = (x * x).sum(1)
        with np.errstate(divide="ignore"):
            return np.where(s > 0, f32(1) / np.sqrt(s.astype(f32)), f32(0)).astype(f32)
    c = (((a @ b.T).astype(f32) * inv(a)[:, None]) * inv(b)[None, :]).astype(f32)
    ssd = (f32(2) - f32(2) * c).astype(f32)
    out = []
    for i in range(len(a)):
        row = ssd[i]
        j = int(np.argmin(row))
        best = row[j]
        second = np.partition(row, 1)[1] if len(row) > 1 else f32(np.inf)
        with np.errstate(divide="ignore", invalid="ignore"):
            r = f32(best) / f32(second)
        if best <= f32(thr) and r <= f32(ratio):
            out.append((i + 1, j + 1))
    return np.array(out, np.uint32).reshape(-1, 2)


def test_match_against_numpy_restatement(oracle):
    rng = np.random.default_rng(4)
    base = rng.integers(0, 140, (300, 128)).astype(np.uint8)
    F1 = base[:200].copy()
    F2 = np.clip(base[50:].astype(int) + rng.integers(-4, 5, (250, 128)), 0, 255).astype(np.uint8)
    F2[10] = F2[11]          # duplicate in F2 -> ambiguous (ratio 1)
    F1[5] = 0                # zero descriptor row
    F2[20] = 0
    got = oracle.match(F1, F2)
    ref = _np_match(F1, F2)
    assert len(ref) > 50
    assert np.array_equal(got, ref)


def test_match_edge_cases(oracle):
    rng = np.random.default_rng(5)
    F = rng.integers(0, 100, (10, 128)).astype(np.uint8)
    assert oracle.match(F, F[:0]).shape == (0, 2)
    assert oracle.match(F[:0], F).shape == (0, 2)
    one = oracle.match(F, F[3:4])            # a single candidate: ratio test passes (second = inf)
    assert one.tolist() == [[4, 1]]
    same = oracle.match(F, F)                # identical sets -> identity pairs, ascending in column 1
    assert same.tolist() == [[i + 1, i + 1] for i in range(10)]
    dup = oracle.match(F[:1], np.vstack([F[:1], F[:1]]))   # exact duplicate -> 0/0 ratio -> rejected
    assert dup.shape == (0, 2)


def test_track_index_composition(oracle):
    """find_remaining_points with a hand-built permutation chain."""
    rng = np.random.default_rng(6)
    n = 60

    def jitter(x):
        return np.clip(x.astype(int) + rng.integers(-2, 3, x.shape), 0, 255).astype(np.uint8)
    A = rng.integers(0, 200, (n, 128)).astype(np.uint8)    # old left  (row k)
    Bd = jitter(A)                                         # old right: same points seen from the right
    pl = rng.permutation(n)
    pr = rng.permutation(n)
    cur_l = np.vstack([jitter(A[pl]), rng.integers(0, 200, (7, 128)).astype(np.uint8)])   # + distractors
    cur_r = np.vstack([jitter(Bd[pr]), rng.integers(0, 200, (5, 128)).astype(np.uint8)])
    idx = oracle.track(A, Bd, cur_l, cur_r)
    assert len(idx) == n                                   # every point survives the 4-match chain
    inv_l, inv_r = np.argsort(pl), np.argsort(pr)
    for o, cl, cr in idx:                                  # old row k sits at cur rows inv(p)[k]
        assert cl - 1 == inv_l[o - 1] and cr - 1 == inv_r[o - 1]
    assert idx[:, 1].tolist() == sorted(idx[:, 1].tolist())   # ascending in the last match's F1 order


# ----------------------------------------------------------------- geometry
def test_triangulate_exact_projection(oracle):
    rng = np.random.default_rng(7)
    X = np.stack([rng.uniform(-10, 10, 200), rng.uniform(-2, 2, 200), rng.uniform(4, 60, 200)], 1)
    h1 = np.c_[X, np.ones(200)] @ P1.T
    h2 = np.c_[X, np.ones(200)] @ P2.T
    x1, x2 = h1[:, :2] / h1[:, 2:], h2[:, :2] / h2[:, 2:]
    got = oracle.triangulate(x1, x2, P1, P2)
    # inputs are rounded to single (MATLAB Location is single): tolerance from that rounding
    assert np.max(np.abs(got - X) / X[:, 2:]) < 2e-4


def _rand_pose(rng):
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    a = rng.uniform(0.01, 0.3)
    Kx = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    R = np.eye(3) + math.sin(a) * Kx + (1 - math.cos(a)) * Kx @ Kx
    return R, rng.normal(scale=0.5, size=3)


def test_p3p_recovers_pose(oracle):
    rng = np.random.default_rng(8)
    for _ in range(20):
        R, t = _rand_pose(rng)
        Xw = np.stack([rng.uniform(-5, 5, 3), rng.uniform(-2, 2, 3), rng.uniform(6, 30, 3)], 1)
        Xc = Xw @ R.T + t
        uv = Xc[:, :2] / Xc[:, 2:] * 718.856 + K[:2, 2]
        Rs, ts = oracle.p3p(uv, Xw, K)
        assert len(Rs) >= 1
        err = min(np.abs(Ri - R).max() + np.abs(ti - t).max() for Ri, ti in zip(Rs, ts))
        assert err < 2e-5


def test_estworldpose_noise_free_with_outliers(oracle):
    rng = np.random.default_rng(9)
    R, t = _rand_pose(rng)
    n = 300
    Xw = np.stack([rng.uniform(-10, 10, n), rng.uniform(-2, 2, n), rng.uniform(6, 50, n)], 1)
    Xc = Xw @ R.T + t
    uv = Xc[:, :2] / Xc[:, 2:] * 718.856 + K[:2, 2]
    out = rng.random(n) < 0.3
    uv[out] += rng.uniform(5, 50, (out.sum(), 2)) * rng.choice([-1, 1], (out.sum(), 2))
    st, T, inl, nin = oracle.estworldpose(uv, Xw, K)
    assert st == 0
    # camera pose in world: [R^T, -R^T t]
    assert np.abs(T[:3, :3] - R.T).max() < 1e-8
    assert np.abs(T[:3, 3] - (-R.T @ t)).max() < 1e-8
    assert np.array_equal(inl, ~out)


def test_estworldpose_degenerate(oracle):
    st, *_ = oracle.estworldpose(np.zeros((3, 2)), np.ones((3, 3)), K)
    assert st == -3                         # VO_ERR_TOO_FEW_POINTS (estworldpose throws)
    # four points that are all behind the camera: no hypothesis scores a finite
    # 4th-point error -> no model -> VO_ERR_NO_CONSENSUS
    st, *_ = oracle.estworldpose(np.array([[100.0, 100], [300, 120], [500, 90], [200, 300]]),
                                 np.array([[0.0, 0, 0], [0, 0, 0], [0, 0, 0], [0, 0, 0]]), K)
    assert st == -4


def test_landmarks_quirks(oracle):
    """VO.m:145-158 + CreateLandmarksFromFeatures.m quirks Q3/Q4."""
    X = np.array([[0.0, 0.0, 10.0], [1.0, 0.5, 20.0], [2.0, 0.0, 90.0], [-1.0, 0.2, 15.0], [0.5, 0.1, 30.0]])
    h1 = np.c_[X, np.ones(5)] @ P1.T
    h2 = np.c_[X, np.ones(5)] @ P2.T
    l = (h1[:, :2] / h1[:, 2:]).astype(np.float32)
    r = (h2[:, :2] / h2[:, 2:]).astype(np.float32)
    pose = np.eye(4)
    pose[:3, 3] = [10.0, 0.0, 5.0]
    none = np.zeros((0, 2), np.float32)
    out = oracle.landmarks(l, r, none, none, P1, P2, pose)
    # odd 1-based rows 1,3,5 are triangulated; row 3 (z=90) is gated out; rows 2,4 stay zero
    assert out.shape == (5, 3)
    assert np.allclose(out[0], X[0] + [10, 0, 5], atol=1e-3)
    assert np.allclose(out[4], X[4] + [10, 0, 5], atol=1e-3)
    assert not out[1].any() and not out[2].any() and not out[3].any()
    # any-x-or-y equality against old points removes a row (x of old left == x of point 0)
    old_l = np.array([[l[0, 0], -7.0]], np.float32)
    old_r = np.array([[-1.0, -1.0]], np.float32)
    out2 = oracle.landmarks(l, r, old_l, old_r, P1, P2, pose)
    # new list is points 1..4 -> odd rows are points 1 and 3 (z 20, 15)
    assert out2.shape == (3, 3)
    assert np.allclose(out2[0], X[1] + [10, 0, 5], atol=1e-3)
    assert np.allclose(out2[2], X[3] + [10, 0, 5], atol=1e-3)
    # nothing new -> zeros(2,3)
    out3 = oracle.landmarks(l[:1], r[:1], l[:1], r[:1], P1, P2, pose)
    assert out3.shape == (2, 3) and not out3.any()


def test_sequence_tracks_ground_truth(oracle, syn):
    s = 0.4
    A, B = syn.calib(s)
    L, R, gt = syn.sequence(4, rows=150, cols=497, scale=s)
    outs, lm = oracle.run_sequence(L, R, A, B)
    assert outs["status"].tolist() == [0, 0, 0, 0]
    err = np.linalg.norm(outs["pose"][:, :3, 3] - gt[:, :3, 3], axis=1)
    assert err.max() < 0.5
    assert lm.shape[0] == outs["n_landmarks"].sum()


def test_match_f32_known_answers(oracle):
    """The float SSD restatement of matchFeatures (oracle_match_f32, libvo's spec for non-u8
    features): hand-built rows with known nearest / second-nearest neighbours.  Scale invariance
    (rows are normalised), the 0.04 SSD threshold, the 0.6 ratio, a single candidate, duplicate
    F2 rows (0/0 ratio: rejected) and a zero row."""
    e = np.eye(128, dtype=np.float32)
    F2 = np.stack([e[0], e[1], e[2], e[2]])                        # rows 2 and 3 duplicates
    q = lambda v: (v / np.linalg.norm(v)).astype(np.float32)
    F1 = np.stack([
        5.0 * q(e[0] + 0.05 * e[5]),        # near e0 (ssd ~ 0.0025), far from e1: accepted -> 1
        q(e[1] + 0.3 * e[0]),               # ssd to e1 ~ 0.087 > 0.04: rejected by threshold
        q(e[2] + 0.01 * e[7]),              # nearest rows 2 and 3 tie: best/second = 1: rejected
        np.zeros(128, np.float32),          # zero row: ssd 1 to everything: rejected
        q(e[1] + 0.1 * e[9]),               # ssd ~ 0.0099 to e1, ~ 2 to the rest: accepted -> 2
    ])
    got = oracle.match_f32(F1, F2)
    assert got.tolist() == [[1, 1], [5, 2]]
    # one candidate: the ratio is 0, only the threshold decides
    assert oracle.match_f32(F1[:1], e[:1]).tolist() == [[1, 1]]
    assert oracle.match_f32(F1[1:2], e[1:2]).tolist() == []
    assert oracle.match_f32(F1[:0], F2).shape == (0, 2) and oracle.match_f32(F1, F2[:0]).shape == (0, 2)
