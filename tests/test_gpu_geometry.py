"""GPU parity for the rest of the per-frame path, through libvo.so vs the CPU
oracle: find_remaining_points (index sets), triangulate (f64 bit-exact),
estworldpose (pose bit-exact, inlier masks bit-exact), landmarks, and the whole
VO.m loop over a synthetic sequence (batched and frame-by-frame)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def seq(syn):
    L, R, gt = syn.sequence(6)
    return L, R, gt


@pytest.fixture(scope="module")
def calib(vo, syn):
    return vo.calib_from(syn.KITTI00_P0, syn.KITTI00_P1)


def test_track_bit_exact(vo, oracle, syn, seq):
    L, R, _ = seq
    k0l, d0l = oracle.sift(L[0])
    k0r, d0r = oracle.sift(R[0])
    m = oracle.match(d0l, d0r)
    old_l, old_r = d0l[m[:, 0] - 1], d0r[m[:, 1] - 1]
    _, d1l = oracle.sift(L[1])
    _, d1r = oracle.sift(R[1])
    ref = oracle.track(old_l, old_r, d1l, d1r)
    ctx = vo.Context(375, 1242, 1)
    got = ctx.track(old_l, old_r, d1l, d1r)
    assert len(ref) > 100
    assert np.array_equal(got, ref)


def test_triangulate_bit_exact(vo, oracle, syn):
    rng = np.random.default_rng(5)
    n = 3000
    X = np.stack([rng.uniform(-20, 20, n), rng.uniform(-3, 3, n), rng.uniform(4, 90, n)], 1)
    P1, P2 = syn.KITTI00_P0, syn.KITTI00_P1
    def proj(P):
        h = np.c_[X, np.ones(n)] @ P.T
        return (h[:, :2] / h[:, 2:]) + 1.0 + rng.normal(0, 0.3, (n, 2))
    x1 = proj(P1).astype(np.float32)
    x2 = proj(P2).astype(np.float32)
    ctx = vo.Context(375, 1242, 1)
    got = ctx.triangulate(x1, x2, P1, P2)
    ref = oracle.triangulate(x1, x2, P1, P2)
    assert np.array_equal(got, ref)
    # sanity vs truth (1-based pixel offset is part of the spec, so compare loosely)
    assert np.median(np.abs(ref[:, 2] - X[:, 2]) / X[:, 2]) < 0.05


def _pose_problem(rng, n=600, outlier_frac=0.2, noise=0.3):
    K = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1.0]])
    Xw = np.stack([rng.uniform(-15, 15, n), rng.uniform(-2, 2, n), rng.uniform(5, 60, n)], 1)
    a = np.deg2rad(0.4)
    Rcw = np.array([[np.cos(a), 0, -np.sin(a)], [0, 1, 0], [np.sin(a), 0, np.cos(a)]])
    tcw = np.array([0.02, -0.01, -0.95])
    Xc = Xw @ Rcw.T + tcw
    uv = (Xc[:, :2] / Xc[:, 2:]) * 718.856 + K[:2, 2] + rng.normal(0, noise, (n, 2))
    bad = rng.random(n) < outlier_frac
    uv[bad] += rng.uniform(-40, 40, (bad.sum(), 2))
    return uv, Xw, K


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_estworldpose_bit_exact(vo, oracle, seed):
    rng = np.random.default_rng(seed)
    uv, Xw, K = _pose_problem(rng)
    ctx = vo.Context(375, 1242, 1)
    st, T, inl, nin = ctx.estworldpose(uv, Xw, K, frame_key=seed)
    rst, rT, rinl, rnin = oracle.estworldpose(uv, Xw, K, frame_key=seed)
    assert st == rst == 0
    assert np.array_equal(T, rT)
    assert np.array_equal(inl, rinl) and nin == rnin
    assert nin > 0.6 * len(uv)


@pytest.mark.parametrize("outlier_frac,max_trials", [(0.6, 1000), (0.75, 2048), (0.2, 10), (0.5, 100), (0.9, 130)])
def test_estworldpose_lazy_chunks_equal_oracle_and_eager(vo, oracle, outlier_frac, max_trials):
    """k_msac walks the slots in chunks of 64 and stops at the chunk where the adaptive replay
    stops: at high outlier ratios the replay runs over several chunks (or all of them), at
    small MaxNumTrials the last chunk is partial.  Results equal the oracle's sequential MSAC
    and the eager kernels (every slot generated and scored; compiled only into the test build
    libvo_exp.so, selected by vo_exp_set) bit for bit."""
    rng = np.random.default_rng(int(outlier_frac * 100) + max_trials)
    uv, Xw, K = _pose_problem(rng, n=500, outlier_frac=outlier_frac)
    rp = vo.default_ransac_params()
    rp.max_num_trials = max_trials
    orp = oracle.ransac_params()
    orp.max_num_trials = max_trials
    ref = oracle.estworldpose(uv, Xw, K, params=orp, frame_key=7)
    if os.environ.get("VO_LIBPATH") and not vo.experimental_library_path().exists():
        pytest.skip("variant build without its own libvo_exp.so")
    exp = vo.load_experimental_library()
    for eager, lib in ((0, None), (1, exp)):
        ctx = vo.Context(375, 1242, 1, ransac=rp, lib=lib)
        if lib is not None:
            lib.vo_exp_set(0, 1)
        try:
            st, T, inl, nin = ctx.estworldpose(uv, Xw, K, params=rp, frame_key=7, raise_on_failure=False)
        finally:
            if lib is not None:
                lib.vo_exp_set(0, 0)
            ctx.close()
        assert st == ref[0], (eager, st, ref[0])
        if st == 0:
            assert np.array_equal(T, ref[1]) and np.array_equal(inl, ref[2]) and nin == ref[3]


def test_estworldpose_too_few_points(vo, oracle):
    ctx = vo.Context(375, 1242, 1)
    K = np.eye(3)
    with pytest.raises(vo.VOError) as e:
        ctx.estworldpose(np.zeros((3, 2)), np.ones((3, 3)), K)
    assert e.value.code == vo.VO_ERR_TOO_FEW_POINTS
    st, *_ = oracle.estworldpose(np.zeros((3, 2)), np.ones((3, 3)), K)
    assert st == vo.VO_ERR_TOO_FEW_POINTS


def test_landmarks_bit_exact(vo, oracle, syn, calib):
    rng = np.random.default_rng(9)
    S, Kn = 900, 300
    X = np.stack([rng.uniform(-20, 20, S), rng.uniform(-3, 3, S), rng.uniform(2, 120, S)], 1)
    h1 = np.c_[X, np.ones(S)] @ syn.KITTI00_P0.T
    h2 = np.c_[X, np.ones(S)] @ syn.KITTI00_P1.T
    l = (h1[:, :2] / h1[:, 2:] + 1).astype(np.float32)
    r = (h2[:, :2] / h2[:, 2:] + 1).astype(np.float32)
    old_l = rng.uniform(0, 1200, (Kn, 2)).astype(np.float32)
    old_r = rng.uniform(0, 1200, (Kn, 2)).astype(np.float32)
    old_l[:20, 0] = l[100:120, 0]        # x equality -> not new (quirk Q3)
    old_r[20:40, 1] = r[300:320, 1]      # right y equality -> not new
    pose = np.eye(4)
    pose[:3, 3] = [1.5, -0.2, 30.0]
    ctx = vo.Context(375, 1242, 1, calib=calib)
    got = ctx.landmarks(l, r, old_l, old_r, pose)
    ref = oracle.landmarks(l, r, old_l, old_r, syn.KITTI00_P0, syn.KITTI00_P1, pose)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)


def _compare_seq(outs, lm, routs, rlm):
    for f in range(len(outs)):
        for k in ("status", "n_left", "n_right", "n_stereo", "n_tracked", "n_inliers", "n_landmarks"):
            assert outs[f][k] == routs[f][k], (f, k, outs[f][k], routs[f][k])
        assert np.array_equal(outs[f]["rel_pose"], routs[f]["rel_pose"]), f
        assert np.array_equal(outs[f]["pose"], routs[f]["pose"]), f
    assert np.array_equal(lm, rlm)


def test_sequence_batched_bit_exact(vo, oracle, syn, seq, calib):
    L, R, gt = seq
    routs, rlm = oracle.run_sequence(L, R, syn.KITTI00_P0, syn.KITTI00_P1)
    ctx = vo.Context(375, 1242, 3, calib=calib)
    outs = np.concatenate([ctx.step_batch(L[0:3], R[0:3]), ctx.step_batch(L[3:6], R[3:6])])
    _compare_seq(outs, ctx.get_landmarks(), routs, rlm)
    # and the trajectory is right (synthetic ground truth)
    err = np.linalg.norm(outs["pose"][:, :3, 3] - gt[:, :3, 3], axis=1)
    assert err.max() < 0.5, err


def test_sequence_stepwise_bit_exact(vo, oracle, syn, seq, calib):
    L, R, _ = seq
    n = 4
    routs, rlm = oracle.run_sequence(L[:n], R[:n], syn.KITTI00_P0, syn.KITTI00_P1)
    ctx = vo.Context(375, 1242, 2, calib=calib)
    outs = np.array([ctx.step(L[f], R[f]) for f in range(n)], dtype=routs.dtype)
    _compare_seq(outs, ctx.get_landmarks(), routs, rlm)
    ctx.reset()
    outs2 = np.array([ctx.step(L[f], R[f]) for f in range(n)], dtype=routs.dtype)
    _compare_seq(outs2, ctx.get_landmarks(), routs, rlm)


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_sequence_pipelined_bit_exact(vo, oracle, syn, seq, calib, depth):
    """vo_step_submit_dev / vo_step_collect (two buffer sets, three result slots: batch n+1's
    SIFT overlapping batch n's geometry, batch n+2's scale space queued before batch n's
    geometry ends) give the oracle's VO.m loop bit for bit, with ragged batches, whether 1, 2
    or 3 batches are kept in flight -- in the world-frame and the camera-frame landmark modes."""
    import torch
    L, R, _ = seq
    routs, rlm = oracle.run_sequence(L, R, syn.KITTI00_P0, syn.KITTI00_P1)
    ctx = vo.Context(375, 1242, 3, calib=calib)
    dl, dr = torch.from_numpy(np.ascontiguousarray(L)).cuda(), torch.from_numpy(np.ascontiguousarray(R)).cuda()
    torch.cuda.synchronize()
    fs = L[0].size
    bounds = [(0, 2), (2, 3), (3, 4), (4, 6)]

    def run():
        outs = []
        for a, b in bounds:
            ctx.step_submit_dev(dl.data_ptr() + a * fs, dr.data_ptr() + a * fs, b - a)
            if ctx.steps_pending() == depth:
                outs.append(ctx.step_collect())
        while ctx.steps_pending():
            outs.append(ctx.step_collect())
        return np.concatenate(outs)
    _compare_seq(run(), ctx.get_landmarks(), routs, rlm)
    # camera-frame rows kept on the device (the sharded path): the same rows, moved to the world
    ctx.reset()
    ctx.set_landmark_frame(True)
    outs = run()
    X, keep = ctx.get_landmark_rows()
    assert np.array_equal(vo.landmarks_to_world_frames(outs["pose"], outs["n_landmarks"], X, keep), rlm)
    # the camera-frame rows themselves, zero rows included, are the oracle's
    _, (oX, okeep) = oracle.run_sequence(L, R, syn.KITTI00_P0, syn.KITTI00_P1, camera_rows=True)
    assert np.array_equal(keep.astype(bool), okeep.astype(bool)) and X.tobytes() == np.ascontiguousarray(oX, np.float32).tobytes()
    ctx.set_landmark_frame(False)
    # pipeline rules: at most VO_STEP_DEPTH (3) batches pending, other calls refused meanwhile
    ctx.reset()
    for k in range(vo.STEP_DEPTH):
        ctx.step_submit_dev(dl.data_ptr() + k * fs, dr.data_ptr() + k * fs, 1)
    with pytest.raises(vo.VOError):
        ctx.step_submit_dev(dl.data_ptr() + 3 * fs, dr.data_ptr() + 3 * fs, 1)
    with pytest.raises(vo.VOError):
        ctx.step_batch_dev(dl.data_ptr(), dr.data_ptr(), 1)
    ctx.step_collect()
    with pytest.raises(vo.VOError):              # the collected batch's buffer set is in use again
        ctx.fetch_tracks(0)
    ctx.step_collect()
    ctx.step_collect()
    with pytest.raises(vo.VOError):
        ctx.step_collect()
    # reset drops pending work; the synchronous form still works afterwards
    ctx.reset()
    ctx.step_submit_dev(dl.data_ptr(), dr.data_ptr(), 3)
    ctx.reset()
    assert ctx.steps_pending() == 0
    s1 = ctx.step_batch_dev(dl.data_ptr(), dr.data_ptr(), 3)
    s2 = ctx.step_batch_dev(dl.data_ptr() + 3 * fs, dr.data_ptr() + 3 * fs, 3)
    _compare_seq(np.concatenate([s1, s2]), ctx.get_landmarks(), routs, rlm)
    ctx.close()


def test_sequence_kitti_resolution_bit_exact(vo, oracle, syn):
    """The whole loop body at KITTI-00's real image size (376 x 1241: odd width, even height),
    pipelined, equals the oracle's VO.m loop bit for bit."""
    import torch
    n = 4
    L, R, _ = syn.sequence(n, rows=376, cols=1241, step_m=0.5)
    routs, rlm = oracle.run_sequence(L, R, syn.KITTI00_P0, syn.KITTI00_P1)
    ctx = vo.Context(376, 1241, 2, calib=vo.calib_from(syn.KITTI00_P0, syn.KITTI00_P1))
    dl, dr = torch.from_numpy(np.ascontiguousarray(L)).cuda(), torch.from_numpy(np.ascontiguousarray(R)).cuda()
    torch.cuda.synchronize()
    fs = L[0].size
    ctx.step_submit_dev(dl.data_ptr(), dr.data_ptr(), 2)
    ctx.step_submit_dev(dl.data_ptr() + 2 * fs, dr.data_ptr() + 2 * fs, 2)
    outs = np.concatenate([ctx.step_collect(), ctx.step_collect()])
    assert np.all(outs["status"][1:] == 0)
    _compare_seq(outs, ctx.get_landmarks(), routs, rlm)
    ctx.close()


@pytest.mark.parametrize("B", [128, 320])
def test_full_path_big_batch_equals_batches_of_64(vo, syn, calib, B):
    """The whole loop body at a large batch (B chained frames in one vo_step_batch_dev call: at
    320, over 256 match jobs per launch, so the stereo and tracking launches split at
    VO_MP_MAX_JOBS and the second part's frames compose their lists at frame offset 256) gives
    the same per-frame outputs and landmark map as the same frames in 64-frame calls (that path
    is pinned to the oracle by the tests above)."""
    import torch
    SL, SR, _ = syn.sequence(32, 375, 1242, seed=syn.SEED_BASE + 0x777, step_m=0.25, yaw_deg=0.1)
    loop = np.arange(B) % 64
    loop = np.where(loop < 32, loop, 63 - loop)
    L, R = np.ascontiguousarray(SL[loop]), np.ascontiguousarray(SR[loop])
    dl, dr = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    torch.cuda.synchronize()
    fs = L[0].size
    big = vo.Context(375, 1242, B, calib=calib)
    a = big.step_batch_dev(dl.data_ptr(), dr.data_ptr(), B)
    lm_a = big.get_landmarks()
    big.close()
    half = vo.Context(375, 1242, 64, calib=calib)
    b = np.concatenate([half.step_batch_dev(dl.data_ptr() + b0 * fs, dr.data_ptr() + b0 * fs, 64)
                        for b0 in range(0, B, 64)])
    lm_b = half.get_landmarks()
    half.close()
    assert (a["status"][1:] == 0).all()
    assert a.tobytes() == b.tobytes()
    assert lm_a.shape == lm_b.shape and lm_a.tobytes() == lm_b.tobytes()


def test_full_path_bench_configuration_pipelined(vo, syn, calib):
    """bench.py's full-path configuration: 256 frames per vo_step_submit_dev, three batches in
    flight (kitti._pipelined's default depth), camera-frame landmark rows kept on the device --
    equal, frame for frame and row for row, to the same 768 chained frames in 64-frame
    synchronous calls (pinned to the oracle by the tests above)."""
    import torch
    from r7020e_visual_odometry_amd import kitti
    SL, SR, _ = syn.sequence(32, 375, 1242, seed=syn.SEED_BASE + 0x778, step_m=0.25, yaw_deg=0.1)
    n = 768
    loop = np.arange(n) % 64
    loop = np.where(loop < 32, loop, 63 - loop)
    L, R = np.ascontiguousarray(SL[loop]), np.ascontiguousarray(SR[loop])
    dl, dr = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    torch.cuda.synchronize()
    fs = L[0].size
    big = vo.Context(375, 1242, 256, calib=calib)
    big.set_landmark_frame(True)
    a = np.concatenate(kitti._pipelined(big, kitti.device_batches(dl, dr, 256), torch.device("cuda", 0)))
    Xa, ka = big.get_landmark_rows()
    big.close()
    half = vo.Context(375, 1242, 64, calib=calib)
    half.set_landmark_frame(True)
    b = np.concatenate([half.step_batch_dev(dl.data_ptr() + b0 * fs, dr.data_ptr() + b0 * fs, 64)
                        for b0 in range(0, n, 64)])
    Xb, kb = half.get_landmark_rows()
    half.close()
    assert (a["status"][1:] == 0).all() and len(a) == n
    assert a.tobytes() == b.tobytes()
    assert Xa.tobytes() == Xb.tobytes() and ka.tobytes() == kb.tobytes()
