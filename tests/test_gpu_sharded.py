"""GPU parity of the multi-GPU path and of VO.m's estworldpose defaults, through libvo.so.

* A KITTI-00 stretch rendered along the reference's ground truth (street.py) at 376x1241:
  libvo shards (block + one-frame halo, camera-frame landmark rows), run one after another
  in this process exactly as the ranks of kitti.run_distributed would, then the frame
  records and landmark rows concatenated in rank order (what the all-gathers produce),
  chained and moved to the world -- equal bit for bit to a single libvo run AND to the
  oracle's single-process VO.m loop (poses, per-frame records, landmark map).
* MaxNumTrials 1000 (VO.m:123-127 uses estworldpose's defaults) on a 25 %-inlier problem
  whose adaptive trial count exceeds 1000: libvo equals the oracle at the default, and the
  cap is what decides the result (1000 and 2048 replay different slot counts).
* vo_fetch_* after a batched call and a later vo_sift read the vo_sift result."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROWS, COLS = 376, 1241
FRAMES = range(2000, 2008)


@pytest.fixture(scope="module")
def street_seq():
    import torch
    from r7020e_visual_odometry_amd import street
    gt = street.kitti00_gt()
    P0, P1 = street.kitti00_calib()
    w = street.kitti00_world(device="cuda:0")
    L, R = street.render_frames(w, gt, FRAMES, P0, P1, chunk=8)
    torch.cuda.synchronize()
    return L, R, P0, P1, gt[FRAMES.start:FRAMES.stop]


@pytest.fixture(scope="module")
def single_run(vo, street_seq):
    from r7020e_visual_odometry_amd import kitti
    L, R, P0, P1, _ = street_seq
    ctx = vo.Context(ROWS, COLS, 3, calib=vo.calib_from(P0, P1))
    outs = np.concatenate(kitti._pipelined(ctx, kitti.device_batches(L, R, 3), None))
    lm = ctx.get_landmarks()
    ctx.close()
    return outs, lm


def test_street_sequence_single_run_equals_oracle(vo, oracle, street_seq, single_run):
    L, R, P0, P1, gt = street_seq
    outs, lm = single_run
    routs, rlm = oracle.run_sequence(L.cpu().numpy(), R.cpu().numpy(), P0, P1)
    assert outs.tobytes() == routs.tobytes()
    assert lm.shape == rlm.shape and np.array_equal(lm, rlm)
    assert (outs["status"][1:] == 0).all()
    assert 1500 < outs["n_left"].mean() < 3500
    # the trajectory is right: relative translations within 5 cm of the rendered ground truth
    rel_gt = np.stack([np.linalg.inv(gt[i - 1]) @ gt[i] for i in range(1, len(gt))])
    assert np.abs(outs["rel_pose"][1:, :3, 3] - rel_gt[:, :3, 3]).max() < 0.05


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_libvo_equals_single_run(vo, street_seq, single_run, world):
    from r7020e_visual_odometry_amd import kitti, sharding
    L, R, P0, P1, _ = street_seq
    outs1, lm1 = single_run
    seq = (L, R, P0, P1)
    ctx = vo.Context(ROWS, COLS, 2, calib=vo.calib_from(P0, P1))
    parts = [kitti.run_shard(seq, r, world, 2, 0, ctx=ctx) for r in range(world)]
    ctx.close()
    outs = np.concatenate([p[0] for p in parts])
    X = np.concatenate([p[1] for p in parts])
    keep = np.concatenate([p[2] for p in parts])
    steps = sharding.steps_of(outs)
    poses, lm = kitti.assemble(steps, X, keep)
    assert np.array_equal(steps["rel_pose"], outs1["rel_pose"])
    for k in sharding.STEP_FIELDS:
        assert np.array_equal(steps[k], outs1[k]), k
    assert np.array_equal(poses, outs1["pose"])
    assert lm.shape == lm1.shape and np.array_equal(lm, lm1)


@pytest.mark.parametrize("world", [1, 2, 3, 10])
def test_device_world_transform_of_shards_equals_single_run(vo, street_seq, single_run, world):
    """kitti.finish_shard's per-rank step: each shard's own rows moved to the world on the device
    (vo_landmarks_world_dev, k_lm_world) with the chained poses of its frames, halo frame
    included; the shards' float32 rows concatenated in rank order equal the single run's map.
    (world 10 over 8 frames: two ranks own no frame and run only their halo.)"""
    import torch
    from r7020e_visual_odometry_amd import kitti, sharding
    L, R, P0, P1, _ = street_seq
    outs1, lm1 = single_run
    n = L.shape[0]
    seq = (L, R, P0, P1)
    ctx = vo.Context(ROWS, COLS, 3, calib=vo.calib_from(P0, P1))
    outs = [kitti.run_shard(seq, r, world, 3, 0, ctx=ctx, rows_to_host=False)[0] for r in range(world)]
    steps = sharding.steps_of(np.concatenate(outs))
    poses = vo.chain_poses(steps["rel_pose"], steps["status"])
    assert np.array_equal(poses, outs1["pose"])
    counts = sharding.rank_row_counts(steps["n_landmarks"], n, world)
    parts = []
    for r in range(world):                       # each "rank" again, its rows left on the device
        kitti.run_shard(seq, r, world, 3, 0, ctx=ctx, rows_to_host=False)
        s, e = sharding.shard_range(n, world, r)
        h = sharding.halo_start(s)
        assert ctx.landmarks_world_dev(poses[h:e], 0, 0) == counts[r]          # count only
        buf = torch.full((counts[r] + 5, 3), float("nan"), device="cuda:0")
        assert ctx.landmarks_world_dev(poses[h:e], buf.data_ptr(), buf.shape[0]) == counts[r]
        assert torch.isnan(buf[counts[r]:]).all()                                # nothing past the rows
        parts.append(buf[: counts[r]].cpu().numpy())
        with pytest.raises(vo.VOError):                                         # one pose per collected frame
            ctx.landmarks_world_dev(poses[h:e - 1], buf.data_ptr(), buf.shape[0])
        if counts[r]:
            with pytest.raises(vo.VOError):                                     # capacity
                ctx.landmarks_world_dev(poses[h:e], buf.data_ptr(), counts[r] - 1)
    ctx.close()
    lm = np.concatenate(parts)
    assert lm.shape == lm1.shape and np.array_equal(lm.astype(np.float64), lm1)


def test_camera_frame_rows_transform_to_world_rows(vo, street_seq, single_run):
    """vo_set_landmark_frame(1) + vo_landmarks_to_world == the world rows of mode 0."""
    from r7020e_visual_odometry_amd import kitti, sharding
    L, R, P0, P1, _ = street_seq
    outs1, lm1 = single_run
    ctx = vo.Context(ROWS, COLS, 3, calib=vo.calib_from(P0, P1))
    ctx.set_landmark_frame(True)
    outs = np.concatenate(kitti._pipelined(ctx, kitti.device_batches(L, R, 3), None))
    X, keep = ctx.get_landmark_rows()
    assert ctx.lib.vo_set_landmark_frame(ctx.h, 2) == vo.VO_ERR_ARG
    ctx.close()
    assert outs.tobytes() == outs1.tobytes()
    lm = sharding.world_landmarks(outs["pose"], outs["n_landmarks"], X, keep, vo.landmarks_to_world)
    assert np.array_equal(lm, lm1)
    assert (~keep).sum() > 0 and keep.sum() > 100          # zero rows (quirk Q4) and kept rows


def _low_inlier_problem(seed, n=600, inlier_frac=0.25):
    rng = np.random.default_rng(seed)
    K = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1.0]])
    Xw = np.stack([rng.uniform(-15, 15, n), rng.uniform(-2, 2, n), rng.uniform(5, 60, n)], 1)
    a = np.deg2rad(0.6)
    Rcw = np.array([[np.cos(a), 0, -np.sin(a)], [0, 1, 0], [np.sin(a), 0, np.cos(a)]])
    Xc = Xw @ Rcw.T + np.array([0.03, -0.01, -0.9])
    uv = (Xc[:, :2] / Xc[:, 2:]) * 718.856 + K[:2, 2] + rng.normal(0, 0.2, (n, 2))
    bad = rng.random(n) >= inlier_frac
    uv[bad] += rng.uniform(-60, 60, (bad.sum(), 2))
    return uv, Xw, K


@pytest.mark.parametrize("seed", [11, 12])
def test_estworldpose_default_1000_trials_equals_oracle(vo, oracle, seed):
    uv, Xw, K = _low_inlier_problem(seed)
    ctx = vo.Context(375, 1242, 1)
    assert ctx.ransac_params.max_num_trials == 1000          # VO.m:123-127: estworldpose defaults
    st, T, inl, nin = ctx.estworldpose(uv, Xw, K, frame_key=seed)
    rst, rT, rinl, rnin = oracle.estworldpose(uv, Xw, K, frame_key=seed)
    assert st == rst == 0
    assert np.array_equal(T, rT) and np.array_equal(inl, rinl) and nin == rnin
    # adaptive count N = log(0.01) / log(1 - w^4) at the final inlier ratio exceeds the cap
    w = nin / len(uv)
    assert np.log(0.01) / np.log1p(-w ** 4) > 1000
    # the 2048-slot configuration replays more hypotheses; it also equals the oracle at 2048
    rp = vo.default_ransac_params()
    rp.max_num_trials = 2048
    big = vo.Context(375, 1242, 1, ransac=rp)
    st2, T2, inl2, nin2 = big.estworldpose(uv, Xw, K, params=rp, frame_key=seed)
    rst2, rT2, rinl2, rnin2 = oracle.estworldpose(uv, Xw, K, params=oracle.ransac_params(2048), frame_key=seed)
    assert st2 == rst2 == 0 and np.array_equal(T2, rT2) and np.array_equal(inl2, rinl2)
    with pytest.raises(vo.VOError):                           # more trials than the context allocated
        ctx.estworldpose(uv, Xw, K, params=rp, frame_key=seed)


def test_fetch_after_batch_then_sift_reads_the_sift_result(vo, syn, oracle):
    """a batched call on buffer set 1 followed by vo_sift must not leave the fetch
    calls pointing at set 1."""
    import torch
    L, R = syn.independent_pairs(2, 375, 1242)
    ctx = vo.Context(375, 1242, 2)
    dl, dr = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    torch.cuda.synchronize()
    ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), 2, stats=False)   # set 0
    ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), 2, stats=False)   # set 1
    img = syn.stereo_pair(syn.SEED_BASE + 999)[0]
    k, d = ctx.sift(img)
    fk, fd = ctx.fetch_keypoints(0)
    assert np.array_equal(fk, k) and np.array_equal(fd, d)
    rk, rd = oracle.sift(img)
    assert np.array_equal(k, rk)
    ctx.close()
