"""KITTI I/O, trajectory output, accuracy evaluation and map persistence (SURVEY §8(f) rows
1-3).  The reference's own KITTI-00 data files: calib.txt, poses/00.txt, times.txt and the
digitised error curve in data/kitti/ (the package reads them), the first 60 lines of
poses/00.txt and times.txt under tests/golden/kitti/."""
from pathlib import Path

import numpy as np
import pytest

GOLD = Path(__file__).resolve().parent / "golden" / "kitti"
DATA = Path(__file__).resolve().parent.parent / "data" / "kitti"


@pytest.fixture(scope="module")
def kitti():
    import vo_amd  # noqa: F401
    from r7020e_visual_odometry_amd import kitti as k
    return k


def test_calib_matches_vo_m_constants(kitti, syn):
    cal = kitti.read_calib(DATA / "calib_00.txt")
    assert set(cal) >= {"P0", "P1", "P2", "P3"}
    # VO.m:35-38 intrinsics: fu = fv = 718.856, principal point 607.1928, 185.2157
    assert cal["P0"][0, 0] == 718.856 and cal["P0"][1, 1] == 718.856
    assert cal["P0"][0, 2] == 607.1928 and cal["P0"][1, 2] == 185.2157
    assert cal["P1"][0, 3] == -386.1448                       # baseline * f
    assert np.array_equal(cal["P0"], syn.KITTI00_P0) and np.array_equal(cal["P1"], syn.KITTI00_P1)


def test_times_and_poses(kitti, tmp_path):
    t = kitti.read_times(GOLD / "times_00_head60.txt")
    assert len(t) == 60 and t[0] == 0.0 and t[1] == 1.037359e-01 and np.all(np.diff(t) > 0)
    P = kitti.read_poses(GOLD / "poses_00_head60.txt")
    assert P.shape == (60, 4, 4)
    assert np.allclose(P[0], np.eye(4), atol=1e-9)
    assert np.allclose(P[:, 3], [0, 0, 0, 1])
    R = P[:, :3, :3]
    assert np.allclose(R @ R.transpose(0, 2, 1), np.eye(3), atol=1e-5)   # rotations
    assert P[-1, 2, 3] > 40.0                                  # KITTI-00 drives forward (+z)
    kitti.write_poses(tmp_path / "p.txt", P)
    Q = kitti.read_poses(tmp_path / "p.txt")
    assert np.allclose(P, Q, rtol=1e-9, atol=1e-12)


def test_lagged_xz_error_semantics(kitti):
    gt = kitti.read_poses(GOLD / "poses_00_head60.txt")
    # an estimate that is exactly one frame ahead of GT reproduces PlotOnMap's lag: zero error
    est = np.concatenate([np.eye(4)[None], gt[:-1]])
    ahead = gt.copy()
    ahead[1:] = gt[:-1]
    assert np.allclose(kitti.lagged_xz_error(ahead, gt), 0.0)
    # a perfect estimate shows the per-frame xz step of the ground truth (quirk Q5)
    e = kitti.lagged_xz_error(gt, gt)
    step = np.linalg.norm(gt[1:, [0, 2], 3] - gt[:-1, [0, 2], 3], axis=1)
    assert e.shape == (59,) and np.allclose(e, step)
    assert est.shape == gt.shape


def test_ate_rmse(kitti):
    gt = kitti.read_poses(GOLD / "poses_00_head60.txt")
    assert kitti.ate_rmse(gt, gt) == 0.0
    est = gt.copy()
    est[1:, 0, 3] += 1.0
    assert abs(kitti.ate_rmse(est, gt) - np.sqrt(59 / 60)) < 1e-12


@pytest.mark.parametrize("ext", [".npy", ".ply"])
def test_landmark_map_round_trip(kitti, tmp_path, ext):
    rng = np.random.default_rng(5)
    pts = rng.normal(size=(257, 3)) * 30
    pts[3] = 0.0                                               # zero rows are kept (quirk Q4)
    kitti.save_landmarks(tmp_path / f"m{ext}", pts)
    back = kitti.load_landmarks(tmp_path / f"m{ext}")
    assert back.shape == pts.shape
    assert np.allclose(back, pts, rtol=1e-8, atol=0)


def write_kitti_layout(root: Path, L: np.ndarray, R: np.ndarray, seq: str = "00"):
    from PIL import Image
    d = root / seq
    for name, imgs in (("image_0", L), ("image_1", R)):
        (d / name).mkdir(parents=True, exist_ok=True)
        for i, im in enumerate(imgs):
            Image.fromarray(im).save(d / name / f"{i:06d}.png")
    (d / "calib.txt").write_text((DATA / "calib_00.txt").read_text())
    (d / "times.txt").write_text("\n".join(f"{0.1 * i:.6e}" for i in range(len(L))) + "\n")


def test_sequence_loader_round_trip(kitti, syn, tmp_path):
    L, R = syn.independent_pairs(5, 64, 96)
    write_kitti_layout(tmp_path, L, R)
    seq = kitti.KittiSequence(tmp_path, "00", threads=3)
    assert len(seq) == 5 and (seq.rows, seq.cols) == (64, 96) and seq.gt is None
    assert np.array_equal(seq.P1, syn.KITTI00_P0) and np.array_equal(seq.P2, syn.KITTI00_P1)
    got = list(seq.batches(2))
    assert [g[0] for g in got] == [0, 2, 4]
    assert np.array_equal(np.concatenate([g[1] for g in got]), L)
    assert np.array_equal(np.concatenate([g[2] for g in got]), R)
    assert kitti.undistort_identity(seq.P1[:, :3], rows=seq.rows, cols=seq.cols)
    seq.close()


def test_undistort_zero_distortion_is_identity(kitti, syn):
    """VO.m:50-51 builds cameraIntrinsics with zero distortion, so VO.m:75-76's undistortImage
    returns every u8 frame unchanged (the frames go to libvo as they are); a non-zero
    distortion does change them, so the check is not vacuous."""
    L, _ = syn.stereo_pair(syn.SEED_BASE + 5)
    K = syn.KITTI00_P0[:, :3]
    assert kitti.undistort_identity(K, rows=375, cols=1242)
    assert np.array_equal(kitti.undistort(L, K), L)
    assert not kitti.undistort_identity(K, (-0.05, 0.0, 0.0, 0.0), rows=375, cols=1242)
    out = kitti.undistort(L, K, (-0.05, 0.0, 0.0, 0.0))
    assert (out != L).mean() > 0.2
    # principal point: the map is the identity there even with radial distortion
    us, vs = kitti.undistort_map(K, (-0.05, 0.01), 375, 1242)
    assert abs(us[185, 607] - 607) < 0.2 and abs(vs[185, 607] - 185) < 0.3


def test_reference_error_curve_fixture():
    """The reference's published KITTI-00 accuracy (4500/error.png, VO.m on MATLAB over the real
    images), digitised into a fixture by tests/golden/digitize_ref_error.py: 0..470.5 s (KITTI-00's
    times.txt span), peak ~40.8 m near t = 460 s, final ~34.6 m."""
    from pathlib import Path
    d = np.loadtxt(DATA / "ref_error_digitized.csv", delimiter=",")
    t = np.loadtxt(DATA / "times_00.txt")
    assert len(d) > 500 and np.all(np.diff(d[:, 0]) > 0)
    assert abs(d[-1, 0] - t[-1]) < 1.0
    assert 40.0 < d[:, 1].max() < 41.5 and 450 < d[np.argmax(d[:, 1]), 0] < 470
    assert 34.0 < d[-1, 1] < 35.3 and 13.5 < d[:, 1].mean() < 15.0


def test_threaded_pair_rendering_equals_serial(syn):
    """bench.py renders its synthetic pairs on --cpu-threads threads: every pair depends on its
    seed alone, so the images are the serial ones."""
    L1, R1 = syn.independent_pairs(6, 48, 80, first=3)
    L4, R4 = syn.independent_pairs(6, 48, 80, first=3, threads=4)
    assert np.array_equal(L1, L4) and np.array_equal(R1, R4)
