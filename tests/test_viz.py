"""Visualisation (VO.m:168-199): PNG/SVG writers and the reference's figure
set, on CPU with synthetic inputs (the GPU path is covered in test_gpu_kitti.py)."""
import numpy as np


def test_png_round_trip(tmp_path):
    from r7020e_visual_odometry_amd import viz
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (37, 53, 3)).astype(np.uint8)
    viz.write_png(tmp_path / "a.png", a)
    assert np.array_equal(viz.read_png_rgb(tmp_path / "a.png"), a)
    g = rng.integers(0, 256, (9, 11)).astype(np.uint8)
    viz.write_png(tmp_path / "g.png", g)
    assert np.array_equal(viz.read_png_rgb(tmp_path / "g.png")[:, :, 1], g)


def test_features_on_feed_marks(tmp_path):
    from r7020e_visual_odometry_amd import viz
    img = np.full((40, 60), 100, np.uint8)
    det = np.array([[11.0, 21.0]])                     # 1-based (x, y) -> pixel (10, 20)
    out = viz.features_on_feed(img, np.array([[31.0, 6.0]]), np.array([[41.0, 6.0]]), det)
    assert tuple(out[20, 10]) == (0, 128, 0)            # cross centre, dark green
    assert tuple(out[5, 35]) == (255, 0, 0)             # on the old -> current segment, red
    assert tuple(out[0, 0]) == (100, 100, 100)


def test_snapshot_layout_and_error(tmp_path, syn):
    from r7020e_visual_odometry_amd import kitti, viz
    n = 6
    gt = np.tile(np.eye(4), (n, 1, 1))
    gt[:, 2, 3] = np.arange(n)
    est = gt.copy()
    est[:, 0, 3] = 0.1 * np.arange(n)
    tracks = {"old_l": np.array([[10.0, 10.0]]), "cur_l": np.array([[12.0, 11.0]]),
              "world": np.array([[1.0, 2.0, 3.0]]), "det": np.array([[5.0, 5.0], [20.0, 9.0]])}
    d = viz.snapshot(tmp_path, 5, np.zeros((30, 40), np.uint8), tracks, est, gt, np.arange(n) * 0.1,
                     np.array([[0.0, 0.0, 5.0], [1.0, -1.0, 8.0]]))
    for f in ("view.png", "view.txt", "map.svg", "error.svg", "3d_map.svg"):
        assert (d / f).exists(), f
    svg, err = viz.plot_on_map(est, gt)
    assert np.allclose(err, kitti.lagged_xz_error(est, gt)) and svg.startswith("<svg")
    assert viz.read_png_rgb(d / "view.png").shape == (30, 40, 3)
