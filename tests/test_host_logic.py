"""Host-side logic: frame sharding, the pose chain, the roofline byte model."""
import numpy as np
import pytest


def test_shard_range_partitions(vo_pkg=None):
    from r7020e_visual_odometry_amd import sharding
    for n in (1, 7, 64, 4541):
        for w in (1, 2, 3, 8):
            spans = [sharding.shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    assert sharding.halo_start(0) == 0 and sharding.halo_start(5) == 4


def test_chain_matches_oracle_sequence(oracle, syn):
    from r7020e_visual_odometry_amd import sharding
    z = np.load(__import__("pathlib").Path(__file__).resolve().parent / "golden" / "sequence.npz")
    rel = z["out_rel_pose"]
    assert np.array_equal(sharding.chain(rel), z["out_pose"])


def test_roofline_model_matches_survey():
    from r7020e_visual_odometry_amd import roofline
    dims = roofline.octave_dims(375, 1242)
    assert len(dims) == 9 and dims[0] == (750, 2484)
    P = sum(r * c for r, c in dims)
    assert abs(P - 2.483e6) / 2.483e6 < 0.01                       # P = 2.483 Mpx
    per_frame = 2 * roofline.pyramid_bytes_per_image(375, 1242)
    assert abs(per_frame - 438e6) / 438e6 < 0.01                    # 438 MB / stereo frame
    # default path: per-level blurs (k_blur_fused, one launch per level of octaves 0..3; level 3
    # also stores the next octave's base, so no k_down pass), octaves 4..8 (<= 9216 px per
    # plane) in the single LDS-resident k_blur_small
    kb = roofline.kernel_bytes(375, 1242, 2, fused=False)
    assert roofline.fused_octaves(375, 1242, enabled=False) == 0
    assert kb["k_blur_fused"][1] == 4 * 5 and "k_down" not in kb and kb["k_blur_small"][1] == 1
    assert kb["k_blur_fused"][0] == 2 * sum(8 * 5 * r * c + (4 * dims[o + 1][0] * dims[o + 1][1] if o < 3 else 0)
                                            for o, (r, c) in enumerate(dims[:4]))
    assert kb["k_ext_inner<3>"][0] == 2 * sum(4 * 4 * r * c for r, c in dims)      # G_1..G_4 streamed
    kd = roofline.kernel_bytes(375, 1242, 2, fused=False, ext_inner=False)
    assert kd["k_ext_stream<3>"][0] == 2 * sum(4 * 6 * r * c for r, c in dims)     # all L+3 levels
    # experimental k_octave path (test build libvo_exp.so, vo_exp_set): octaves 0..3 (>= 256 columns, >= 64 rows)
    # are one launch each (levels, extremum test, next base)
    kf = roofline.kernel_bytes(375, 1242, 2, fused=True)
    assert roofline.fused_octaves(375, 1242, enabled=True) == 4
    assert all(kf[f"k_octave_o{o}"][1] == 1 for o in range(4)) and "k_blur_fused" not in kf and "k_down" not in kf
    assert kf["k_blur_base"][1] == 1 and kf["k_blur_small"][1] == 1
    R, C = dims[0]
    assert kf["k_octave_o0"][0] == 2 * (4 * R * C * 6 + 4 * dims[1][0] * dims[1][1])   # G0 in, G1..5 out, next base
    # other layer counts keep the per-level kernels
    kb5 = roofline.kernel_bytes(375, 1242, 2, layers=4, fused=True)
    assert kb5["k_blur_fused"][1] == 4 * 6 and "k_down" not in kb5


def test_libvo_host_chain_and_landmark_transform_equal_references(vo, oracle):
    """vo_chain_poses / vo_landmarks_to_world_frames (host-only libvo entry points used after the
    multi-GPU gathers; no GPU needed) == sharding.chain (libvo's collect arithmetic restated) and
    the oracle's CreateLandmarksFromFeatures.m:17, bit for bit, with failed frames holding the pose."""
    from r7020e_visual_odometry_amd import sharding
    rng = np.random.default_rng(1)
    rel = rng.normal(size=(60, 4, 4))
    rel[:, 3] = [0, 0, 0, 1]
    st = np.zeros(60, np.int64)
    st[[0, 3, 17, 59]] = [0, -4, -3, -4]
    poses = vo.chain_poses(rel, st)
    assert np.array_equal(poses, sharding.chain(rel, status=st))
    assert np.array_equal(poses[3], poses[2]) and np.array_equal(poses[17], poses[16])
    n = rng.integers(0, 25, 60)
    X = rng.normal(size=(n.sum(), 3)).astype(np.float32)
    keep = rng.random(n.sum()) < 0.6
    got = vo.landmarks_to_world_frames(poses, n, X, keep)
    assert np.array_equal(got, sharding.world_landmarks(poses, n, X, keep, oracle.landmarks_to_world))
    assert np.all(got[~keep] == 0)
    with pytest.raises(vo.VOError):
        vo.landmarks_to_world_frames(poses, n + 1, X, keep)


def test_block_imbalance():
    """sharding.block_imbalance: max / mean of the partition's per-block cost (halo included)."""
    from r7020e_visual_odometry_amd import sharding
    assert sharding.block_imbalance(np.ones(8), 1) == 1.0
    # 8 frames over 2 ranks: rank 0 frames 0-3 (4), rank 1 halo 3 + frames 4-7 (5): 5 / 4.5
    assert abs(sharding.block_imbalance(np.ones(8), 2) - 5 / 4.5) < 1e-12
    cost = np.r_[np.full(4, 10.0), np.ones(4)]                       # heavy first half
    assert abs(sharding.block_imbalance(cost, 2) - 40 / ((40 + 14) / 2)) < 1e-12


def test_feature_byte_model():
    """roofline.feature_bytes: mask geometry of the extremum test and window pricing."""
    from r7020e_visual_odometry_amd import roofline
    w, s = roofline.mask_geometry(375, 1242)
    # octave 0 (750 x 2484): 740 interior rows x 40 words x 3 layers, dominant
    assert w > 3 * 740 * 38 and s == (w + 1023) // 1024
    one = roofline.feature_bytes(375, 1242, [100], [50], [5.0], [0], [0.0], [0], [(10, 10, 5)])
    two = roofline.feature_bytes(375, 1242, [200], [100], [5.0, 5.0], [0, 0], [0.0, 0.0], [0, 0], [(10, 10, 5)])
    assert two["k_refine"]["algorithmic"] > one["k_refine"]["algorithmic"]
    for k, v in one.items():
        assert v["line_floor"] >= v["algorithmic"] > 0, k
    # a larger keypoint reads a larger descriptor window
    big = roofline.feature_bytes(375, 1242, [100], [50], [20.0], [0], [0.0], [0], [(10, 10, 5)])
    assert big["k_desc"]["algorithmic"] > one["k_desc"]["algorithmic"]
