"""How far the deterministic spec (which libvo equals bit for bit) is from an OpenCV-literal
float SIFT and a MATLAB-literal float matcher (VERDICT r1 "what's missing" 5).

The spec departs from a literal float implementation in four places, all in
include/vo_spec.h / DESIGN.md §3: histograms summed in 2^-10 fixed point, vo_spec.h
transcendentals (vs libm and OpenCV's fastAtan2), no removeDuplicatedSorted, and SSD
computed as 2 - 2 cos from exact integer dot products.  oracle/liboracle_cv.so is the same
C restatement built with -DVO_CV_LITERAL, which puts the literal float forms back.  These
tests measure the divergence on the golden pair, a synthetic pair, full-size KITTI-00 street
frames and a KITTI-00 stretch, and enforce the thresholds DESIGN.md §3.8 states (round 5:
tightened to the measured values plus a small margin, so that a perf-motivated change of
vo_spec.h cannot give the margin back silently -- any such change must pass these BEFORE the
goldens are regenerated):

  keypoints   >= 99 % of keypoints agree (same x, y, octave, layer; angle within 2 deg), and
              >= 99.8 % net of the exact duplicates the spec keeps and OpenCV's
              removeDuplicatedSorted drops (measured 100 %: every other keypoint agrees)
  descriptors mean L-inf <= 0.2, 99th percentile <= 1, max <= 4 (u8 units; measured 0.09-0.12 / 1 / 1)
  matches     Jaccard of the stereo match sets >= 0.99 (measured 0.995-1.0)
  poses       8-frame trajectories differ by <= 3 % of the path (translation), <= 1 deg,
              and both stay within 3 % of the path of the rendered ground truth

What this cannot pin: MATLAB's own detectSIFTFeatures/matchFeatures (closed; not here)."""
import numpy as np
import pytest

from spec_divergence import pair_divergence, sequence_divergence


AGREE, AGREE_DEDUP = 0.99, 0.998
DESC_MEAN, DESC_P99, DESC_MAX = 0.2, 1, 4
JACCARD = 0.99


def _check_image(d):
    assert d["agreement"] >= AGREE and d["agreement_dedup"] >= AGREE_DEDUP, d
    assert d["desc_linf_mean"] <= DESC_MEAN and d["desc_linf_p99"] <= DESC_P99 and d["desc_linf_max"] <= DESC_MAX, d


def _check_pair(d):
    _check_image(d["left"])
    _check_image(d["right"])
    assert d["match_jaccard"] >= JACCARD, d


def test_golden_pair_divergence(oracle):
    from pathlib import Path
    z = np.load(Path(__file__).parent / "golden" / "sift_pair.npz")
    _check_pair(pair_divergence(oracle, z["left"], z["right"]))


def test_synthetic_pair_divergence(oracle, syn):
    L, R = syn.stereo_pair(syn.SEED_BASE + 41)
    _check_pair(pair_divergence(oracle, L, R))


def test_kitti00_street_frames_divergence(oracle):
    """Full-size (376 x 1241) frames rendered along KITTI-00's ground truth (keypoint
    and descriptor agreement on the street world, where the full path runs)."""
    import torch
    from r7020e_visual_odometry_amd import street
    torch.set_num_threads(4)
    gt = street.kitti00_gt()
    P0, P1 = street.kitti00_calib()
    L, R = street.render_frames(street.kitti00_world(), gt, [700, 2600], P0, P1, chunk=2)
    for i in range(2):
        _check_pair(pair_divergence(oracle, L[i].numpy(), R[i].numpy()))


def test_cv_literal_mode_is_a_different_implementation(oracle, syn):
    """Guard: the two libraries really differ (float histograms, fastAtan2, dedupe)."""
    L, _ = syn.stereo_pair(syn.SEED_BASE + 41)
    _, ds = oracle.sift(L)
    _, dc = oracle.sift(L, cv=True)
    assert ds.shape != dc.shape or not np.array_equal(ds, dc)


def test_kitti00_stretch_pose_divergence(oracle, syn):
    import torch
    from r7020e_visual_odometry_amd import street
    torch.set_num_threads(4)
    gt = street.kitti00_gt()
    P0, P1 = syn.calib(0.5)
    L, R = street.render_frames(street.kitti00_world(), gt, range(2600, 2608), P0, P1, rows=188, cols=620, chunk=8)
    d = sequence_divergence(oracle, L.numpy(), R.numpy(), P0, P1, gt=gt[2600:2608])
    assert d["status_spec"] == [0] * 8 and d["status_cv"] == [0] * 8
    assert d["max_translation_gap_m"] <= 0.03 * d["path_length_m"], d
    assert d["max_rotation_gap_deg"] <= 1.0, d
    assert max(d["max_error_spec_m"], d["max_error_cv_m"]) <= 0.03 * d["path_length_m"], d
