"""The HIP path (libvo.so) reproduces the committed golden fixtures bit for bit
at the fixtures' own (small) image size."""
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
G = Path(__file__).resolve().parent / "golden"


def test_gpu_golden_sift_pair(vo):
    z = np.load(G / "sift_pair.npz")
    H, W = z["left"].shape
    ctx = vo.Context(H, W, 1)
    kl, dl = ctx.sift(z["left"])
    kr, dr = ctx.sift(z["right"])
    for f in kl.dtype.names:
        assert np.array_equal(kl[f], z["kl_" + f]), f
        assert np.array_equal(kr[f], z["kr_" + f]), f
    assert np.array_equal(dl, z["desc_l"]) and np.array_equal(dr, z["desc_r"])
    assert np.array_equal(ctx.match(dl, dr), z["pairs"])


def test_gpu_golden_track_and_pose(vo):
    z = np.load(G / "track.npz")
    ctx = vo.Context(112, 373, 1)
    assert np.array_equal(ctx.track(z["old_l"], z["old_r"], z["cur_l"], z["cur_r"]), z["idx"])
    p = np.load(G / "pose.npz")
    st, T, inl, nin = ctx.estworldpose(p["uv"], p["world"], p["K"], frame_key=int(p["frame_key"]))
    assert st == int(p["status"]) and nin == int(p["n_inliers"])
    assert np.array_equal(T, p["T"]) and np.array_equal(inl, p["inliers"])


@pytest.mark.parametrize("batch", [1, 2, 3])
def test_gpu_golden_sequence(vo, batch):
    z = np.load(G / "sequence.npz")
    L, R = z["L"], z["R"]
    ctx = vo.Context(L.shape[1], L.shape[2], batch, calib=vo.calib_from(z["P1"], z["P2"]))
    outs = np.concatenate([ctx.step_batch(L[i:i + batch], R[i:i + batch]) for i in range(0, len(L), batch)])
    for k in outs.dtype.names:
        if k == "flags":                 # no capacity was exceeded (the oracle has no caps)
            assert not outs[k].any()
            continue
        assert np.array_equal(outs[k], z["out_" + k]), k
    assert np.array_equal(ctx.get_landmarks(), z["landmarks"])
