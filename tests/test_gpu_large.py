"""GPU parity at BASELINE configs[4]'s resolution: 1920x1080 synthetic stereo with ~8k
keypoints per image (dense 8k x 8k descriptor block on the i8 MFMA match kernel).
SIFT records, descriptors and stereo match index pairs equal the CPU oracle bit for bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_large_pair_bit_exact(vo, oracle, syn):
    import torch
    L, R = syn.large_pairs(1, first=11)
    rows, cols = syn.LARGE_ROWS, syn.LARGE_COLS
    ctx = vo.Context(rows, cols, 1)
    dl = torch.from_numpy(L).cuda()
    dr = torch.from_numpy(R).cuda()
    torch.cuda.synchronize()
    stats = ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), 1)
    kl, dsl = ctx.fetch_keypoints(0)
    kr, dsr = ctx.fetch_keypoints(1)
    pairs = ctx.fetch_stereo_pairs(0)
    rkl, rdl = oracle.sift(L[0])
    rkr, rdr = oracle.sift(R[0])
    assert 6500 <= len(rkl) <= 10000, len(rkl)
    for a, b in ((kl, rkl), (kr, rkr)):
        assert len(a) == len(b)
        for f in ("x", "y", "size", "angle", "response", "octave", "layer", "scale"):
            assert np.array_equal(a[f], b[f]), f
    assert np.array_equal(dsl, rdl) and np.array_equal(dsr, rdr)
    ref = oracle.match(rdl, rdr)
    assert stats[0][2] == len(ref)
    assert np.array_equal(pairs, ref)
    ctx.close()
