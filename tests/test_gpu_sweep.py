"""GPU parity sweep: many seeded inputs of assorted sizes and textures (SIFT records,
descriptors and stereo matches), and descriptor sets built to produce exact and near ties in
the ratio test (the cosine-domain top-2 of k_match_partial must reproduce the oracle's SSD
ranking).  Every comparison is bit for bit against the CPU oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [(96, 128, 0), (150, 200, 1), (201, 333, 2), (240, 320, 3), (255, 511, 4), (300, 640, 5),
         (128, 700, 6), (400, 180, 7)]


@pytest.mark.parametrize("rows,cols,k", CASES)
def test_sift_match_assorted_sizes(vo, oracle, syn, rows, cols, k):
    import torch
    B = 3
    L = np.empty((B, rows, cols), np.uint8)
    R = np.empty((B, rows, cols), np.uint8)
    for f in range(B):
        seed = syn.SEED_BASE + 1000 * k + f
        planes = syn.random_scene(seed, rows, cols, px_per_cell=8.0 + 4.0 * ((k + f) % 4))
        L[f], R[f] = syn.stereo_pair(seed, rows, cols, noise_sd=1.0 + (k % 3), planes=planes)
    ctx = vo.Context(rows, cols, B)
    dl, dr = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    torch.cuda.synchronize()
    ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B)
    for f in range(B):
        kl, dsl = ctx.fetch_keypoints(2 * f)
        kr, dsr = ctx.fetch_keypoints(2 * f + 1)
        rkl, rdl = oracle.sift(L[f])
        rkr, rdr = oracle.sift(R[f])
        for a, b in ((kl, rkl), (kr, rkr)):
            assert len(a) == len(b)
            for fld in ("x", "y", "size", "angle", "response", "octave", "layer", "scale"):
                assert np.array_equal(a[fld], b[fld]), fld
        assert np.array_equal(dsl, rdl) and np.array_equal(dsr, rdr)
        assert np.array_equal(ctx.fetch_stereo_pairs(f), oracle.match(rdl, rdr))
    ctx.close()


@pytest.mark.parametrize("seed", range(6))
def test_match_ties_bit_exact(vo, oracle, seed):
    """Rows whose best and second-best candidates are exact duplicates, permuted copies or
    one-unit perturbations (equal or adjacent SSD), spread over two F2 chunks (VO_MATCH_CHUNK =
    4096 columns), so the chunk merge of k_match_finish sees the ties too."""
    rng = np.random.default_rng(100 + seed)
    n1, n2 = 300 + 37 * seed, 4500 + 211 * seed
    F1 = rng.integers(0, 90, (n1, 128)).astype(np.uint8)
    F2 = rng.integers(0, 90, (n2, 128)).astype(np.uint8)
    for i in range(n1):
        kind = i % 4
        j1, j2 = rng.integers(0, n2, 2)
        F2[j1] = F1[i]
        if kind == 0:
            F2[j2] = F1[i]                                  # exact duplicate: 0/0, rejected
        elif kind == 1:
            F2[j2] = np.roll(F1[i], 1)                      # same norm, different dot
        elif kind == 2:
            v = F1[i].astype(int)
            v[rng.integers(0, 128)] += 1
            F2[j2] = np.clip(v, 0, 255)                     # near tie
        else:
            v = F1[i].astype(int) + rng.integers(-2, 3, 128)
            F2[j2] = np.clip(v, 0, 255)
    ctx = vo.Context(375, 1242, 1)
    got = ctx.match(F1, F2)
    ref = oracle.match(F1, F2)
    assert np.array_equal(got, ref)
    ctx.close()
