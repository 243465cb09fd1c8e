"""GPU parity of the Gaussian scale space itself: every level of every octave of
libvo's pyramid (k_blur_base, the level blurs k_blur_stream, k_down,
k_blur_small) equals the CPU oracle's plane bit for bit, on assorted image sizes
(strip/band edges, reflect-101 borders on all four sides, odd widths)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [(375, 1242), (376, 1241), (240, 700), (97, 131), (131, 97), (400, 1800), (77, 101)]


def _planes(oracle, img, L=3):
    """oracle.pyramid -> {(octave, level): plane} for the Gaussian levels."""
    flat = oracle.pyramid(img)
    r, c = 2 * img.shape[0], 2 * img.shape[1]
    out, off, o = {}, 0, 0
    while off < flat.size:
        if o:
            r, c = r // 2, c // 2
        for i in range(L + 3):
            out[(o, i)] = flat[off: off + r * c].reshape(r, c)
            off += r * c
        off += (L + 2) * r * c
        o += 1
    return out


@pytest.mark.parametrize("shape", SIZES)
def test_gaussian_levels_bit_exact(vo, oracle, syn, shape):
    import torch
    rows, cols = shape
    B = 2
    L = np.empty((B, rows, cols), np.uint8)
    R = np.empty((B, rows, cols), np.uint8)
    for f in range(B):
        L[f], R[f] = syn.stereo_pair(syn.SEED_BASE + 300 + f, rows, cols)
    ctx = vo.Context(rows, cols, B)
    dl, dr = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    torch.cuda.synchronize()
    ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B)
    for img in (0, 3):
        src = L[img // 2] if img % 2 == 0 else R[img // 2]
        ref = _planes(oracle, src)
        for (o, i), plane in ref.items():
            got = ctx.fetch_gaussian(img, o, i)
            assert got.shape == plane.shape, (o, i, got.shape, plane.shape)
            bad = np.argwhere(got.view(np.uint32) != plane.view(np.uint32))
            assert bad.size == 0, f"image {img} octave {o} level {i}: {len(bad)} mismatches, first {bad[:4].tolist()}"


@pytest.mark.parametrize("shape", [(375, 1242), (400, 1800), (240, 700)])
def test_experimental_fused_octave_path_equals_default(vo, oracle, syn, shape):
    """The experimental k_octave path (octave.hip, compiled only into the test build
    libvo_exp.so and selected there by vo_exp_set: levels 1..5, extremum test and next base of
    each large octave in one launch) gives the same Gaussian planes, keypoints, descriptors and
    stereo pairs as the product libvo.so's per-level kernels, bit for bit."""
    import torch
    rows, cols = shape
    B = 2
    L = np.empty((B, rows, cols), np.uint8)
    R = np.empty((B, rows, cols), np.uint8)
    for f in range(B):
        L[f], R[f] = syn.stereo_pair(syn.SEED_BASE + 310 + f, rows, cols)
    dl, dr = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    torch.cuda.synchronize()
    if os.environ.get("VO_LIBPATH") and not vo.experimental_library_path().exists():
        pytest.skip("variant build without its own libvo_exp.so")
    exp = vo.load_experimental_library()
    outs = []
    for lib in (None, exp):
        if lib is not None:
            lib.vo_exp_set(1, 0)
        try:
            ctx = vo.Context(rows, cols, B, lib=lib)
            ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B)
            planes = [ctx.fetch_gaussian(img, o, i) for img in (0, 3) for o in range(3) for i in range(6)]
            kps = [ctx.fetch_keypoints(img) for img in range(2 * B)]
            pairs = [ctx.fetch_stereo_pairs(f) for f in range(B)]
            outs.append((planes, kps, pairs))
            ctx.close()
        finally:
            if lib is not None:
                lib.vo_exp_set(0, 0)
    (p0, k0, s0), (p1, k1, s1) = outs
    for a, b in zip(p0, p1):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    for (ka, da), (kb, db) in zip(k0, k1):
        assert ka.tobytes() == kb.tobytes() and np.array_equal(da, db)
    for a, b in zip(s0, s1):
        assert np.array_equal(a, b)
    assert sum(len(ka) for ka, _ in k0) > 100 and sum(len(a) for a in s0) > 20
