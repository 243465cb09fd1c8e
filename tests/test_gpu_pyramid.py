"""GPU parity of the Gaussian scale space itself: every level of every octave of
libvo's pyramid (k_blur_base, the level blurs k_blur_stream, k_down,
k_blur_small) equals the CPU oracle's plane bit for bit, on assorted image sizes
(strip/band edges, reflect-101 borders on all four sides, odd widths)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [(375, 1242), (376, 1241), (240, 700), (97, 131), (131, 97), (400, 1800)]


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
