"""GPU parity: SIFT detect+describe and stereo matchFeatures through libvo.so
vs the CPU oracle, bit for bit (keypoint records, descriptors, index pairs)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same_kps(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for f in ("x", "y", "size", "angle", "response", "octave", "layer", "scale"):
        assert np.array_equal(a[f], b[f]), f


def test_sift_single_image_bit_exact(vo, oracle, syn):
    L, R = syn.stereo_pair(syn.SEED_BASE + 7)
    ctx = vo.Context(375, 1242, 1)
    k_gpu, d_gpu = ctx.sift(L)
    k_ref, d_ref = oracle.sift(L)
    assert len(k_ref) > 1000
    _same_kps(k_gpu, k_ref)
    assert np.array_equal(d_gpu, d_ref)


def test_sift_match_batch_bit_exact(vo, oracle, syn):
    import torch
    B = 3
    L, R = syn.independent_pairs(B)
    ctx = vo.Context(375, 1242, B)
    dl = torch.from_numpy(L).cuda()
    dr = torch.from_numpy(R).cuda()
    torch.cuda.synchronize()
    stats = ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B)
    for f in range(B):
        kl, dl_ = ctx.fetch_keypoints(2 * f)
        kr, dr_ = ctx.fetch_keypoints(2 * f + 1)
        rkl, rdl = oracle.sift(L[f])
        rkr, rdr = oracle.sift(R[f])
        _same_kps(kl, rkl)
        _same_kps(kr, rkr)
        assert np.array_equal(dl_, rdl) and np.array_equal(dr_, rdr)
        pairs = ctx.fetch_stereo_pairs(f)
        ref = oracle.match(rdl, rdr)
        assert stats[f][2] == len(ref)
        assert np.array_equal(pairs, ref)


def test_match_host_bit_exact(vo, oracle):
    rng = np.random.default_rng(3)
    base = rng.integers(0, 120, (700, 128)).astype(np.uint8)
    F1 = base[:500].copy()
    F2 = np.clip(base[100:].astype(int) + rng.integers(-3, 4, (600, 128)), 0, 255).astype(np.uint8)
    F2[7] = F2[8]                       # exact duplicate -> ratio test edge
    ctx = vo.Context(375, 1242, 1)
    got = ctx.match(F1, F2)
    ref = oracle.match(F1, F2)
    assert len(ref) > 100
    assert np.array_equal(got, ref)


def test_stream_concurrency_is_invisible(vo, syn):
    """Splitting a batch over 1, 2, 3 or 4 forked streams gives identical results."""
    import torch
    B = 5
    L, R = syn.independent_pairs(B)
    dl = torch.from_numpy(L).cuda()
    dr = torch.from_numpy(R).cuda()
    torch.cuda.synchronize()
    ctx = vo.Context(375, 1242, B)
    ref = None
    for n in (1, 2, 3, 4):
        ctx.set_concurrency(n)
        stats = ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B)
        got = [stats]
        for f in range(B):
            for i in (2 * f, 2 * f + 1):
                k, d = ctx.fetch_keypoints(i)
                got.append((k.tobytes(), d.tobytes()))
            got.append(ctx.fetch_stereo_pairs(f).tobytes())
        if ref is None:
            ref = got
        else:
            assert got == ref, n
    with pytest.raises(Exception):
        ctx.set_concurrency(0)


@pytest.mark.parametrize("offset", [1, 3])
def test_misaligned_image_pointers(vo, oracle, syn, offset):
    """Device images at byte offsets (odd row pitch 1242, unaligned base) give the oracle's keypoints."""
    import torch
    B = 2
    L, R = syn.independent_pairs(B)
    n = L[0].size
    buf_l = torch.zeros(B * n + 16, dtype=torch.uint8, device="cuda")
    buf_r = torch.zeros(B * n + 16, dtype=torch.uint8, device="cuda")
    buf_l[offset:offset + B * n] = torch.from_numpy(L.reshape(-1)).cuda()
    buf_r[offset:offset + B * n] = torch.from_numpy(R.reshape(-1)).cuda()
    torch.cuda.synchronize()
    ctx = vo.Context(375, 1242, B)
    ctx.sift_match_batch_dev(buf_l.data_ptr() + offset, buf_r.data_ptr() + offset, B)
    for f in range(B):
        for img, src in ((2 * f, L[f]), (2 * f + 1, R[f])):
            k, d = ctx.fetch_keypoints(img)
            rk, rd = oracle.sift(src)
            _same_kps(k, rk)
            assert np.array_equal(d, rd)


def test_batch_128_equals_two_batches_of_64(vo, oracle, syn):
    """A 128-frame batch (256 images + 2 carry slots in one scale-space arena)
    gives the same keypoints, descriptors and stereo matches as the same frames in two
    64-frame calls; frames at both ends are also checked against the oracle."""
    import torch
    B = 128
    L, R = syn.independent_pairs(B)
    dl = torch.from_numpy(L).cuda()
    dr = torch.from_numpy(R).cuda()
    torch.cuda.synchronize()

    def collect(ctx, n):
        out = []
        for f in range(n):
            kl, dsl = ctx.fetch_keypoints(2 * f)
            kr, dsr = ctx.fetch_keypoints(2 * f + 1)
            out.append((kl, dsl, kr, dsr, ctx.fetch_stereo_pairs(f)))
        return out

    big = vo.Context(375, 1242, B)
    big.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B)
    got = collect(big, B)
    big.close()
    half = vo.Context(375, 1242, 64)
    ref = []
    fs = L[0].size
    for b0 in (0, 64):
        half.sift_match_batch_dev(dl.data_ptr() + b0 * fs, dr.data_ptr() + b0 * fs, 64)
        ref += collect(half, 64)
    half.close()
    for f in range(B):
        for a, b in zip(got[f], ref[f]):
            assert np.array_equal(a, b), f
    for f in (0, B - 1):
        rkl, rdl = oracle.sift(L[f])
        assert np.array_equal(got[f][0], rkl) and np.array_equal(got[f][1], rdl), f


def test_bench_batches_256_and_512_equal_64_frame_calls(vo, oracle, syn):
    """The bench's own configuration: one 256-frame call (bench.py's default --batch) and one
    512-frame call (VO_MAX_BATCH; 1024 images + 2 carry slots, so `flat_find_wave`'s image
    search runs far past 258 slots) give every frame's keypoints, descriptors and stereo pairs
    exactly as the same frames in eight 64-frame calls; the first, a middle and the last frame
    are also checked against the oracle (VO.m:79-87).  128 rendered pairs are reused four times,
    each reuse rolled by a different column shift, so every one of the 512 frames is distinct."""
    import torch
    B = 512
    U = 128
    L0, R0 = syn.independent_pairs(U, px_per_cell=syn.BENCH_PX_PER_CELL, threads=16)
    L = np.concatenate([np.roll(L0, 37 * k, axis=2) for k in range(B // U)])
    R = np.concatenate([np.roll(R0, 37 * k, axis=2) for k in range(B // U)])
    dl = torch.from_numpy(L).cuda()
    dr = torch.from_numpy(R).cuda()
    torch.cuda.synchronize()
    fs = L[0].size

    def collect(ctx, n):
        out = []
        for f in range(n):
            kl, dsl = ctx.fetch_keypoints(2 * f)
            kr, dsr = ctx.fetch_keypoints(2 * f + 1)
            out.append((kl, dsl, kr, dsr, ctx.fetch_stereo_pairs(f)))
        return out

    small = vo.Context(375, 1242, 64)
    ref = []
    for b0 in range(0, B, 64):
        small.sift_match_batch_dev(dl.data_ptr() + b0 * fs, dr.data_ptr() + b0 * fs, 64)
        ref += collect(small, 64)
    small.close()
    assert min(len(r[0]) for r in ref) > 1000

    for n in (256, 512):
        ctx = vo.Context(375, 1242, n)
        stats = ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), n)
        got = collect(ctx, n)
        ctx.close()
        for f in range(n):
            assert stats[f][2] == len(ref[f][4]), (n, f)
            for a, b in zip(got[f], ref[f]):
                assert np.array_equal(a, b), (n, f)

    for f in (0, 255, B - 1):
        rkl, rdl = oracle.sift(L[f])
        rkr, rdr = oracle.sift(R[f])
        _same_kps(ref[f][0], rkl)
        _same_kps(ref[f][2], rkr)
        assert np.array_equal(ref[f][1], rdl) and np.array_equal(ref[f][3], rdr), f
        assert np.array_equal(ref[f][4], oracle.match(rdl, rdr)), f
