"""GPU parity on edge cases: odd and tiny image sizes (including KITTI-00's real
376x1241), a blank image (no keypoints), and matchFeatures on empty, single-row,
duplicate and ragged descriptor sets (sizes that are not multiples of the 32-row
MFMA tile or the 512-column F2 chunk).  Everything is compared bit for bit with
the CPU oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [(376, 1241), (120, 200), (77, 101), (64, 64), (33, 47)]


def _same_kps(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for f in ("x", "y", "size", "angle", "response", "octave", "layer", "scale"):
        assert np.array_equal(a[f], b[f]), f


@pytest.mark.parametrize("rows,cols", SIZES)
def test_sift_odd_sizes_bit_exact(vo, oracle, syn, rows, cols):
    import torch
    L, R = syn.stereo_pair(syn.SEED_BASE + 31, rows, cols)
    ctx = vo.Context(rows, cols, 2)
    k, d = ctx.sift(L)
    rk, rd = oracle.sift(L)
    _same_kps(k, rk)
    assert np.array_equal(d, rd)
    # batch path: two frames (the second is the first mirrored), stereo matches included
    Ls = np.ascontiguousarray(np.stack([L, L[:, ::-1]]))
    Rs = np.ascontiguousarray(np.stack([R, R[:, ::-1]]))
    dl, dr = torch.from_numpy(Ls).cuda(), torch.from_numpy(Rs).cuda()
    torch.cuda.synchronize()
    ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), 2)
    for f in range(2):
        kl, dsl = ctx.fetch_keypoints(2 * f)
        kr, dsr = ctx.fetch_keypoints(2 * f + 1)
        rkl, rdl = oracle.sift(Ls[f])
        rkr, rdr = oracle.sift(Rs[f])
        _same_kps(kl, rkl)
        _same_kps(kr, rkr)
        assert np.array_equal(dsl, rdl) and np.array_equal(dsr, rdr)
        assert np.array_equal(ctx.fetch_stereo_pairs(f), oracle.match(rdl, rdr))
    ctx.close()


def test_blank_image_has_no_keypoints(vo):
    import torch
    Z = np.zeros((1, 100, 160), np.uint8)
    ctx = vo.Context(100, 160, 1)
    k, d = ctx.sift(Z[0])
    assert len(k) == 0 and d.shape == (0, 128)
    dz = torch.from_numpy(Z).cuda()
    torch.cuda.synchronize()
    stats = ctx.sift_match_batch_dev(dz.data_ptr(), dz.data_ptr(), 1)
    assert tuple(stats[0][:3]) == (0, 0, 0)
    assert len(ctx.fetch_stereo_pairs(0)) == 0
    ctx.close()


def test_match_edge_cases_bit_exact(vo, oracle):
    rng = np.random.default_rng(5)
    F = rng.integers(0, 100, (10, 128)).astype(np.uint8)
    ctx = vo.Context(375, 1242, 1)
    cases = [
        (F, F[:0]), (F[:0], F),                       # empty sides
        (F, F[3:4]),                                  # a single candidate: ratio test passes
        (F, F),                                       # identity pairs
        (F[:1], np.vstack([F[:1], F[:1]])),           # exact duplicate best: 0/0 ratio, rejected
        (F, np.vstack([F[5:6], F, F[5:6]])),          # duplicates among many
    ]
    for F1, F2 in cases:
        got = ctx.match(F1, F2)
        ref = oracle.match(F1, F2)
        assert np.array_equal(got, ref), (F1.shape, F2.shape)
    assert ctx.match(F, F[3:4]).tolist() == [[4, 1]]
    ctx.close()


@pytest.mark.parametrize("n1,n2", [(1, 1), (31, 33), (33, 511), (513, 513), (1025, 1100), (70, 2049)])
def test_match_ragged_sizes_bit_exact(vo, oracle, n1, n2):
    rng = np.random.default_rng(n1 * 7919 + n2)
    base = rng.integers(0, 140, (max(n1, n2) + 64, 128)).astype(np.uint8)
    F1 = base[:n1].copy()
    # F2: noisy copies of a shifted window of the same rows, so many rows have a true match
    F2 = np.clip(base[32:32 + n2].astype(int) + rng.integers(-4, 5, (n2, 128)), 0, 255).astype(np.uint8)
    ctx = vo.Context(375, 1242, 1)
    got = ctx.match(F1, F2)
    ref = oracle.match(F1, F2)
    assert np.array_equal(got, ref)
    ctx.close()


def test_match_f32_storage_orders_equal_u8_match(vo, oracle, syn):
    """vo_match_f32 (single rows with ld and a storage-order flag, so a MEX gateway
    passes MATLAB's column-major extractFeatures output zero-copy) == vo_match == oracle."""
    L, R = syn.stereo_pair(syn.SEED_BASE + 77)
    _, dl = oracle.sift(L)
    _, dr = oracle.sift(R)
    ref = oracle.match(dl, dr)
    ctx = vo.Context(375, 1242, 1)
    assert np.array_equal(ctx.match(dl, dr), ref)
    fl, fr = dl.astype(np.float32), dr.astype(np.float32)
    assert np.array_equal(ctx.match_f32(np.asfortranarray(fl), np.asfortranarray(fr)), ref)   # MATLAB layout
    assert np.array_equal(ctx.match_f32(fl, fr), ref)                                         # row-major
    pad = np.zeros((fl.shape[0], 160), np.float32)
    pad[:, :128] = fl
    assert np.array_equal(ctx.match_f32(pad[:, :128], fr), ref)                               # row stride 160
    assert len(ctx.match_f32(np.zeros((0, 128), np.float32), fr)) == 0
    # one non-integer value: the whole call takes the float SSD spec (oracle_match_f32)
    gen = fl.copy()
    gen[3, 7] = 0.5
    assert np.array_equal(ctx.match_f32(gen, fr), oracle.match_f32(gen, fr))
    ctx.close()


@pytest.mark.parametrize("n1,n2", [(300, 500), (1, 1), (7, 1), (0, 5), (5, 0), (2100, 2300)])
def test_match_f32_general_features_equal_oracle(vo, oracle, n1, n2):
    """vo_match_f32 on general single features (not u8-valued: matchFeatures for any other MATLAB
    caller of the path-shadowed function) == the oracle's float SSD restatement bit for bit, in
    both storage orders: near-duplicate rows (matches), exact duplicates (0/0 ratio: rejected),
    a single candidate (ratio 0: accepted), zero rows, and F2 beyond one 64-column lane sweep."""
    rng = np.random.default_rng(n1 * 7 + n2)
    F2 = rng.standard_normal((n2, 128)).astype(np.float32)
    F1 = rng.standard_normal((n1, 128)).astype(np.float32)
    if n1 and n2:
        k = min(n1, n2) // 2
        pick = rng.integers(0, n2, k)
        F1[:k] = F2[pick] + 0.02 * rng.standard_normal((k, 128)).astype(np.float32)   # near duplicates
        if n2 > 3 and n1 > k + 1:
            F2[1] = F2[0]
            F1[k] = F2[0]                                                             # exact duplicate pair in F2
            F1[k + 1] = 0.0                                                           # zero row
    ref = oracle.match_f32(F1, F2)
    ctx = vo.Context(375, 1242, 1)
    got = ctx.match_f32(F1, F2)
    assert np.array_equal(got, ref), (len(got), len(ref))
    assert np.array_equal(ctx.match_f32(np.asfortranarray(F1), np.asfortranarray(F2)), ref)
    if n1 > 10 and n2 > 10:
        assert len(ref) >= min(n1, n2) // 2 - 2
    ctx.close()


def test_column_major_images_equal_row_major(vo, oracle, syn):
    """vo_sift_ex / vo_step_batch_ex with col_major = 1 (MATLAB storage, device-side transpose)
    give the row-major results bit for bit: SIFT of one image, and the loop body of 3 frames
    (poses, landmark map)."""
    L, R = syn.stereo_pair(syn.SEED_BASE + 88)
    ctx = vo.Context(375, 1242, 3, calib=vo.calib_from(syn.KITTI00_P0, syn.KITTI00_P1))
    k0, d0 = ctx.sift(L)
    k1, d1 = ctx.sift(np.asfortranarray(L))
    assert len(k0) > 500 and np.array_equal(k0, k1) and np.array_equal(d0, d1)
    rk, rd = oracle.sift(L)
    assert np.array_equal(k0, rk) and np.array_equal(d0, rd)
    SL, SR, _ = syn.sequence(3)
    a = ctx.step_batch(SL, SR)
    la = ctx.get_landmarks()
    ctx.reset()
    b = ctx.step_batch(SL, SR, col_major=True)
    lb = ctx.get_landmarks()
    assert a.tobytes() == b.tobytes() and np.array_equal(la, lb)
    ctx.close()


def test_padded_and_flipped_views(vo, oracle, syn):
    """Strided host views through vo_sift_ex: a padded Fortran view (ld > rows, the staging copy
    stops at the last pixel rather than ld * cols bytes), a padded row-major view, and flipped
    views (negative strides are packed on the host) -- all equal the oracle on the same pixels."""
    L, _ = syn.stereo_pair(syn.SEED_BASE + 89)
    ctx = vo.Context(375, 1242, 1)
    rk, rd = oracle.sift(L)
    big = np.zeros((390, 1242), np.uint8, order="F")
    big[10:385] = L
    view = big[10:385]                                    # Fortran, ld = 390 > rows = 375
    assert view.strides == (1, 390)
    k, d = ctx.sift(view)
    assert np.array_equal(k, rk) and np.array_equal(d, rd)
    wide = np.zeros((375, 1300), np.uint8)
    wide[:, :1242] = L
    k, d = ctx.sift(wide[:, :1242])                       # row-major, ld = 1300
    assert np.array_equal(k, rk) and np.array_equal(d, rd)
    fk, fd = oracle.sift(np.ascontiguousarray(L[::-1]))
    k, d = ctx.sift(L[::-1])                              # negative row stride
    assert np.array_equal(k, fk) and np.array_equal(d, fd)
    k, d = ctx.sift(np.asfortranarray(L)[::-1])           # Fortran order, negative row stride
    assert np.array_equal(k, fk) and np.array_equal(d, fd)
    ctx.close()


def test_create_refuses_sigma_beyond_the_orientation_bound(vo):
    """k_orient's u32 column sums hold windows up to a bound (sift_params_supported);
    vo_create refuses a Sigma whose orientation windows could exceed it instead of wrapping a bin."""
    for sigma in (float("nan"), 0.0, -1.6, 40.0):
        p = vo.default_sift_params()
        p.sigma = sigma
        with pytest.raises(vo.VOError):
            vo.Context(64, 64, 1, sift=p)
    p = vo.default_sift_params()
    p.sigma = 4.0                                      # well inside the bound: accepted
    vo.Context(64, 64, 1, sift=p).close()


def test_candidate_overflow_is_reported(vo, syn):
    """With max_keypoints small enough that the candidate list (4 x max_keypoints) overflows,
    the extremum candidates k_seg_emit drops are reported: VO_FLAG_CANDIDATES in the batch
    stats and VO_ERR_CAPACITY from vo_sift (a truncated keypoint set never passes silently);
    the default capacity reports nothing."""
    import torch
    L, R = syn.independent_pairs(2, px_per_cell=syn.BENCH_PX_PER_CELL)
    dl = torch.from_numpy(L).cuda()
    dr = torch.from_numpy(R).cuda()
    torch.cuda.synchronize()
    small = vo.Context(375, 1242, 2, sift=vo.default_sift_params(64))
    st = small.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), 2)
    assert all(s[3] & 2 for s in st), st            # VO_FLAG_CANDIDATES
    with pytest.raises(vo.VOError) as e:
        small.sift(L[0])
    assert e.value.code == vo.VO_ERR_CAPACITY and "candidates" in str(e.value)
    small.close()
    full = vo.Context(375, 1242, 2)
    st = full.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), 2)
    assert all(s[3] == 0 for s in st), st
    full.close()
