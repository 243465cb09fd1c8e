"""Algorithmic byte model of the hot-path kernels.

SURVEY §8(d) prices the SIFT scale space as a materialised fp32 pyramid in
which every Gaussian and DoG level is written once and read once:
    B_img = W*H + 4 * (2*G + 2*D),  G = 6P, D = 5P,  P = sum of octave pixels.
libvo never materialises the DoG planes (D = G_{i+1} - G_i is formed inside the
extremum test and the refinement), so its kernels move fewer bytes than that
model; `pyramid_bytes_per_image` keeps the SURVEY figure for comparison and
`kernel_bytes` prices each launch by the bytes it must move given its own
inputs and outputs, each touched once.  bench.py's `roofline.achieved` =
bytes per launch / average launch duration of the dominant kernel.
"""
from __future__ import annotations

import math

import numpy as np

SMALL_PX = 9216   # csrc/sift.hip VO_SMALL_PX


def octave_dims(rows: int, cols: int, upsample: bool = True) -> list[tuple[int, int]]:
    R, C = (rows * 2, cols * 2) if upsample else (rows, cols)
    n = int(round(math.log2(min(R, C)) - 2)) + (1 if upsample else 0)
    dims = []
    for o in range(n):
        if o:
            R //= 2
            C //= 2
        dims.append((R, C))
    return dims


def pyramid_bytes_per_image(rows: int, cols: int, layers: int = 3) -> int:
    """SURVEY §8(d) model for one image (u8 read + fp32 G/D written+read once)."""
    P = sum(r * c for r, c in octave_dims(rows, cols))
    G, D = (layers + 3) * P, (layers + 2) * P
    return rows * cols + 4 * (2 * G + 2 * D)


FUSED_MIN_COLS, FUSED_MIN_ROWS = 256, 64   # csrc/octave.hip octave_fused_ok (default SIFT radii, 3 layers)


def fused_octaves(rows: int, cols: int, layers: int = 3, enabled: bool = False) -> int:
    """Octaves [0, n) the test build libvo_exp.so builds with k_octave when vo_exp_set selects it
    (levels 1..L+2, extremum test and the next base in one pass): the leading octaves at least
    256 columns wide and 64 rows tall.  The product libvo.so has no k_octave: 0 by default."""
    if layers != 3 or not enabled:
        return 0
    dims = octave_dims(rows, cols)
    o_small = next((o for o in range(1, len(dims)) if all(r * c <= SMALL_PX for r, c in dims[o:])), len(dims))
    n = 0
    while n < min(len(dims), o_small) and dims[n][1] >= FUSED_MIN_COLS and dims[n][0] >= FUSED_MIN_ROWS:
        n += 1
    return n


def kernel_bytes(rows: int, cols: int, n_img: int, layers: int = 3, fused: bool = False, ext_inner: bool = True) -> dict:
    """Algorithmic bytes per CALL (all launches of that kernel name in one
    batch of n_img images) and launches per call, per kernel name.  ext_inner: the
    extremum test as k_ext_inner (the default build, VO_EXT_INNER=1: G_1..G_{L+1} streamed,
    the outer levels checked by k_refine around candidates) instead of k_ext_stream (all L+3)."""
    dims = octave_dims(rows, cols)
    lv = layers + 2          # blurred levels per octave (1..L+2)
    n_fused = fused_octaves(rows, cols, layers, fused)
    out = {}

    def add(name, nbytes, launches):
        b, l = out.get(name, (0, 0))
        out[name] = (b + nbytes, l + launches)

    R0, C0 = dims[0]
    add("k_blur_base", n_img * (rows * cols + 4 * R0 * C0), 1)           # u8 in (x2 upsample fused), G0 out
    # octaves from o_small on are built by one k_blur_small launch in LDS (planes <= SMALL_PX)
    o_small = next((o for o in range(1, len(dims)) if all(r * c <= SMALL_PX for r, c in dims[o:])), len(dims))
    for o, (R, C) in enumerate(dims):
        px = R * C * n_img
        if o >= o_small:
            add("k_blur_small", 4 * px * (1 + lv), 1 if o == o_small else 0)  # decimated base in, G_0..G_{L+2} out
            continue
        # octave o's base (o >= 1, below o_small) is stored by the level-L blur of octave o - 1
        # (priced with k_blur_fused below); k_blur_small decimates its own first base
        if o < n_fused:
            # k_octave: G_0 in once, G_1..G_{L+2} out once, the next octave's base out (1/4 px)
            nxt = 4 * dims[o + 1][0] * dims[o + 1][1] * n_img if o + 1 < len(dims) else 0
            add(f"k_octave_o{o}", 4 * px * (1 + lv) + nxt, 1)
            continue
        nb = 4 * dims[o + 1][0] * dims[o + 1][1] * n_img if o + 1 < o_small else 0
        add("k_blur_fused", 8 * px * lv + nb, lv)                         # G_{i-1} in, G_i out (+ next base)
    # extremum test reads the L+1 (k_ext_inner) or L+3 (k_ext_stream) Gaussian levels of every
    # octave once (DoG formed on chip)
    # two launches when octave 0 is tested separately (on the feature stream, beside the scale
    # space of octaves 1..; the rest at the scale space's tail)
    nlev = layers + 1 if ext_inner else layers + 3
    ext = sum(4 * nlev * r * c for o, (r, c) in enumerate(dims) if o >= n_fused) * n_img
    if ext:
        add(f"k_ext_{'inner' if ext_inner else 'stream'}<{layers}>", ext, 2 if n_fused == 0 and len(dims) > 1 else 1)
    return out


# ---------------------------------------------------------------------------
# Feature stages (VO.m:79-87: detectSIFTFeatures after the scale space, extractFeatures,
# matchFeatures).  Their reads are windows around candidates and keypoints, so the model
# prices each launch from the call's counts (candidates, accepted candidates, keypoint scales
# and angles, match sizes) two ways:
#   algorithmic : the bytes the arithmetic needs, each 4-B value once;
#   line_floor  : the 128-B lines those windows occupy (HBM moves whole lines: a window row of
#                 w floats at a random 4-B offset spans 1 + (4w - 4) / 128 lines on average).
# tools/fetch_calib.hip measured FETCH_SIZE at exactly half the 128-B line bytes for these
# access shapes too (profiles/r06_c_fetch_calib.txt), so PMC (FETCH_SIZE x 2 + WRITE_SIZE)
# over line_floor is the over-fetch beyond the line granularity: re-reads of lines evicted
# between two uses.
# ---------------------------------------------------------------------------
BORDER = 5                # VO_SIFT_BORDER
SEG_WORDS = 1024          # VO_SEG_WORDS
MAX_PEAKS = 18            # VO_SIFT_MAX_PEAKS
CANDOUT_BYTES = 48 + 4 * (MAX_PEAKS + 2)
KP_BYTES = 32             # vo_keypoint; the internal KpInt record is 32 B too
DESC_BYTES = 128 + 8      # u8 descriptor + DescMeta
MATCH_CHUNK = 4096        # VO_MATCH_CHUNK
ORI_RADIUS, DESCR_SCL, DESCR_WIDTH = 4.5, 3.0, 4


def mask_geometry(rows: int, cols: int, layers: int = 3, upsample: bool = True) -> tuple[int, int]:
    """(mask words, 1024-word segments) of one image (csrc/sift.hip build_pyramid_geometry)."""
    w = 0
    for R, C in octave_dims(rows, cols, upsample):
        ir, ic = max(R - 2 * BORDER, 0), max(C - 2 * BORDER, 0)
        wrow = ((C - BORDER - 1) // 64 + 2) // 2 * 2 if ic > 0 else 0
        w += layers * ir * wrow
    return w, (w + SEG_WORDS - 1) // SEG_WORDS


def _lines(width_floats):
    """Expected 128-B lines of a row segment of `width_floats` floats at a random 4-B offset."""
    return 1.0 + (4.0 * np.maximum(width_floats, 1) - 4.0) / 128.0


def feature_bytes(rows: int, cols: int, n_cand, n_acc, kp_size, kp_octave, kp_angle, kp_image,
                  matches, layers: int = 3) -> dict:
    """Per-call byte model of the feature kernels of one batched call over n_img images.
    n_cand / n_acc: per image extremum candidates / accepted ones (vo_fetch_candidate_counts);
    kp_size / kp_octave / kp_angle / kp_image: every keypoint's Size, octave (-1 = upsampled),
    angle (degrees) and image; matches: per stereo frame (n_left, n_right, n_pairs).
    Returns {kernel: {"algorithmic": bytes, "line_floor": bytes}}."""
    n_cand = np.asarray(n_cand, np.float64)
    n_acc = np.asarray(n_acc, np.float64)
    n_img = len(n_cand)
    words, segs = mask_geometry(rows, cols, layers)
    C, A = float(n_cand.sum()), float(n_acc.sum())
    out = {}

    def put(name, alg, line=None):
        out[name] = {"algorithmic": float(alg), "line_floor": float(alg if line is None else line)}

    put("k_seg_count", n_img * (8 * words + 4 * segs))
    put("k_seg_scan", n_img * (8 * segs + 8))
    put("k_seg_emit", n_img * (8 * words + 4 * segs) + 4 * C)
    # k_refine: the candidate, the 3x3 DoG cube of its layer (4 Gaussian levels x 3 rows x 3
    # columns at its first position), its output record and peak count; the accepted list
    put("k_refine", C * (4 + 4 * 3 * 3 * 4 + CANDOUT_BYTES + 4) + 4 * A,
        C * (4 + 4 * 3 * _lines(3) * 128 + CANDOUT_BYTES + 4) + 4 * A)
    # octave-relative scale of each keypoint (Size = 2 scl 2^octave)
    size = np.asarray(kp_size, np.float64)
    octv = np.asarray(kp_octave, np.float64)
    scl = size / (2.0 * np.exp2(octv))
    # k_orient: one window per accepted candidate (keypoints of one candidate share it: unique
    # (image, size, octave) rows stand for the candidates), (2r+1)^2 samples + the 1-px gradient
    # border, r = round(4.5 scl)
    key = np.stack([np.asarray(kp_image, np.float64), size, octv], 1)
    _, first = np.unique(key, axis=0, return_index=True)
    r = np.floor(ORI_RADIUS * scl[first] + 0.5)
    side = 2 * r + 3
    scale_acc = A / max(len(first), 1)                   # candidates accepted but without a keypoint: none expected
    put("k_orient", scale_acc * float(np.sum(side * side * 4)) + A * (4 + CANDOUT_BYTES),
        scale_acc * float(np.sum(side * _lines(side) * 128)) + A * (4 + CANDOUT_BYTES))
    put("k_scan_cands", C * 8 + 4 * n_img)
    n_kp = len(size)
    put("k_expand", A * CANDOUT_BYTES + C * 4 + n_kp * 2 * KP_BYTES)
    # k_desc: the rotated square of side (d+1) hist_width (hist_width = 3 scl) the sample loop
    # visits, plus its 1-px gradient border; vertical extent s (|cos| + |sin|)
    s = (DESCR_WIDTH + 1) * DESCR_SCL * scl + 2.0
    th = np.radians(np.asarray(kp_angle, np.float64))
    ext = s * (np.abs(np.cos(th)) + np.abs(np.sin(th)))
    area = s * s
    put("k_desc", float(np.sum(area * 4)) + n_kp * (2 * KP_BYTES + DESC_BYTES),
        float(np.sum(ext + (4 * area - 4 * ext) / 128.0) * 128) + n_kp * (2 * KP_BYTES + DESC_BYTES))
    m = np.asarray(matches, np.float64).reshape(-1, 3)
    n1, n2, P = m[:, 0], m[:, 1], m[:, 2]
    nch = np.ceil(n2 / MATCH_CHUNK)
    put("k_match_partial", float(np.sum((n1 + n2) * DESC_BYTES + 16 * n1 * nch)))
    put("k_match_finish", float(np.sum(16 * n1 * nch + 8 * P + 4)))
    return out
