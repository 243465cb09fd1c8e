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
