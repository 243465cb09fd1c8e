"""Seeded synthetic stereo scenes (BASELINE.md "Inputs").

KITTI-00 images are not available anywhere in this pipeline, so every
benchmark and parity run uses rendered stereo pairs with the KITTI-00
calibration (reference kitti/00/calib.txt:1-2, VO.m:24-48):

* textured fronto-parallel planes at 5-80 m (plus a far backdrop), rendered
  by ray casting for the left camera and the right camera (baseline
  386.1448 / 718.856 = 0.53717 m, so disparity = 386.14 / Z px);
* texture = smooth lattice noise defined in world coordinates on each plane
  (so the right view is the left view warped by the true disparity, with
  correct occlusions), mapped to u8 with mean 128 / sd 40;
* independent sensor noise N(0, 2^2) on both images;
* sequences: the camera moves 1 m forward per frame and yaws 0.3 deg per
  frame; ground-truth camera-to-world poses are returned for ATE.

Seeds: frame f of an independent-pairs batch uses seed 0x5EED0000 + f.
Pure numpy; this module is input generation, not the measured path.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

KITTI00_P0 = np.array([[718.856, 0.0, 607.1928, 0.0],
                       [0.0, 718.856, 185.2157, 0.0],
                       [0.0, 0.0, 1.0, 0.0]])
KITTI00_P1 = np.array([[718.856, 0.0, 607.1928, -386.1448],
                       [0.0, 718.856, 185.2157, 0.0],
                       [0.0, 0.0, 1.0, 0.0]])
SEED_BASE = 0x5EED0000
# BASELINE configs[4]: 1920x1080, ~8k keypoints per image.  At the default 16 px per texture
# cell the oracle finds ~6.8k; 14.5 px per cell gives 8k +- 10 % (tests/test_gpu_large.py).
LARGE_ROWS, LARGE_COLS, LARGE_PX_PER_CELL = 1080, 1920, 14.5
# BASELINE configs[1]: ~2k keypoints per 1242x375 image.  16 px per cell gives the oracle ~1790,
# 15 px ~2020 (16 pairs), inside SURVEY §8(d)'s 2000 +- 200.
BENCH_PX_PER_CELL = 15.0


@dataclass
class Plane:
    z: float          # world depth of the plane (fronto-parallel to frame 0)
    x0: float         # lateral extent [x0, x1] x [y0, y1] in metres
    x1: float
    y0: float
    y1: float
    spacing: float    # lattice spacing of the texture in metres
    seed: int


def _hash_gauss(ix: np.ndarray, iy: np.ndarray, seed: int, table: np.ndarray) -> np.ndarray:
    s = np.int64((seed * 83492791) & 0x7FFFFFFF)
    h = (ix.astype(np.int64) * 73856093) ^ (iy.astype(np.int64) * 19349663) ^ s
    h = (h ^ (h >> 13)) * 0x5BD1E995
    h = h ^ (h >> 15)
    return table[h & (table.size - 1)]


_GAUSS_TABLE = np.random.default_rng(12345).standard_normal(1 << 20).astype(np.float64)


def _lattice_noise(u: np.ndarray, v: np.ndarray, spacing: float, seed: int) -> np.ndarray:
    """Smooth value noise (quintic interpolation) with 2 octaves, ~unit variance."""
    out = np.zeros_like(u)
    amp_total = 0.0
    for octv, amp in ((1.0, 1.0), (0.5, 0.35)):
        s = spacing * octv
        gx, gy = u / s, v / s
        ix, iy = np.floor(gx), np.floor(gy)
        fx, fy = gx - ix, gy - iy
        wx = fx * fx * fx * (fx * (fx * 6 - 15) + 10)
        wy = fy * fy * fy * (fy * (fy * 6 - 15) + 10)
        sd = seed * 7 + int(octv * 16)
        v00 = _hash_gauss(ix, iy, sd, _GAUSS_TABLE)
        v10 = _hash_gauss(ix + 1, iy, sd, _GAUSS_TABLE)
        v01 = _hash_gauss(ix, iy + 1, sd, _GAUSS_TABLE)
        v11 = _hash_gauss(ix + 1, iy + 1, sd, _GAUSS_TABLE)
        top = v00 + (v10 - v00) * wx
        bot = v01 + (v11 - v01) * wx
        out += amp * (top + (bot - top) * wy)
        amp_total += amp * amp
    return out / math.sqrt(amp_total) * 1.35   # quintic interpolation shrinks variance


def random_scene(seed: int, rows: int, cols: int, f: float = 718.856,
                 zmin: float = 5.0, zmax: float = 80.0, n_planes: int | None = None,
                 px_per_cell: float = 16.0) -> list[Plane]:
    """6-10 planes at depths in [zmin, zmax] covering the view, plus a backdrop."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(6, 11)) if n_planes is None else n_planes
    planes = []
    cu, cv = KITTI00_P0[0, 2] * f / 718.856, KITTI00_P0[1, 2] * f / 718.856
    for i in range(n):
        z = float(np.exp(rng.uniform(np.log(zmin), np.log(zmax))))
        # frustum extent at depth z
        xl, xr = -cu / f * z, (cols - cu) / f * z
        yt, yb = -cv / f * z, (rows - cv) / f * z
        w = (xr - xl) * rng.uniform(0.25, 0.6)
        h = (yb - yt) * rng.uniform(0.3, 0.8)
        xc = rng.uniform(xl, xr)
        yc = rng.uniform(yt, yb)
        spacing = z * px_per_cell / f * float(rng.uniform(0.8, 1.25))
        planes.append(Plane(z, xc - w / 2, xc + w / 2, yc - h / 2, yc + h / 2, spacing, seed * 131 + i))
    zb = zmax * 1.5
    planes.append(Plane(zb, -1e6, 1e6, -1e6, 1e6, zb * px_per_cell / f, seed * 131 + 99))
    return planes


def _render(planes: list[Plane], R_wc: np.ndarray, c_w: np.ndarray, rows: int, cols: int,
            K: np.ndarray) -> np.ndarray:
    """Ray-cast the planes for a camera with orientation R_wc (cam->world) at centre c_w."""
    ys, xs = np.mgrid[0:rows, 0:cols].astype(np.float64)
    xn = (xs - K[0, 2]) / K[0, 0]
    yn = (ys - K[1, 2]) / K[1, 1]
    d = np.stack([xn, yn, np.ones_like(xn)], axis=-1) @ R_wc.T   # world ray directions
    best = np.full((rows, cols), np.inf)
    img = np.zeros((rows, cols))
    for p in planes:
        with np.errstate(divide="ignore", invalid="ignore"):
            t = (p.z - c_w[2]) / d[..., 2]
        X = c_w[0] + t * d[..., 0]
        Y = c_w[1] + t * d[..., 1]
        hit = (t > 0.1) & (t < best) & (X >= p.x0) & (X <= p.x1) & (Y >= p.y0) & (Y <= p.y1)
        if not hit.any():
            continue
        val = _lattice_noise(X[hit], Y[hit], p.spacing, p.seed)
        img[hit] = val
        best[hit] = t[hit]
    return img


def _to_u8(img: np.ndarray, rng: np.random.Generator, noise_sd: float) -> np.ndarray:
    out = 128.0 + 40.0 * img + rng.normal(0.0, noise_sd, img.shape)
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def baseline_m(P1: np.ndarray = KITTI00_P0, P2: np.ndarray = KITTI00_P1) -> float:
    return float(-P2[0, 3] / P2[0, 0] + P1[0, 3] / P1[0, 0])


def stereo_pair(seed: int, rows: int = 375, cols: int = 1242, noise_sd: float = 2.0,
                planes: list[Plane] | None = None, R_wc: np.ndarray | None = None,
                c_w: np.ndarray | None = None) -> tuple[np.ndarray, np.ndarray]:
    """One rectified stereo pair (left = P0 camera, right = P1 camera)."""
    K = KITTI00_P0[:, :3]
    if planes is None:
        planes = random_scene(seed, rows, cols)
    if R_wc is None:
        R_wc = np.eye(3)
    if c_w is None:
        c_w = np.zeros(3)
    B = baseline_m()
    left = _render(planes, R_wc, c_w, rows, cols, K)
    right = _render(planes, R_wc, c_w + R_wc @ np.array([B, 0.0, 0.0]), rows, cols, K)
    rng = np.random.default_rng(seed ^ 0xABCDEF)
    return _to_u8(left, rng, noise_sd), _to_u8(right, rng, noise_sd)


def independent_pairs(n: int, rows: int = 375, cols: int = 1242, first: int = 0,
                      px_per_cell: float = 16.0, threads: int = 1):
    """n independent stereo pairs; frame f uses seed 0x5EED0000 + f. -> (L, R) [n, rows, cols] u8.
    `threads` > 1 renders pairs concurrently (numpy releases the GIL in its array loops); every
    pair depends on its seed alone, so the result does not depend on `threads`."""
    L = np.empty((n, rows, cols), np.uint8)
    R = np.empty((n, rows, cols), np.uint8)

    def one(i):
        seed = SEED_BASE + first + i
        L[i], R[i] = stereo_pair(seed, rows, cols, planes=random_scene(seed, rows, cols, px_per_cell=px_per_cell))

    if threads > 1 and n > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(min(threads, n)) as ex:
            list(ex.map(one, range(n)))
    else:
        for i in range(n):
            one(i)
    return L, R


def large_pairs(n: int, first: int = 0, threads: int = 1):
    """BASELINE configs[4] inputs: n independent 1920x1080 pairs with ~8k keypoints per image."""
    return independent_pairs(n, LARGE_ROWS, LARGE_COLS, first, LARGE_PX_PER_CELL, threads)


def yaw(deg: float) -> np.ndarray:
    a = math.radians(deg)
    return np.array([[math.cos(a), 0.0, math.sin(a)], [0.0, 1.0, 0.0], [-math.sin(a), 0.0, math.cos(a)]])


def calib(scale: float = 1.0) -> tuple[np.ndarray, np.ndarray]:
    """KITTI-00 P0/P1 for an image scaled by `scale` (focal and principal point scale,
    the baseline stays 0.537 m)."""
    S = np.diag([scale, scale, 1.0])
    return S @ KITTI00_P0, S @ KITTI00_P1


def sequence(n: int, rows: int = 375, cols: int = 1242, seed: int = SEED_BASE, step_m: float = 1.0,
             yaw_deg: float = 0.3, zmin: float = 20.0, zmax: float = 120.0, scale: float = 1.0):
    """A moving-camera sequence.  Returns (L, R, gt) with gt [n, 4, 4] camera-to-world
    poses (frame 0 = identity), the quantity VO.m's `pose` estimates.  With
    scale != 1 the images are rendered with calib(scale) (use rows/cols to match)."""
    if scale != 1.0:
        return _sequence_scaled(n, rows, cols, seed, step_m, yaw_deg, zmin, zmax, scale)
    planes = random_scene(seed, rows, cols, zmin=zmin, zmax=zmax, n_planes=10)
    # widen planes so the moving camera keeps seeing texture
    for p in planes[:-1]:
        cx, w = (p.x0 + p.x1) / 2, (p.x1 - p.x0) * 1.6
        p.x0, p.x1 = cx - w / 2, cx + w / 2
    L = np.empty((n, rows, cols), np.uint8)
    R = np.empty((n, rows, cols), np.uint8)
    gt = np.zeros((n, 4, 4))
    c = np.zeros(3)
    for f in range(n):
        Rwc = yaw(yaw_deg * f)
        gt[f, :3, :3] = Rwc
        gt[f, :3, 3] = c
        gt[f, 3, 3] = 1.0
        L[f], R[f] = stereo_pair(seed + 1000 + f, rows, cols, planes=planes, R_wc=Rwc, c_w=c.copy())
        c = c + Rwc @ np.array([0.0, 0.0, step_m])
    return L, R, gt


def _sequence_scaled(n, rows, cols, seed, step_m, yaw_deg, zmin, zmax, scale):
    P0, _ = calib(scale)
    K = P0[:, :3]
    f = K[0, 0]
    planes = random_scene(seed, int(round(375 * scale)), int(round(1242 * scale)), f=f, zmin=zmin, zmax=zmax,
                          n_planes=10, px_per_cell=16.0 * scale)
    for p in planes[:-1]:
        cx, w = (p.x0 + p.x1) / 2, (p.x1 - p.x0) * 1.6
        p.x0, p.x1 = cx - w / 2, cx + w / 2
    B = baseline_m()
    L = np.empty((n, rows, cols), np.uint8)
    R = np.empty((n, rows, cols), np.uint8)
    gt = np.zeros((n, 4, 4))
    c = np.zeros(3)
    for fr in range(n):
        Rwc = yaw(yaw_deg * fr)
        gt[fr, :3, :3] = Rwc
        gt[fr, :3, 3] = c
        gt[fr, 3, 3] = 1.0
        left = _render(planes, Rwc, c.copy(), rows, cols, K)
        right = _render(planes, Rwc, c + Rwc @ np.array([B, 0.0, 0.0]), rows, cols, K)
        rng = np.random.default_rng((seed + 1000 + fr) ^ 0xABCDEF)
        L[fr], R[fr] = _to_u8(left, rng, 2.0), _to_u8(right, rng, 2.0)
        c = c + Rwc @ np.array([0.0, 0.0, step_m])
    return L, R, gt
