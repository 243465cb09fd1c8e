"""Synthetic stereo sequences rendered along a KITTI ground-truth trajectory
(BASELINE.json configs[2]/[3]: "full per-frame path on KITTI-00", "KITTI-00
4500-frame run").

The KITTI-00 images are not available anywhere in this pipeline, but the
reference holds the sequence's ground-truth camera trajectory
(`kitti/poses/00.txt`, 4541 camera-to-world poses, 3.7 km) and calibration
(`kitti/00/calib.txt`).  This module builds a street world around that
trajectory and ray-casts the left/right images of every frame, so the VO loop
runs the real KITTI-00 motion (speeds, turns, stops, 4541 frames) at KITTI's
376x1241 with KITTI-00's P0/P1, and its output can be scored with the
reference's own accuracy metric (`PlotOnMap.m:8-20`, lagged xz error) and ATE
against the exact trajectory the images were rendered from.

World (x right, y down, z forward = KITTI camera-0 frame of frame 0):
  * a grid of 3 m cells over the trajectory's bounding box (+150 m);
  * street cells = within `street_half_width` of a trajectory sample, plus a
    random fringe of open cells (set-backs, plazas) so depths vary;
  * every other cell is a building: vertical facades from the local ground up
    to a random roof height (6-24 m);
  * terraced ground: each cell's ground is 1.65 m below the camera height of
    the nearest trajectory sample (KITTI's camera height);
  * facades and ground carry smooth lattice noise defined in world
    coordinates (per-cell seeds), the sky is flat;
  * sensor noise: a per-(frame, camera, pixel) integer hash, Box-Muller,
    sd 2 grey levels -- no RNG state, so any frame renders identically on any
    rank, in any chunking, in any order.

The renderer is torch code that runs on the GPU (or the CPU for the small test
sequences) and is strictly element-wise per ray: a frame's pixels do not
depend on which other frames share the launch.  It is input generation, never
inside a timed region.
"""
from __future__ import annotations

import math
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
KITTI00_POSES = ROOT / "data" / "kitti" / "poses_00.txt"
KITTI00_CALIB = ROOT / "data" / "kitti" / "calib_00.txt"
KITTI_ROWS, KITTI_COLS = 376, 1241
CAM_HEIGHT = 1.65


def kitti00_gt() -> np.ndarray:
    """KITTI-00 ground truth, [4541, 4, 4] camera-to-world (reference kitti/poses/00.txt)."""
    from .kitti import read_poses
    return read_poses(KITTI00_POSES)


def kitti00_calib() -> tuple[np.ndarray, np.ndarray]:
    """(P0, P1) of reference kitti/00/calib.txt (VO.m:23-32)."""
    from .kitti import read_calib
    c = read_calib(KITTI00_CALIB)
    return c["P0"], c["P1"]


def _mix64(h):
    """splitmix64-style finaliser on int64 tensors (wrapping arithmetic)."""
    h = h ^ (h >> 31)
    h = h * 0x3C79AC492BA7B653
    h = h ^ (h >> 29)
    h = h * 0x1C69B3F74AC4AE35
    return h ^ (h >> 32)


class StreetWorld:
    """Street-canyon world around a trajectory (camera centres [n, 3])."""

    def __init__(self, centres: np.ndarray, seed: int = 0x5EED00, cell: float = 3.0,
                 street_half_width: float = 7.0, margin: float = 150.0, open_fringe: float = 0.3,
                 facade_spacing: float = 0.49, ground_spacing: float = 0.38, device="cpu"):
        import torch
        from scipy.spatial import cKDTree
        c = np.asarray(centres, np.float64)
        self.cell = float(cell)
        self.x0 = math.floor((c[:, 0].min() - margin) / cell) * cell
        self.z0 = math.floor((c[:, 2].min() - margin) / cell) * cell
        self.nx = int(math.ceil((c[:, 0].max() + margin - self.x0) / cell))
        self.nz = int(math.ceil((c[:, 2].max() + margin - self.z0) / cell))
        gx = self.x0 + (np.arange(self.nx) + 0.5) * cell
        gz = self.z0 + (np.arange(self.nz) + 0.5) * cell
        X, Z = np.meshgrid(gx, gz, indexing="ij")
        tree = cKDTree(c[:, [0, 2]])
        q = np.stack([X.ravel(), Z.ravel()], 1)
        dist, near = tree.query(q)
        # ground: inverse-distance blend of the 16 nearest samples' camera heights (smooth across
        # the places where the trajectory passes twice)
        dk, nk = tree.query(q, k=16)
        wk = 1.0 / np.maximum(dk, 1.0) ** 2
        ground = (c[nk, 1] * wk).sum(1) / wk.sum(1) + CAM_HEIGHT      # y down: ground below camera
        rng = np.random.default_rng(seed)
        fringe = (dist >= street_half_width) & (dist < street_half_width + 4 * cell)
        free = (dist < street_half_width) | (fringe & (rng.random(dist.size) < open_fringe))
        roof = ground - rng.uniform(6.0, 24.0, dist.size)
        self.device = torch.device(device)
        t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=self.device)  # noqa: E731
        self.occ = t(~free, torch.bool)
        self.ground = t(ground)
        self.roof = t(roof)
        self.cell_seed = t(rng.integers(1, 1 << 30, dist.size), torch.int64)
        self.facade_spacing = facade_spacing
        self.ground_spacing = ground_spacing
        self.gauss = t(np.random.default_rng(12345).standard_normal(1 << 20))

    # ---- texture: two-octave value noise on a hashed Gaussian lattice ----
    def _noise(self, u, v, spacing, seed):
        import torch
        out = torch.zeros_like(u)
        amp2 = 0.0
        for k, (octv, amp) in enumerate(((1.0, 1.0), (0.5, 0.35))):
            s = spacing * octv
            gu, gv = u / s, v / s
            iu, iv = torch.floor(gu), torch.floor(gv)
            fu, fv = gu - iu, gv - iv
            wu = fu * fu * fu * (fu * (fu * 6 - 15) + 10)
            wv = fv * fv * fv * (fv * (fv * 6 - 15) + 10)
            iu, iv = iu.to(torch.int64), iv.to(torch.int64)
            sd = seed * 7 + k * 0x9E3779B97F4A7C1

            def lat(a, b):
                return self.gauss[_mix64(a * 73856093 ^ b * 19349663 ^ sd) & ((1 << 20) - 1)]
            v00, v10, v01, v11 = lat(iu, iv), lat(iu + 1, iv), lat(iu, iv + 1), lat(iu + 1, iv + 1)
            top = v00 + (v10 - v00) * wu
            bot = v01 + (v11 - v01) * wu
            out = out + amp * (top + (bot - top) * wv)
            amp2 += amp * amp
        return out / math.sqrt(amp2) * 1.35

    # ---- ray casting ----
    def cast(self, o, d, max_range: float = 160.0):
        """Rays o + t d (o [N, 3], d [N, 3], float64 tensors) -> (kind [N] int8: 0 sky, 1 facade
        crossed along x, 2 facade crossed along z, 3 ground; t [N]; cell [N])."""
        import torch
        N = o.shape[0]
        dev = o.device
        kind = torch.zeros(N, dtype=torch.int8, device=dev)
        thit = torch.zeros(N, dtype=torch.float64, device=dev)
        chit = torch.zeros(N, dtype=torch.int64, device=dev)
        c = self.cell
        fx = (o[:, 0] - self.x0) / c
        fz = (o[:, 2] - self.z0) / c
        ix, iz = torch.floor(fx).to(torch.int64), torch.floor(fz).to(torch.int64)
        dx, dy, dz = d[:, 0], d[:, 1], d[:, 2]
        inf = torch.full_like(dx, float("inf"))
        sx = torch.where(dx > 0, 1, -1).to(torch.int64)
        sz = torch.where(dz > 0, 1, -1).to(torch.int64)
        bx = torch.where(dx > 0, ix + 1, ix).to(torch.float64)
        bz = torch.where(dz > 0, iz + 1, iz).to(torch.float64)
        tmx = torch.where(dx != 0, (bx - fx) * c / dx, inf)
        tmz = torch.where(dz != 0, (bz - fz) * c / dz, inf)
        tdx = torch.where(dx != 0, c / dx.abs(), inf)
        tdz = torch.where(dz != 0, c / dz.abs(), inf)
        tin = torch.zeros_like(dx)
        act = torch.arange(N, device=dev)
        oy = o[:, 1]
        max_steps = int(2 * max_range / c) + 4
        for _ in range(max_steps):
            if act.numel() == 0:
                break
            cid = ix * self.nz + iz
            # ground inside the current cell's segment [tin, tout]
            tout = torch.minimum(tmx, tmz)
            g = self.ground[cid]
            tg = torch.where(dy > 0, (g - oy) / dy, float("inf"))
            below = (oy + tin * dy) > g                                # entered below this cell's ground (a terrace step)
            hit_g = ((tg <= tout) & (tg >= tin)) | below
            tg = torch.where(below, tin, tg)
            # step into the next cell
            use_x = tmx < tmz
            t_en = tout
            nix = torch.where(use_x, ix + sx, ix)
            niz = torch.where(use_x, iz, iz + sz)
            tmx = torch.where(use_x, tmx + tdx, tmx)
            tmz = torch.where(use_x, tmz, tmz + tdz)
            out = (nix < 0) | (nix >= self.nx) | (niz < 0) | (niz >= self.nz) | (t_en > max_range)
            ncid = (nix.clamp(0, self.nx - 1)) * self.nz + niz.clamp(0, self.nz - 1)
            hit_w = ~out & self.occ[ncid] & ((oy + t_en * dy) > self.roof[ncid])
            fin = hit_g | hit_w | out
            k = torch.where(hit_g, 3, torch.where(hit_w, torch.where(use_x, 1, 2), 0)).to(torch.int8)
            tt = torch.where(hit_g, tg, t_en)
            cc = torch.where(hit_g, cid, ncid)
            kind[act[fin]] = k[fin]
            thit[act[fin]] = tt[fin]
            chit[act[fin]] = cc[fin]
            keep = ~fin
            act = act[keep]
            ix, iz, tmx, tmz, tin = nix[keep], niz[keep], tmx[keep], tmz[keep], t_en[keep]
            sx, sz, tdx, tdz = sx[keep], sz[keep], tdx[keep], tdz[keep]
            dx, dy, dz, oy = dx[keep], dy[keep], dz[keep], oy[keep]
        return kind, thit, chit

    def shade(self, o, d, kind, t, cid):
        """Texture value (zero-mean, ~unit sd) of every ray hit; sky = 0."""
        import torch
        P = o + t[:, None] * d
        val = torch.zeros_like(t)
        seed = self.cell_seed[cid]
        fa = (kind == 1) | (kind == 2)
        if fa.any():
            u = torch.where(kind[fa] == 1, P[fa, 2], P[fa, 0])
            val[fa] = self._noise(u, P[fa, 1], self.facade_spacing, seed[fa])
        gr = kind == 3
        if gr.any():
            val[gr] = 0.6 * self._noise(P[gr, 0], P[gr, 2], self.ground_spacing, seed[gr] + 0x51ED)
        return val


def _pixel_noise(base, idx, sd: float = 2.0):
    """N(0, sd^2) per (frame, camera, pixel) from an integer hash (Box-Muller); `base` [N]
    int64 = (frame * 2 + camera) * 0x100000001B3 + 0x5EED, `idx` [N] pixel index."""
    import torch
    h1 = _mix64(idx * 2 + base)
    h2 = _mix64(idx * 2 + 1 + base * 7)
    u1 = ((h1 >> 11) & ((1 << 53) - 1)).to(torch.float64) * (1.0 / (1 << 53)) + 2.0 ** -54
    u2 = ((h2 >> 11) & ((1 << 53) - 1)).to(torch.float64) * (1.0 / (1 << 53))
    return sd * torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2 * math.pi * u2)


def render_frames(world: StreetWorld, poses: np.ndarray, frames, P0: np.ndarray, P1: np.ndarray,
                  rows: int = KITTI_ROWS, cols: int = KITTI_COLS, chunk: int = 16, out=None):
    """Left/right u8 images of `frames` (global indices into `poses`, [n, 4, 4] camera-to-world
    of the left camera) as torch tensors [len(frames), rows, cols] on the world's device
    (or into `out` = (L, R) of that shape).  `chunk` frames (2 * chunk images) are cast in one
    pass; every per-ray operation is element-wise, so the pixels do not depend on `chunk`."""
    import torch
    dev = world.device
    frames = [int(f) for f in frames]
    K = P0[:, :3]
    base = -P1[0, 3] / P1[0, 0] + P0[0, 3] / P0[0, 0]          # 0.537 m for KITTI-00
    npix = rows * cols
    pix = torch.arange(npix, dtype=torch.int64, device=dev)
    xn_img = ((pix % cols).to(torch.float64) - K[0, 2]) / K[0, 0]
    yn_img = ((pix // cols).to(torch.float64) - K[1, 2]) / K[1, 1]
    if out is None:
        L = torch.empty((len(frames), rows, cols), dtype=torch.uint8, device=dev)
        R = torch.empty_like(L)
    else:
        L, R = out
    for c0 in range(0, len(frames), chunk):
        fr = frames[c0:c0 + chunk]
        n = len(fr)
        Rw = np.stack([np.asarray(poses[f], np.float64)[:3, :3] for f in fr])
        cen = np.stack([np.asarray(poses[f], np.float64)[:3, 3] for f in fr])
        cen_r = np.stack([cen[k] + Rw[k] @ np.array([base, 0.0, 0.0]) for k in range(n)])
        # images of the chunk: [left of each frame, right of each frame]
        Rimg = torch.as_tensor(np.concatenate([Rw, Rw]), device=dev)
        Cimg = torch.as_tensor(np.concatenate([cen, cen_r]), device=dev)
        fidx = torch.as_tensor(fr + fr, dtype=torch.int64, device=dev)
        cam = torch.as_tensor([0] * n + [1] * n, dtype=torch.int64, device=dev)
        img = torch.arange(2 * n, device=dev).repeat_interleave(npix)
        xn, yn, p = xn_img.repeat(2 * n), yn_img.repeat(2 * n), pix.repeat(2 * n)
        Ri = Rimg[img]
        # element-wise d = Rwc @ [xn, yn, 1] (no GEMM: per-ray arithmetic is chunking-independent)
        d = torch.stack([Ri[:, a, 0] * xn + Ri[:, a, 1] * yn + Ri[:, a, 2] for a in range(3)], 1)
        del Ri, xn, yn
        o = Cimg[img]
        kind, t, cid = world.cast(o, d)
        val = world.shade(o, d, kind, t, cid)
        del o, d, t, cid, kind
        nb = (fidx * 2 + cam) * 0x100000001B3 + 0x5EED
        v = 128.0 + 40.0 * val + _pixel_noise(nb[img], p)
        u8 = torch.clamp(torch.round(v), 0, 255).to(torch.uint8).view(2 * n, rows, cols)
        L[c0:c0 + n] = u8[:n]
        R[c0:c0 + n] = u8[n:]
        del v, u8, val, img, p
    return L, R


def kitti00_world(device="cpu", poses: np.ndarray | None = None) -> StreetWorld:
    gt = kitti00_gt() if poses is None else poses
    return StreetWorld(gt[:, :3, 3], device=device)
