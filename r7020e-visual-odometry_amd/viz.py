"""Host-side visualisation: the figures VO.m saves every 100th frame
(`VO.m:168-199`), written without a plotting library:

* ``features_on_feed``  — ShowFeaturesOnFeed.m: the left frame with every current detection
  as a dark-green cross and each tracked point's previous -> current left position as a red
  segment (the reference's per-point distance labels are written to ``view.txt`` instead of
  being drawn);
* ``plot_on_map``       — PlotOnMap.m: ground truth (black) and estimate (dashed) in the
  xz plane, returning the reference's lagged xz error (quirk Q5, ``kitti.lagged_xz_error``);
* ``plot_error``        — the error-over-time figure (``VO.m:183-188``);
* ``pose_and_landmarks``— ShowPoseAndLandmarks.m: landmarks as red dots and the camera path
  in blue, oblique 3-D projection.

Raster output is PNG (zlib + struct), plots are SVG.  ``snapshot`` writes the reference's
``img/<i>/`` layout (view.png, map.svg, error.svg, 3d_map.svg, view.txt).
"""
from __future__ import annotations

import os
import struct
import zlib
from pathlib import Path

import numpy as np

from . import kitti


# ------------------------------------------------------------------------------- raster
def write_png(path: str | os.PathLike, rgb: np.ndarray) -> None:
    """8-bit RGB (H, W, 3) or gray (H, W) array -> PNG file."""
    a = np.ascontiguousarray(rgb, np.uint8)
    if a.ndim == 2:
        a = np.repeat(a[:, :, None], 3, axis=2)
    h, w, _ = a.shape
    raw = b"".join(b"\x00" + a[y].tobytes() for y in range(h))      # filter type 0 per row

    def chunk(tag: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)
    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    Path(path).write_bytes(png)


def read_png_rgb(path: str | os.PathLike) -> np.ndarray:
    """Inverse of write_png for its own files (8-bit RGB, filter 0) -- used by the tests."""
    b = Path(path).read_bytes()
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    pos, w, h, idat = 8, 0, 0, b""
    while pos < len(b):
        n = struct.unpack(">I", b[pos:pos + 4])[0]
        tag, data = b[pos + 4:pos + 8], b[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            w, h = struct.unpack(">II", data[:8])
        elif tag == b"IDAT":
            idat += data
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 3 * w + 1)
    return raw[:, 1:].reshape(h, w, 3).copy()


def _line(img: np.ndarray, x0: float, y0: float, x1: float, y1: float, color) -> None:
    n = int(max(abs(x1 - x0), abs(y1 - y0))) + 1
    xs = np.rint(np.linspace(x0, x1, n)).astype(int)
    ys = np.rint(np.linspace(y0, y1, n)).astype(int)
    ok = (xs >= 0) & (xs < img.shape[1]) & (ys >= 0) & (ys < img.shape[0])
    img[ys[ok], xs[ok]] = color


def features_on_feed(img: np.ndarray, old_l: np.ndarray, cur_l: np.ndarray, det: np.ndarray) -> np.ndarray:
    """ShowFeaturesOnFeed.m on a u8 left frame.  Positions are MATLAB 1-based (x, y)."""
    out = np.repeat(np.asarray(img, np.uint8)[:, :, None], 3, axis=2).copy()
    green, red = (0, 128, 0), (255, 0, 0)
    for x, y in np.asarray(det, np.float64).reshape(-1, 2) - 1.0:          # 'x' markers, 5 px
        for d in (-2, 2):
            _line(out, x - 2, y - 2 * np.sign(d), x + 2, y + 2 * np.sign(d), green)
    for (xo, yo), (xc, yc) in zip(np.asarray(old_l, np.float64).reshape(-1, 2) - 1.0,
                                  np.asarray(cur_l, np.float64).reshape(-1, 2) - 1.0):
        _line(out, xo, yo, xc, yc, red)
    return out


# ------------------------------------------------------------------------------- vector
def _svg(series, title: str, xlabel: str, ylabel: str, equal: bool = False, size=(640, 480)) -> str:
    """series: list of (xs, ys, stroke, dash, kind) with kind 'line' or 'dots'."""
    W, H = size
    m = 50
    xs_all = np.concatenate([np.asarray(s[0], np.float64) for s in series if len(s[0])] or [np.zeros(1)])
    ys_all = np.concatenate([np.asarray(s[1], np.float64) for s in series if len(s[1])] or [np.zeros(1)])
    x0, x1 = float(np.nanmin(xs_all)), float(np.nanmax(xs_all))
    y0, y1 = float(np.nanmin(ys_all)), float(np.nanmax(ys_all))
    sx = (W - 2 * m) / max(x1 - x0, 1e-9)
    sy = (H - 2 * m) / max(y1 - y0, 1e-9)
    if equal:
        sx = sy = min(sx, sy)

    def px(x):
        return m + (np.asarray(x, np.float64) - x0) * sx

    def py(y):
        return H - m - (np.asarray(y, np.float64) - y0) * sy
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{W}" height="{H}" viewBox="0 0 {W} {H}">',
           f'<rect width="{W}" height="{H}" fill="white"/>',
           f'<text x="{W / 2}" y="20" text-anchor="middle" font-size="14">{title}</text>',
           f'<text x="{W / 2}" y="{H - 10}" text-anchor="middle" font-size="12">{xlabel}</text>',
           f'<text x="14" y="{H / 2}" font-size="12" transform="rotate(-90 14 {H / 2})" text-anchor="middle">{ylabel}</text>',
           f'<rect x="{m}" y="{m}" width="{W - 2 * m}" height="{H - 2 * m}" fill="none" stroke="#888"/>',
           f'<text x="{m}" y="{H - m + 14}" font-size="10">{x0:.3g}</text>',
           f'<text x="{W - m}" y="{H - m + 14}" font-size="10" text-anchor="end">{x1:.3g}</text>',
           f'<text x="{m - 4}" y="{H - m}" font-size="10" text-anchor="end">{y0:.3g}</text>',
           f'<text x="{m - 4}" y="{m + 8}" font-size="10" text-anchor="end">{y1:.3g}</text>']
    for xs, ys, stroke, dash, kind in series:
        X, Y = px(xs), py(ys)
        if kind == "dots":
            out += [f'<circle cx="{a:.1f}" cy="{b:.1f}" r="0.8" fill="{stroke}"/>' for a, b in zip(X, Y)]
        elif len(X):
            pts = " ".join(f"{a:.1f},{b:.1f}" for a, b in zip(X, Y))
            da = ' stroke-dasharray="6,4"' if dash else ""
            out.append(f'<polyline points="{pts}" fill="none" stroke="{stroke}" stroke-width="1.5"{da}/>')
    out.append("</svg>")
    return "\n".join(out)


def plot_on_map(poses: np.ndarray, gt: np.ndarray) -> tuple[str, np.ndarray]:
    """PlotOnMap.m: xz travel map of GT (black) and estimate (dashed); returns (svg, error)
    with the reference's one-frame-lagged xz error."""
    poses = np.asarray(poses, np.float64)
    gt = np.asarray(gt, np.float64)
    n = min(len(poses), len(gt))
    svg = _svg([(gt[:n, 0, 3], gt[:n, 2, 3], "black", False, "line"),
                (poses[:n, 0, 3], poses[:n, 2, 3], "#1f77b4", True, "line")],
               "Travel map", "x coordinate", "z coordinate", equal=True)
    return svg, kitti.lagged_xz_error(poses, gt)


def plot_error(times: np.ndarray, error: np.ndarray) -> str:
    t = np.asarray(times, np.float64)[: len(error)]
    return _svg([(t, np.asarray(error)[: len(t)], "#1f77b4", False, "line")],
                "Error in xz-plane over time", "Time[s]", "Error[m]")


def pose_and_landmarks(poses: np.ndarray, landmarks: np.ndarray, end_index: int | None = None) -> str:
    """ShowPoseAndLandmarks.m: landmarks (red dots) and camera path (blue), projected with a
    fixed oblique view (x right, z into the page, y down as in the camera frame)."""
    poses = np.asarray(poses, np.float64)[: end_index]
    lm = np.asarray(landmarks, np.float64).reshape(-1, 3)

    def proj(P):
        P = np.asarray(P, np.float64).reshape(-1, 3)
        return P[:, 0] + 0.5 * P[:, 2], -P[:, 1] + 0.35 * P[:, 2]
    lx, ly = proj(lm) if len(lm) else (np.zeros(0), np.zeros(0))
    cx, cy = proj(poses[:, :3, 3])
    return _svg([(lx, ly, "red", False, "dots"), (cx, cy, "blue", False, "line")],
                "Poses and landmarks", "x + z/2 [m]", "-y + 0.35 z [m]", equal=True)


def snapshot(out_dir: str | os.PathLike, i: int, left: np.ndarray, tracks: dict, poses: np.ndarray,
             gt: np.ndarray | None, times: np.ndarray | None, landmarks: np.ndarray) -> Path:
    """Write the reference's `img/<i>/` figures for frame i (VO.m:168-199)."""
    d = Path(out_dir) / "img" / str(i)
    d.mkdir(parents=True, exist_ok=True)
    write_png(d / "view.png", features_on_feed(left, tracks["old_l"], tracks["cur_l"], tracks["det"]))
    world = np.asarray(tracks.get("world", np.zeros((0, 3))))
    with open(d / "view.txt", "w") as fh:                        # the reference's per-point labels
        for (x, y), X in zip(np.asarray(tracks["cur_l"]), world):
            fh.write(f"{x:.2f} {y:.2f} {X[0]:.3f} {X[1]:.3f} {X[2]:.3f}\n")
    if gt is not None:
        svg, err = plot_on_map(poses, gt)
        (d / "map.svg").write_text(svg)
        if times is not None and len(err):
            (d / "error.svg").write_text(plot_error(times, err))          # frame_times(1:numel(error))
    (d / "3d_map.svg").write_text(pose_and_landmarks(poses, landmarks))
    return d
