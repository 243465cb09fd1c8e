"""Digitise the reference's published KITTI-00 accuracy curve (reference 4500/error.png: the
lagged x-z error of PlotOnMap.m:8-20 for VO.m's MATLAB run on the real KITTI-00 images) into
data/kitti/ref_error_digitized.csv (time [s], error [m]) -- a data fixture, the only
numeric output of the reference's own run that the repository holds.

Plot geometry (read from the PNG): axes box x 64..741 px = 0..500 s, y 562..28 px = 0..45 m;
the curve is MATLAB's default blue (0, 114, 189).  One sample per pixel column (mean of the
curve's pixels in that column); resolution ~0.74 s and ~0.08 m.
    python tests/golden/digitize_ref_error.py /root/reference/4500/error.png
"""
import sys
from pathlib import Path

import numpy as np
from PIL import Image

X0, X1, T1 = 64, 741, 500.0
Y0, Y1, E1 = 562, 28, 45.0


def digitize(path):
    im = np.asarray(Image.open(path).convert("RGB")).astype(int)
    r, g, b = im[..., 0], im[..., 1], im[..., 2]
    blue = (b > 150) & (r < 80) & (g > 60) & (g < 160)
    out = []
    for x in range(X0, X1 + 1):
        ys = np.nonzero(blue[:, x])[0]
        if len(ys):
            out.append(((x - X0) / (X1 - X0) * T1, (Y0 - ys.mean()) / (Y0 - Y1) * E1))
    return np.array(out)


if __name__ == "__main__":
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/4500/error.png"
    d = digitize(src)
    dst = Path(__file__).resolve().parent.parent.parent / "data" / "kitti" / "ref_error_digitized.csv"
    np.savetxt(dst, d, fmt="%.3f", delimiter=",", header="time_s,lagged_xz_error_m (digitised from reference 4500/error.png)")
    print(f"{len(d)} samples, t {d[0, 0]:.1f}..{d[-1, 0]:.1f} s, error mean {d[:, 1].mean():.2f} max {d[:, 1].max():.2f} final {d[-1, 1]:.2f} m")
