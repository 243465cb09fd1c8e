"""Diagnostic: camera-frame landmark rows of the pipelined path (batch B, depth D) vs 64-frame
synchronous calls over the same 768 chained synthetic frames; prints where rows differ."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np
import torch
import vo_amd  # noqa
from r7020e_visual_odometry_amd import vo, kitti, synthetic as syn

n = 768
SL, SR, _ = syn.sequence(32, 375, 1242, seed=syn.SEED_BASE + 0x778, step_m=0.25, yaw_deg=0.1)
loop = np.arange(n) % 64
loop = np.where(loop < 32, loop, 63 - loop)
L, R = np.ascontiguousarray(SL[loop]), np.ascontiguousarray(SR[loop])
dl, dr = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
torch.cuda.synchronize()
fs = L[0].size
calib = vo.calib_from(syn.KITTI00_P0, syn.KITTI00_P1)
half = vo.Context(375, 1242, 64, calib=calib)
half.set_landmark_frame(True)
b = np.concatenate([half.step_batch_dev(dl.data_ptr() + b0 * fs, dr.data_ptr() + b0 * fs, 64) for b0 in range(0, n, 64)])
Xb, kb = half.get_landmark_rows()
half.close()
off = np.r_[0, np.cumsum(b["n_landmarks"])]
for B, D in [(256, 1), (256, 2), (256, 3), (64, 3), (128, 3)]:
    ctx = vo.Context(375, 1242, B, calib=calib)
    ctx.set_landmark_frame(True)
    a = np.concatenate(kitti._pipelined(ctx, kitti.device_batches(dl, dr, B), torch.device("cuda", 0), depth=D))
    Xa, ka = ctx.get_landmark_rows()
    ctx.close()
    rec = a.tobytes() == b.tobytes()
    bad = np.nonzero(np.any(Xa.reshape(-1, 3) != Xb.reshape(-1, 3), axis=1) | (ka != kb))[0] if len(Xa) == len(Xb) else None
    if bad is None:
        print(B, D, "records", rec, "row counts differ", len(Xa), len(Xb))
        continue
    frames = np.unique(np.searchsorted(off, bad, side="right") - 1)
    print(B, D, "records", rec, "rows", len(Xa), "bad rows", len(bad), "frames", frames[:20], len(frames),
          "zero-in-a", int(np.sum(np.all(Xa.reshape(-1, 3)[bad] == 0, axis=1))) if len(bad) else 0, flush=True)
