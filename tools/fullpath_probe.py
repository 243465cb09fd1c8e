#!/usr/bin/env python3
"""Per-kernel breakdown of the full per-frame path (BASELINE configs[2] on the synthetic
sequence bench.py uses): wall time per batch and libvo's HIP-event kernel times.
usage: python tools/fullpath_probe.py [frames] [batch] [pipe]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import vo_amd  # noqa: E402,F401
from r7020e_visual_odometry_amd import vo, synthetic as syn  # noqa: E402

nf = int(sys.argv[1]) if len(sys.argv) > 1 else 64
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
half = (nf + 1) // 2
SL, SR, _ = syn.sequence(half, 375, 1242, seed=syn.SEED_BASE, step_m=0.25, yaw_deg=0.1)
SL = np.ascontiguousarray(np.concatenate([SL, SL[::-1]])[:nf])
SR = np.ascontiguousarray(np.concatenate([SR, SR[::-1]])[:nf])
dl, dr = torch.from_numpy(SL).cuda(), torch.from_numpy(SR).cuda()
P1, P2 = syn.calib()
ctx = vo.Context(375, 1242, B, calib=vo.calib_from(P1, P2))
fs = SL[0].size


PIPE = len(sys.argv) > 3 and sys.argv[3] == "pipe"


def run():
    ctx.reset()
    if not PIPE:
        return np.concatenate([ctx.step_batch_dev(dl.data_ptr() + b * fs, dr.data_ptr() + b * fs, B) for b in range(0, nf, B)])
    outs = []
    for b in range(0, nf, B):
        ctx.step_submit_dev(dl.data_ptr() + b * fs, dr.data_ptr() + b * fs, B)
        if ctx.steps_pending() == 2:
            outs.append(ctx.step_collect())
    while ctx.steps_pending():
        outs.append(ctx.step_collect())
    return np.concatenate(outs)


run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    out = run()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 3
print(f"frames {nf} batch {B}: {dt * 1e3:.2f} ms per sequence, {nf / dt:.1f} stereo frames/s, "
      f"poses ok {int((out['status'][1:] == 0).sum())}/{nf - 1}")
ctx.set_profiling(True)
run()
torch.cuda.synchronize()
kt = ctx.kernel_times()
ctx.set_profiling(False)
tot = sum(v[0] for v in kt.values())
print(f"kernel time sum {tot:.2f} ms")
for n, (ms, calls) in sorted(kt.items(), key=lambda kv: -kv[1][0]):
    print(f"  {n:24s} {ms:8.3f} ms  {calls:5d} calls")
