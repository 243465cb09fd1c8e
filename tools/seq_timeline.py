#!/usr/bin/env python3
"""Timeline of the pipelined full per-frame path (BASELINE configs[2]) for a kernel trace:
N KITTI-00 street frames rendered into HBM, one warm-up pass, then a marked pass
(torch.cuda._sleep spin kernels before and after) with the host time of every submit and
collect call.  Run under `rocprofv3 --kernel-trace`, analyse with tools/timeline.py.
usage: python tools/seq_timeline.py [frames=640] [batch=64]"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import vo_amd  # noqa: E402,F401
from r7020e_visual_odometry_amd import vo, street, kitti  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 640
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
dev = torch.device("cuda", 0)
gt = street.kitti00_gt()
P0, P1 = street.kitti00_calib()
wld = street.kitti00_world(device="cuda:0", poses=gt)
dL = torch.empty((N, street.KITTI_ROWS, street.KITTI_COLS), dtype=torch.uint8, device=dev)
dR = torch.empty_like(dL)
street.render_frames(wld, gt, range(N), P0, P1, out=(dL, dR))
del wld
torch.cuda.synchronize()
rp = vo.default_ransac_params()
rp.max_num_trials = 2048
ctx = vo.Context(street.KITTI_ROWS, street.KITTI_COLS, B, calib=vo.calib_from(P0, P1), ransac=rp)
host = {"submit": [], "collect": []}
sub0, col0 = ctx.step_submit_dev, ctx.step_collect


def sub(*a):
    t = time.perf_counter()
    sub0(*a)
    host["submit"].append(time.perf_counter() - t)


def col():
    t = time.perf_counter()
    r = col0()
    host["collect"].append(time.perf_counter() - t)
    return r


def run():
    ctx.reset()
    ctx.set_landmark_frame(True)
    return kitti._pipelined(ctx, kitti.device_batches(dL, dR, B, 0, N), dev)


run()
torch.cuda.synchronize()
ctx.step_submit_dev, ctx.step_collect = sub, col
torch.cuda._sleep(2_000_000)
torch.cuda.synchronize()
t0 = time.perf_counter()
outs = np.concatenate(run())
torch.cuda.synchronize()
wall = time.perf_counter() - t0
torch.cuda._sleep(2_000_000)
torch.cuda.synchronize()
print(json.dumps({"frames": N, "batch": B, "wall_ms": wall * 1e3, "fps": N / wall,
                  "host_submit_ms": [round(x * 1e3, 3) for x in host["submit"]],
                  "host_collect_ms": [round(x * 1e3, 3) for x in host["collect"]],
                  "mean_tracked": float(outs["n_tracked"][1:].mean())}))
