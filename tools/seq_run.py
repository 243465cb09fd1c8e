"""Driver for rocprofv3 passes over the full per-frame path (BASELINE configs[2]): N KITTI-00
street frames rendered into HBM, then the pipelined loop body (vo_step_submit_dev /
vo_step_collect, 2048 MSAC hypotheses) in batches of B with D batches in flight, twice (the
first pass warms up).  usage: seq_run.py [N=1024] [B=256] [D=3]"""
import sys
import time
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import torch
import vo_amd  # noqa
from r7020e_visual_odometry_amd import vo, street, kitti

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
D = int(sys.argv[3]) if len(sys.argv) > 3 else 3
gt = street.kitti00_gt()
P0, P1 = street.kitti00_calib()
dev = torch.device("cuda", 0)
wld = street.kitti00_world(device="cuda:0", poses=gt)
dL = torch.empty((N, street.KITTI_ROWS, street.KITTI_COLS), dtype=torch.uint8, device=dev)
dR = torch.empty_like(dL)
street.render_frames(wld, gt, range(N), P0, P1, out=(dL, dR))
del wld
torch.cuda.synchronize()
rp = vo.default_ransac_params()
rp.max_num_trials = 2048
ctx = vo.Context(street.KITTI_ROWS, street.KITTI_COLS, B, calib=vo.calib_from(P0, P1), ransac=rp)
for rep in range(2):
    ctx.reset()
    ctx.set_landmark_frame(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kitti._pipelined(ctx, kitti.device_batches(dL, dR, B, 0, N), dev, depth=D)
    torch.cuda.synchronize()
    print(f"pass {rep}: {N / (time.perf_counter() - t0):.1f} frames/s", flush=True)
print("done")
