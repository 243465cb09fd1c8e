"""Small driver for rocprofv3 passes: N batches of the bench workload, issued back to back
(asynchronous pipeline, like bench.py's timed loop), then one synchronising call.
usage: prof_run.py [B=16] [N=3] [street]  -- `street`: the first B KITTI-00 frames rendered along
the reference's ground truth (376x1241) instead of the bench's synthetic pairs (content A/B)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import torch
import vo_amd  # noqa
from r7020e_visual_odometry_amd import vo, synthetic as syn

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
N = int(sys.argv[2]) if len(sys.argv) > 2 else 3
if len(sys.argv) > 3 and sys.argv[3] == "street":
    from r7020e_visual_odometry_amd import street
    gt = street.kitti00_gt()
    P0, P1 = street.kitti00_calib()
    dl, dr = street.render_frames(street.kitti00_world(device="cuda:0", poses=gt), gt, range(B), P0, P1, chunk=B)
    dl, dr = dl.contiguous(), dr.contiguous()
    rows, cols = street.KITTI_ROWS, street.KITTI_COLS
else:
    L, R = syn.independent_pairs(B, px_per_cell=syn.BENCH_PX_PER_CELL, threads=16)
    dl, dr = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    rows, cols = 375, 1242
torch.cuda.synchronize()
ctx = vo.Context(rows, cols, B)
for _ in range(N):
    ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B, stats=False)
ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B, stats=True)
torch.cuda.synchronize()
print("done")
