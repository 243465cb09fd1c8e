"""Small driver for rocprofv3 passes: N batches of the bench workload, issued back to back
(asynchronous pipeline, like bench.py's timed loop), then one synchronising call."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import torch
import vo_amd  # noqa
from r7020e_visual_odometry_amd import vo, synthetic as syn

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
N = int(sys.argv[2]) if len(sys.argv) > 2 else 3
L, R = syn.independent_pairs(B, px_per_cell=syn.BENCH_PX_PER_CELL)
dl, dr = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
torch.cuda.synchronize()
ctx = vo.Context(375, 1242, B)
for _ in range(N):
    ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B, stats=False)
ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B, stats=True)
torch.cuda.synchronize()
print("done")
