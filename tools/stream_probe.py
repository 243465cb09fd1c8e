"""Probe: frames/s of one libvo context vs batch size and vo_set_concurrency."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import torch
import vo_amd  # noqa
from r7020e_visual_odometry_amd import vo, synthetic as syn

for B in (16, 32):
    L, R = syn.independent_pairs(B)
    dl, dr = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    ctx = vo.Context(375, 1242, B)
    for ns in (1, 2, 3, 4):
        ctx.set_concurrency(ns)
        for _ in range(2):
            ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B, stats=False)
        torch.cuda.synchronize()
        steps = 10
        t0 = time.perf_counter()
        for _ in range(steps):
            ctx.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B, stats=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"B={B} streams={ns}: {B * steps / dt:.0f} frames/s", flush=True)
    ctx.close()
