"""Probe: throughput of N libvo contexts (own HIP streams) sharing one GPU, each
with B frames per call, calls issued back to back without host sync."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import torch
import vo_amd  # noqa
from r7020e_visual_odometry_amd import vo, synthetic as syn

for nctx, B in [(1, 16), (2, 8), (2, 16), (4, 8), (1, 32), (1, 64)]:
    L, R = syn.independent_pairs(B)
    dl, dr = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    ctxs = [vo.Context(375, 1242, B) for _ in range(nctx)]
    for c in ctxs:
        c.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B, stats=False)
    torch.cuda.synchronize()
    steps = 10
    t0 = time.perf_counter()
    for _ in range(steps):
        for c in ctxs:
            c.sift_match_batch_dev(dl.data_ptr(), dr.data_ptr(), B, stats=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"ctx={nctx} B={B}: {nctx * B * steps / dt:.0f} frames/s", flush=True)
    for c in ctxs:
        c.close()
    del dl, dr
    torch.cuda.empty_cache()
