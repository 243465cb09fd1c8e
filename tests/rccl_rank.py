"""Child process of tests/test_gpu_rccl.py (not collected by pytest): one rank of a real RCCL
process group on this box's GPU.

The group is created FIRST -- `dist.init_process_group("nccl", device_id=cuda:0)` from the env
rendezvous (MASTER_ADDR/MASTER_PORT/RANK/WORLD_SIZE set by the parent) before any other GPU
work -- exactly as bench.py's ranks do.  Then a KITTI-00 stretch rendered along the reference's
ground truth (street.py) runs through the sharded path with the collectives on device tensors
(kitti.finish_shard with collective_device=cuda: the records all-gather and the gather of the
device-transformed world rows to rank 0 run through RCCL), and through a plain single-process libvo
run; rank 0 prints one JSON line comparing the two (VO.m:130-134 chain,
CreateLandmarksFromFeatures.m:17 map)."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    rank, world = dist.get_rank(), dist.get_world_size()
    import vo_amd  # noqa: F401
    from r7020e_visual_odometry_amd import kitti, street, vo
    frames = range(int(os.environ.get("VO_RCCL_FIRST", "2000")), int(os.environ.get("VO_RCCL_LAST", "2009")))
    n = len(frames)
    gt = street.kitti00_gt()
    P0, P1 = street.kitti00_calib()
    w = street.kitti00_world(device=f"cuda:{local}")
    L, R = street.render_frames(w, gt, frames, P0, P1, chunk=n)
    del w
    torch.cuda.synchronize()
    B = 3
    # the sharded path, collectives on device tensors (RCCL)
    sctx = vo.Context(street.KITTI_ROWS, street.KITTI_COLS, B, device=local, calib=vo.calib_from(P0, P1))
    outs, _, _ = kitti.run_shard((L, R, P0, P1), rank, world, B, local, n, ctx=sctx, rows_to_host=False)
    poses, steps, lm = kitti.finish_shard(sctx, outs, n, rank, world, local, collective_device=dev)
    sctx.close()
    t = torch.tensor([float(rank) + 0.25], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)                    # bench.py's max_over_ranks
    maxv = float(t.item())
    # the plain single-process run
    ctx = vo.Context(street.KITTI_ROWS, street.KITTI_COLS, B, device=local, calib=vo.calib_from(P0, P1))
    ref = np.concatenate(kitti._pipelined(ctx, kitti.device_batches(L, R, B), None))
    lm1 = ctx.get_landmarks()
    ctx.close()
    res = {"backend": dist.get_backend(), "world": world, "frames": n,
           "poses_equal": bool(np.array_equal(poses, ref["pose"])),
           "rel_equal": bool(np.array_equal(steps["rel_pose"], ref["rel_pose"])),
           "status_equal": bool(np.array_equal(steps["status"], ref["status"].astype(np.int64))),
           "n_landmarks_equal": bool(np.array_equal(steps["n_landmarks"], ref["n_landmarks"].astype(np.int64))),
           "landmarks_equal": bool(lm is not None and lm.dtype == np.float32 and lm.shape == lm1.shape
                                   and np.array_equal(lm.astype(np.float64), lm1)),
           "landmark_rows": int(len(lm1)), "frames_with_pose": int((ref["status"][1:] == 0).sum()),
           "max_over_ranks": maxv}
    dist.barrier()
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
