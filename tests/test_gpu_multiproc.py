"""libvo inside a real torch.distributed process group (the multi-GPU path had only
ever run the oracle per rank).  Two spawned ranks on this box's one GPU (gloo for the
collectives; the 8-GPU runs use nccl = RCCL) run kitti.run_distributed over a KITTI-00 stretch
rendered along the reference's ground truth; world poses, per-frame records and the landmark
map (transformed on each rank's device, gathered to rank 0) equal a single-process libvo run bit
for bit."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, path, q):
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist
    import vo_amd  # noqa: F401
    from r7020e_visual_odometry_amd import kitti
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = np.load(path)
    L, R = torch.from_numpy(z["L"]).cuda(), torch.from_numpy(z["R"]).cuda()
    torch.cuda.synchronize()
    poses, steps, lm = kitti.run_distributed((L, R, z["P0"], z["P1"]), batch=2, device=0)
    if rank == 0:
        q.put((poses, steps["rel_pose"], steps["n_landmarks"], lm))
    else:
        assert lm is None                                   # the map is gathered to rank 0 only
    dist.barrier()
    dist.destroy_process_group()


def test_two_process_group_libvo_equals_single_process(vo, tmp_path):
    import torch
    from r7020e_visual_odometry_amd import kitti, street
    gt = street.kitti00_gt()
    P0, P1 = street.kitti00_calib()
    w = street.kitti00_world(device="cuda:0")
    L, R = street.render_frames(w, gt, range(3000, 3007), P0, P1, chunk=7)
    torch.cuda.synchronize()
    path = tmp_path / "seq.npz"
    np.savez(path, L=L.cpu().numpy(), R=R.cpu().numpy(), P0=P0, P1=P1)
    ctx = vo.Context(street.KITTI_ROWS, street.KITTI_COLS, 2, calib=vo.calib_from(P0, P1))
    outs = np.concatenate(kitti._pipelined(ctx, kitti.device_batches(L, R, 2), None))
    lm1 = ctx.get_landmarks()
    ctx.close()
    spawn = mp.get_context("spawn")
    q = spawn.Queue()
    port = _free_port()
    procs = [spawn.Process(target=_rank, args=(r, 2, port, str(path), q)) for r in range(2)]
    for p in procs:
        p.start()
    poses, rel, nlm, lm = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(poses, outs["pose"]) and np.array_equal(rel, outs["rel_pose"])
    assert np.array_equal(nlm, outs["n_landmarks"])
    assert lm.dtype == np.float32 and lm.shape == lm1.shape and np.array_equal(lm.astype(np.float64), lm1)
