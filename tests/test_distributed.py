"""Multi-rank path on CPU (gloo, world_size 2): the sequence is block-sharded
with a one-frame halo, each rank runs its frames (here through the CPU oracle,
standing in for its GPU), relative poses are all-gathered and chained, and the
result equals the single-process run bit for bit (MSAC keys are global frame
indices)."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, result_q):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    import torch.distributed as dist
    import vo_amd  # noqa: F401
    from r7020e_visual_odometry_amd import sharding
    import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = np.load(ROOT / "tests" / "golden" / "sequence.npz")
    L, R = z["L"], z["R"]
    n = len(L)
    s, e = sharding.shard_range(n, world, rank)
    h = sharding.halo_start(s)
    outs, _ = oracle.run_sequence(L[h:e], R[h:e], z["P1"], z["P2"], key0=h)
    rel_local = outs["rel_pose"][s - h:]          # drop the halo frame
    rel = sharding.gather_rel_poses(rel_local, n)
    poses = sharding.chain(rel)
    if rank == 0:
        result_q.put((rel, poses))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharded_sequence_equals_single_process():
    z = np.load(ROOT / "tests" / "golden" / "sequence.npz")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    rel, poses = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(rel, z["out_rel_pose"])
    assert np.array_equal(poses, z["out_pose"])
