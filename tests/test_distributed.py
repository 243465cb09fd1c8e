"""Multi-rank path on CPU (gloo): a sequence is block-sharded with a one-frame halo,
each rank runs its frames (through the CPU oracle, standing in for its GPU: these
ranks are libvo-free), the per-frame records are all-gathered, every rank chains the
relative poses and moves its OWN landmark rows to the world with its frames' chained
poses (CreateLandmarksFromFeatures.m:17), and the world rows are
gathered to rank 0 only (the shape of kitti.finish_shard).  World poses (on every rank)
AND the landmark map (rank 0) equal the single-process run bit for bit (MSAC keys are
global frame indices); the other ranks hold no map."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, result_q):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    import torch
    import torch.distributed as dist
    import vo_amd  # noqa: F401
    from r7020e_visual_odometry_amd import sharding
    import oracle
    torch.set_num_threads(1)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = np.load(path)
    L, R = z["L"], z["R"]
    n = len(L)
    s, e = sharding.shard_range(n, world, rank)
    h = sharding.halo_start(s)
    outs, (X, keep) = oracle.run_sequence(L[h:e], R[h:e], z["P1"], z["P2"], key0=h, camera_rows=True)
    outs = outs[s - h:]                                  # drop the halo frame
    steps = sharding.gather_steps(outs, n)
    poses = sharding.chain(steps["rel_pose"], status=steps["status"])
    counts = sharding.rank_row_counts(steps["n_landmarks"], n, world)
    assert counts[rank] == len(keep)
    own = sharding.world_landmarks(poses[s:e], steps["n_landmarks"][s:e], X, keep, oracle.landmarks_to_world)
    assert np.array_equal(own.astype(np.float32).astype(np.float64), own)     # single-rounded: float32 is exact
    lm = sharding.gather_rows_to_root(own.astype(np.float32), counts)
    if rank == 0:
        result_q.put((steps, poses, lm))
    else:
        assert lm is None
    dist.barrier()
    dist.destroy_process_group()


def _run(world, path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def _check(res, ref_outs, ref_lm):
    steps, poses, lm = res
    assert np.array_equal(steps["rel_pose"], ref_outs["rel_pose"])
    for k in ("status", "n_left", "n_right", "n_stereo", "n_tracked", "n_inliers", "n_landmarks"):
        assert np.array_equal(steps[k], ref_outs[k]), k
    assert np.array_equal(poses, ref_outs["pose"])
    assert lm.dtype == np.float32 and lm.shape == ref_lm.shape and np.array_equal(lm.astype(np.float64), ref_lm)


def test_two_rank_sharded_golden_sequence_equals_single_process(tmp_path):
    z = np.load(ROOT / "tests" / "golden" / "sequence.npz")
    ref = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    _check(_run(2, ROOT / "tests" / "golden" / "sequence.npz"), ref, z["landmarks"])


@pytest.fixture(scope="module")
def street_seq(tmp_path_factory, oracle):
    """6 frames along KITTI-00's ground truth (frames 1500-1505), rendered at half size."""
    import torch
    from r7020e_visual_odometry_amd import street, synthetic as syn
    torch.set_num_threads(4)
    gt = street.kitti00_gt()
    P0, P1 = syn.calib(0.5)
    w = street.kitti00_world()
    L, R = street.render_frames(w, gt, range(1500, 1506), P0, P1, rows=188, cols=620, chunk=6)
    path = tmp_path_factory.mktemp("street") / "seq.npz"
    np.savez(path, L=L.numpy(), R=R.numpy(), P1=P0, P2=P1)
    outs, lm = oracle.run_sequence(L.numpy(), R.numpy(), P0, P1)
    return path, outs, lm


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_street_sequence_poses_and_landmarks_equal_single_process(street_seq, world):
    """world 8 (the configs[3] node) over 6 frames also leaves ranks 6 and 7 without frames."""
    path, outs, lm = street_seq
    assert (outs["status"][1:] == 0).all() and len(lm) > 100
    _check(_run(world, path), outs, lm)


def _agree_worker(rank, world, port, result_q):
    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist
    import vo_amd  # noqa: F401
    from r7020e_visual_odometry_amd import sharding
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # only the last rank fails its check; every rank must learn of it before a later collective
    res = (sharding.any_rank(False), sharding.any_rank(rank == world - 1))
    result_q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_ranks_agree_on_an_error_before_the_gather():
    """kitti.finish_shard raises on every rank when one rank's landmark row count disagrees
    with the records (sharding.any_rank), instead of leaving the others inside dist.gather."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(got[r] == (False, True) for r in range(world)), got
