"""The nccl (RCCL) branch of the sharding collectives, on the CPU with a spy in place of
torch.distributed: with device=<dev> every tensor handed to all_gather / gather is built on that
device (RCCL only takes device tensors), records come back in frame order from a 3-rank world,
world landmark rows reach rank 0 only (in rank = frame order, padding dropped), and the results
are read back through .cpu().  The spy's device is the CPU (no GPU here); what is checked is that
the helpers place every collective buffer on the device they are given, never on a default one
(bench.py passes cuda:LOCAL_RANK under nccl)."""
import types

import numpy as np
import pytest
import torch

from r7020e_visual_odometry_amd import sharding


class SpyDist(types.SimpleNamespace):
    """world-size-W all_gather: rank r's contribution is produced by make(r, template)."""

    def __init__(self, world, rank, make):
        super().__init__()
        self.world, self.rank, self.make, self.calls = world, rank, make, []

    def get_world_size(self, group=None):
        return self.world

    def get_rank(self, group=None):
        return self.rank

    def gather(self, t, gather_list=None, dst=0, group=None):
        self.calls.append((t.device, t.dtype, tuple(t.shape)))
        if self.rank != dst:
            assert gather_list is None
            return
        assert len(gather_list) == self.world
        for r in range(self.world):
            assert gather_list[r].device == t.device and gather_list[r].shape == t.shape
            gather_list[r].copy_(t if r == self.rank else self.make(r, t))

    def all_gather(self, parts, t, group=None):
        self.calls.append((t.device, t.dtype, tuple(t.shape)))
        assert len(parts) == self.world
        for r in range(self.world):
            assert parts[r].device == t.device and parts[r].shape == t.shape
            parts[r].copy_(t if r == self.rank else self.make(r, t))


@pytest.fixture
def spy(monkeypatch):
    def install(world, rank, make):
        d = SpyDist(world, rank, make)
        monkeypatch.setattr(torch.distributed, "get_world_size", d.get_world_size)
        monkeypatch.setattr(torch.distributed, "all_gather", d.all_gather)
        monkeypatch.setattr(torch.distributed, "get_rank", d.get_rank)
        monkeypatch.setattr(torch.distributed, "gather", d.gather)
        return d
    return install


@pytest.mark.parametrize("device", [torch.device("cpu"), "cpu"])
def test_gather_frames_device_tensors(spy, device):
    n, W, world = 10, 23, 3
    full = np.arange(n * W, dtype=np.float64).reshape(n, W) * 0.5

    def make(r, t):
        s, e = sharding.shard_range(n, world, r)
        out = torch.zeros_like(t)
        out[: e - s] = torch.from_numpy(full[s:e])
        return out
    d = spy(world, 1, make)
    s, e = sharding.shard_range(n, world, 1)
    got = sharding.gather_frames(full[s:e], n, device=device)
    assert np.array_equal(got, full)
    assert d.calls and all(c[0] == torch.device(device) and c[1] == torch.float64 for c in d.calls)


@pytest.mark.parametrize("rank", [0, 2])
@pytest.mark.parametrize("as_tensor", [False, True])
@pytest.mark.parametrize("with_out", [False, True])
def test_gather_rows_to_root_device_tensors(spy, rank, as_tensor, with_out):
    world = 3
    rows = {r: np.random.default_rng(r).normal(size=(5 + 3 * r, 3)).astype(np.float32) for r in range(world)}
    counts = [len(rows[r]) for r in range(world)]
    m = max(counts)

    def make(r, t):
        out = torch.full_like(t, float("nan"))                      # padding must be dropped
        out[: counts[r]] = torch.from_numpy(rows[r])
        return out
    dev = torch.device("cpu")
    d = spy(world, rank, make)
    if as_tensor:                                                   # a device buffer of max(counts) rows
        loc = torch.full((m, 3), float("nan"))
        loc[: counts[rank]] = torch.from_numpy(rows[rank])
    else:
        loc = rows[rank]
    out = torch.full((sum(counts) + 3, 3), -7.0) if with_out else None        # a host buffer allocated ahead
    got = sharding.gather_rows_to_root(loc, counts, device=dev, out=out)
    if rank == 0:
        assert got.dtype == np.float32 and np.array_equal(got, np.concatenate([rows[r] for r in range(world)]))
        if with_out:                                                # a view of the caller's buffer
            assert np.shares_memory(got, out.numpy()) and (out[sum(counts):] == -7.0).all()
    else:
        assert got is None
    assert d.calls == [(dev, torch.float32, (m, 3))]


def test_rank_row_counts():
    n = np.array([0, 3, 4, 0, 7, 1, 2])
    assert sharding.rank_row_counts(n, 7, 3) == [7, 7, 3]       # blocks [0,3) [3,5) [5,7)
    assert sharding.rank_row_counts(n, 7, 1) == [17]


def test_gather_steps_frame_order(spy):
    from r7020e_visual_odometry_amd import vo
    n, world = 7, 2
    recs = np.zeros(n, vo.STEP_DTYPE)
    recs["status"] = [0, 0, -4, 0, 0, 0, -3]
    recs["n_tracked"] = np.arange(n) * 10
    recs["rel_pose"] = np.eye(4) + np.arange(n)[:, None, None] * 0.01

    def make(r, t):
        s, e = sharding.shard_range(n, world, r)
        rec = np.concatenate([recs["rel_pose"][s:e].reshape(-1, 16)] +
                             [recs[k][s:e].astype(np.float64).reshape(-1, 1) for k in sharding.STEP_FIELDS], 1)
        out = torch.zeros_like(t)
        out[: e - s] = torch.from_numpy(rec)
        return out
    spy(world, 0, make)
    s, e = sharding.shard_range(n, world, 0)
    steps = sharding.gather_steps(recs[s:e], n, device=torch.device("cpu"))
    assert np.array_equal(steps["rel_pose"], recs["rel_pose"])
    assert np.array_equal(steps["status"], recs["status"]) and np.array_equal(steps["n_tracked"], recs["n_tracked"])
