"""Multi-GPU frame sharding for the sequential VO path.

The per-frame work of VO.m depends only on frames i-1 and i (SIFT of both,
find_remaining_points, P3P-MSAC keyed by the global frame index); the only
sequential part is the 4x4 world-pose chain pose_i = pose_{i-1} * rel_i
(VO.m:130).  So a sequence is block-partitioned over ranks with a one-frame
halo (each rank also processes the frame before its block, whose SIFT/stereo
set seeds the tracking of its first frame), every rank computes its relative
poses independently, and one all-gather of 16 doubles per frame (RCCL over
xGMI with the nccl backend; gloo in the CPU tests) hands them to the chain.

chain() reproduces libvo's host chain (vo_api.hip mat4_mul) operation for
operation, so a sharded run's world poses equal the single-process run's bit
for bit.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_frames: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block [start, end) of frames owned by `rank`."""
    base, rem = divmod(n_frames, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def halo_start(start: int) -> int:
    """First frame a rank must process: one frame before its block (halo)."""
    return start - 1 if start > 0 else 0


def mat4_mul(A, B):
    """Row-major 4x4 double product in libvo's exact operation order."""
    A = [float(v) for v in np.asarray(A, np.float64).reshape(16)]
    B = [float(v) for v in np.asarray(B, np.float64).reshape(16)]
    T = [0.0] * 16
    for i in range(4):
        for j in range(4):
            T[4 * i + j] = A[4 * i] * B[j] + A[4 * i + 1] * B[4 + j] + A[4 * i + 2] * B[8 + j] + A[4 * i + 3] * B[12 + j]
    return np.array(T).reshape(4, 4)


def chain(rel_poses, pose0=None) -> np.ndarray:
    """World poses from relative poses (VO.m:130: pose = pose * rel_pose)."""
    pose = np.eye(4) if pose0 is None else np.asarray(pose0, np.float64)
    out = np.empty((len(rel_poses), 4, 4))
    for i, r in enumerate(rel_poses):
        pose = mat4_mul(pose, r)
        out[i] = pose
    return out


def gather_rel_poses(rel_local: np.ndarray, n_frames: int, group=None, device=None) -> np.ndarray:
    """All-gather every rank's block of relative poses [n_local, 4, 4] into the
    full [n_frames, 4, 4] array (frame order).  One collective per call; works
    with the gloo (CPU tensors) and nccl/RCCL (device tensors) backends."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    maxn = max(shard_range(n_frames, world, r)[1] - shard_range(n_frames, world, r)[0] for r in range(world))
    buf = torch.zeros((maxn, 16), dtype=torch.float64, device=device)
    if len(rel_local):
        buf[: len(rel_local)] = torch.from_numpy(np.asarray(rel_local, np.float64).reshape(-1, 16)).to(buf.device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = np.empty((n_frames, 4, 4))
    for r in range(world):
        s, e = shard_range(n_frames, world, r)
        out[s:e] = parts[r][: e - s].cpu().numpy().reshape(-1, 4, 4)
    return out
