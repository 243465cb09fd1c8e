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

The landmark map: CreateLandmarksFromFeatures.m:17 moves a
frame's new points into the world with that frame's pose, which a rank that
starts mid-sequence only knows after the chain.  Ranks therefore keep their rows
in the camera frame (libvo vo_set_landmark_frame; the rows stay in device memory).
Only the per-frame records are all-gathered (23 doubles per frame); every rank
chains the poses itself, moves its OWN rows to the world with its frames' chained
poses (on the device: libvo vo_landmarks_world_dev; `world_landmarks` is the
host form), and the world rows go to rank 0 alone (`gather_rows_to_root`, one
dist.gather: RCCL from device buffers).  The per-rank tail is thus proportional to
the rank's own rows, and the result equals a single process's rows bit for bit.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_frames: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block [start, end) of frames owned by `rank`."""
    base, rem = divmod(n_frames, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def block_imbalance(cost, world: int) -> float:
    """max / mean over ranks of the per-block cost of `shard_range`'s partition (each rank > 0
    also recomputes its halo frame), for a per-frame cost proxy such as the keypoint count."""
    cost = np.asarray(cost, np.float64)
    n = len(cost)
    tot = []
    for r in range(world):
        s, e = shard_range(n, world, r)
        tot.append(cost[halo_start(s):e].sum() if e > s else 0.0)
    tot = np.asarray(tot)
    return float(tot.max() / tot.mean()) if tot.mean() > 0 else 1.0


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


def chain(rel_poses, pose0=None, status=None) -> np.ndarray:
    """World poses from relative poses (VO.m:130: pose = pose * rel_pose).  Frames whose
    status is not VO_OK hold the pose (libvo's collect skips their product)."""
    pose = np.eye(4) if pose0 is None else np.asarray(pose0, np.float64)
    out = np.empty((len(rel_poses), 4, 4))
    for i, r in enumerate(rel_poses):
        if status is None or status[i] == 0:
            pose = mat4_mul(pose, r)
        out[i] = pose
    return out


def gather_frames(local: np.ndarray, n_frames: int, group=None, device=None) -> np.ndarray:
    """All-gather every rank's block of per-frame float64 records [n_local, W] into the full
    [n_frames, W] array (frame order).  One collective; gloo (CPU tensors) or nccl/RCCL
    (device tensors)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    local = np.asarray(local, np.float64)
    if local.ndim != 2:                          # (a rank may own no frames: n < world)
        local = local.reshape(len(local), -1)
    W = local.shape[1]
    maxn = max(shard_range(n_frames, world, r)[1] - shard_range(n_frames, world, r)[0] for r in range(world))
    buf = torch.zeros((maxn, W), dtype=torch.float64, device=device)
    if len(local):
        buf[: len(local)] = torch.from_numpy(local).to(buf.device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = np.empty((n_frames, W))
    for r in range(world):
        s, e = shard_range(n_frames, world, r)
        out[s:e] = parts[r][: e - s].cpu().numpy()
    return out


def gather_rel_poses(rel_local: np.ndarray, n_frames: int, group=None, device=None) -> np.ndarray:
    """All-gather every rank's block of relative poses [n_local, 4, 4] into the
    full [n_frames, 4, 4] array (frame order)."""
    return gather_frames(np.asarray(rel_local).reshape(-1, 16), n_frames, group, device).reshape(-1, 4, 4)


STEP_FIELDS = ("status", "n_left", "n_right", "n_stereo", "n_tracked", "n_inliers", "n_landmarks")


def gather_steps(outs_local, n_frames: int, group=None, device=None) -> dict:
    """All-gather the per-frame step records of every rank's block (libvo STEP_DTYPE rows,
    halo frame already dropped) -> {"rel_pose": [n, 4, 4], "status": [n], ...} in frame order."""
    rec = np.concatenate([np.asarray(outs_local["rel_pose"], np.float64).reshape(-1, 16)]
                         + [np.asarray(outs_local[k], np.float64).reshape(-1, 1) for k in STEP_FIELDS], 1)
    full = gather_frames(rec, n_frames, group, device)
    out = {"rel_pose": full[:, :16].reshape(-1, 4, 4).copy()}
    for i, k in enumerate(STEP_FIELDS):
        out[k] = full[:, 16 + i].astype(np.int64)
    return out


def steps_of(outs) -> dict:
    """Per-frame records (STEP_DTYPE rows, frame order) in the form gather_steps returns."""
    out = {"rel_pose": np.asarray(outs["rel_pose"], np.float64).reshape(-1, 4, 4).copy()}
    for k in STEP_FIELDS:
        out[k] = np.asarray(outs[k]).astype(np.int64)
    return out


def rank_row_counts(n_landmarks, n_frames: int, world: int) -> list[int]:
    """Landmark rows each rank's block appends (the gathered per-frame n_landmarks summed over
    every rank's `shard_range`): every rank knows every rank's count without a collective."""
    n_landmarks = np.asarray(n_landmarks, np.int64)
    return [int(n_landmarks[slice(*shard_range(n_frames, world, r))].sum()) for r in range(world)]


def any_rank(flag: bool, group=None, device=None) -> bool:
    """True on every rank of the group if `flag` is true on any (one MAX all-reduce of a
    single int: on `device` for RCCL, on the CPU for gloo).  Ranks agree on an error before a
    collective that a failing rank would otherwise leave the others waiting in."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if flag else 0], dtype=torch.int32,
                     device=torch.device("cpu") if device is None else torch.device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(t.item())


def gather_rows_to_root(rows_local, counts, group=None, device=None, out=None):
    """Rank 0 of the group receives every rank's world landmark rows (float32 [counts[r], 3], rank
    order = frame order) as one host array; the other ranks get None.  One dist.gather of
    buffers padded to max(counts): with device=<cuda device> the buffers stay on the device
    (RCCL over xGMI; `rows_local` may already be such a tensor of at least max(counts) rows), with
    device=None they are CPU tensors (gloo).  Only rank 0 copies rows to the host: into `out` (a
    CPU float32 tensor [>= sum(counts), 3], e.g. pinned memory allocated ahead) when given, the
    result then being a view of it."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if len(counts) != world:
        raise ValueError(f"{len(counts)} row counts for a world of {world}")
    m = max(max(counts), 1)
    dev = torch.device("cpu") if device is None else torch.device(device)
    if torch.is_tensor(rows_local) and rows_local.device == dev and rows_local.dtype == torch.float32 \
            and rows_local.dim() == 2 and rows_local.shape[0] >= m and rows_local.shape[1] == 3:
        buf = rows_local[:m]
    else:
        loc = rows_local if torch.is_tensor(rows_local) else torch.from_numpy(np.asarray(rows_local, np.float32))
        loc = loc.reshape(-1, 3)[: counts[rank]]
        buf = torch.zeros((m, 3), dtype=torch.float32, device=dev)
        buf[: loc.shape[0]] = loc.to(dev)
    buf = buf.contiguous()
    dst = 0 if group is None else dist.get_global_rank(group, 0)
    if rank != 0:
        dist.gather(buf, None, dst=dst, group=group)
        return None
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.gather(buf, parts, dst=dst, group=group)
    return to_host(torch.cat([p[:c] for p, c in zip(parts, counts)]), out)


def to_host(rows, out=None):
    """float32 [n, 3] rows -> host numpy: a copy into `out` (CPU tensor with room for them, e.g.
    pinned memory allocated before a timed region: one DMA, no page-locking on the way) viewed as
    numpy, else a plain .cpu() copy."""
    n = rows.shape[0]
    if out is not None and out.dim() == 2 and out.shape[0] >= n and out.shape[1] == 3 and out.dtype == rows.dtype:
        out[:n].copy_(rows)
        return out[:n].numpy()
    return rows.cpu().numpy()


def world_landmarks(poses: np.ndarray, n_landmarks: np.ndarray, X: np.ndarray, keep: np.ndarray,
                    to_world) -> np.ndarray:
    """CreateLandmarksFromFeatures.m:17 after the chain: frame f's n_landmarks[f] camera-frame
    rows (consecutive in X/keep, frame order) go to the world with poses[f].  `to_world(pose,
    X, keep)` is libvo's vo_landmarks_to_world (or the oracle's, in the libvo-free tests)."""
    n_landmarks = np.asarray(n_landmarks, np.int64)
    if int(n_landmarks.sum()) != len(keep):
        raise ValueError(f"landmark rows {len(keep)} != sum of per-frame counts {int(n_landmarks.sum())}")
    out = np.zeros((len(keep), 3))
    r = 0
    for f, k in enumerate(n_landmarks):
        if k:
            out[r:r + k] = to_world(poses[f], X[r:r + k], keep[r:r + k])
            r += k
    return out
