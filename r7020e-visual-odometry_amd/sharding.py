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
in the camera frame (libvo vo_set_landmark_frame), the rows are all-gathered in
frame order (`gather_landmark_rows`), and `world_landmarks` applies :17 per frame
with the chained pose -- the same rows, bit for bit, that a single process
appends.
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
    local = np.asarray(local, np.float64).reshape(len(local), -1)
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


def gather_landmark_rows(X_local: np.ndarray, keep_local: np.ndarray, group=None, device=None):
    """All-gather the camera-frame landmark rows of every rank (rank order = frame order)
    -> (X [L, 3] float32, keep [L] bool).  Two collectives: the row counts, then the rows
    padded to the largest count (float32 x, y, z, keep: exact)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([len(keep_local)], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(max(counts), 1)
    buf = torch.zeros((m, 4), dtype=torch.float32, device=device)
    if len(keep_local):
        loc = np.concatenate([np.asarray(X_local, np.float32).reshape(-1, 3),
                              np.asarray(keep_local, np.float32).reshape(-1, 1)], 1)
        buf[: len(loc)] = torch.from_numpy(loc).to(buf.device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    rows = np.concatenate([parts[r][: counts[r]].cpu().numpy() for r in range(world)])
    return rows[:, :3].copy(), rows[:, 3] != 0


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
