"""KITTI odometry I/O, trajectory output, accuracy evaluation and map persistence
(host side, around the libvo hot path).

Mirrors what `VO.m` does around its per-frame loop:
  * sequence layout and loading   -- `VO.m:13-17` (times.txt, image_0/image_1 PNG datastores),
    `VO.m:23-38` (calib.txt: P0/P1 rows read with `readmatrix`, columns 2:13, row-major 3x4);
  * undistortImage (`VO.m:75-76`): restated (`undistort`), and with the zero-distortion
    `cameraIntrinsics` of `VO.m:50-51` it is the identity on u8 images (`undistort_identity`
    checks the sampling map), so frames go to libvo unchanged;
  * trajectory                    -- `VO.m:130-134` (`pose = pose * rel_pose`, `all_poses`),
    written in the KITTI 3x4 row-major pose format;
  * accuracy                      -- `PlotOnMap.m:1-26`: the reference's lagged xz error
    (estimate of frame k against ground truth of frame k-1, quirk Q5) and the plain
    absolute trajectory error (ATE RMSE, frames aligned by index, both anchored at frame 0);
  * landmark map                  -- `CreateLandmarksFromFeatures.m:20`, `VO.m:253`: the
    accumulated world points as .npy and ASCII .ply.

PNG decoding runs on host threads (PIL) ahead of the GPU; batches are staged in pinned host
memory and copied to the device asynchronously.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
from dataclasses import dataclass
from pathlib import Path

import numpy as np


# ---------------------------------------------------------------------------------------
# text formats
# ---------------------------------------------------------------------------------------
def read_calib(path: str | os.PathLike) -> dict[str, np.ndarray]:
    """calib.txt -> {"P0": 3x4, "P1": 3x4, ...}.  Same values as `VO.m:23-32`
    (readmatrix drops the "Pk:" label column; columns 2:13 reshaped row-major)."""
    out = {}
    for line in Path(path).read_text().splitlines():
        if ":" not in line:
            continue
        key, vals = line.split(":", 1)
        v = np.array([float(x) for x in vals.split()], np.float64)
        if v.size == 12:
            out[key.strip()] = v.reshape(3, 4)
    if "P0" not in out or "P1" not in out:
        raise ValueError(f"{path}: no P0/P1 rows")
    return out


def read_times(path: str | os.PathLike) -> np.ndarray:
    """times.txt -> seconds per frame (`VO.m:13`)."""
    return np.array([float(x) for x in Path(path).read_text().split()], np.float64)


def read_poses(path: str | os.PathLike) -> np.ndarray:
    """KITTI pose file (12 floats per line, 3x4 row-major camera-to-world) -> [n, 4, 4]."""
    rows = [np.array([float(x) for x in ln.split()], np.float64) for ln in Path(path).read_text().splitlines()
            if ln.strip()]
    P = np.zeros((len(rows), 4, 4))
    for i, r in enumerate(rows):
        if r.size != 12:
            raise ValueError(f"{path}:{i + 1}: expected 12 values, got {r.size}")
        P[i, :3, :] = r.reshape(3, 4)
        P[i, 3, 3] = 1.0
    return P


def write_poses(path: str | os.PathLike, poses: np.ndarray) -> None:
    """[n, 4, 4] camera-to-world poses -> KITTI pose file (frame 0 first)."""
    with open(path, "w") as f:
        for T in np.asarray(poses, np.float64):
            f.write(" ".join(f"{v:.9e}" for v in T[:3, :].reshape(-1)) + "\n")


# ---------------------------------------------------------------------------------------
# accuracy (PlotOnMap.m)
# ---------------------------------------------------------------------------------------
def lagged_xz_error(est: np.ndarray, gt: np.ndarray) -> np.ndarray:
    """The reference's error curve (`PlotOnMap.m:8-20`): for j = 1..n-1 (1-based all_poses
    index), || xz(GT row j) - xz(all_poses(j)) || where all_poses(j) is the estimate of
    0-based frame j and GT row j is 0-based frame j-1 -- a one-frame lag (quirk Q5).
    `est` and `gt` are [n, 4, 4] with frame 0 first; returns n-1 errors."""
    est = np.asarray(est, np.float64)
    gt = np.asarray(gt, np.float64)
    n = min(len(est), len(gt) + 1)
    t_est = est[1:n, [0, 2], 3]
    t_gt = gt[0:n - 1, [0, 2], 3]
    return np.linalg.norm(t_gt - t_est, axis=1)


def ate_rmse(est: np.ndarray, gt: np.ndarray) -> float:
    """Absolute trajectory error: RMSE of camera positions, frames matched by index, both
    trajectories anchored at frame 0 (KITTI GT frame 0 is the identity, as is ours)."""
    est = np.asarray(est, np.float64)
    gt = np.asarray(gt, np.float64)
    n = min(len(est), len(gt))
    d = est[:n, :3, 3] - gt[:n, :3, 3]
    return float(np.sqrt(np.mean(np.sum(d * d, axis=1))))


# ---------------------------------------------------------------------------------------
# landmark map (CreateLandmarksFromFeatures.m:20, VO.m:253)
# ---------------------------------------------------------------------------------------
def save_landmarks(path: str | os.PathLike, pts: np.ndarray) -> None:
    """Write the accumulated map: .npy (float64 [L, 3]) or ASCII .ply by extension.
    Zero rows (quirk Q4) are kept, as the reference's `landmarks` array keeps them."""
    pts = np.asarray(pts, np.float64).reshape(-1, 3)
    p = Path(path)
    if p.suffix == ".npy":
        np.save(p, pts)
    elif p.suffix == ".ply":
        with open(p, "w") as f:
            f.write("ply\nformat ascii 1.0\n")
            f.write(f"element vertex {len(pts)}\nproperty double x\nproperty double y\nproperty double z\n")
            f.write("end_header\n")
            for x, y, z in pts:
                f.write(f"{x:.9g} {y:.9g} {z:.9g}\n")
    else:
        raise ValueError(f"{path}: use .npy or .ply")


def load_landmarks(path: str | os.PathLike) -> np.ndarray:
    p = Path(path)
    if p.suffix == ".npy":
        return np.load(p)
    lines = p.read_text().splitlines()
    n = int(next(ln for ln in lines if ln.startswith("element vertex")).split()[2])
    start = lines.index("end_header") + 1
    return np.array([[float(v) for v in ln.split()] for ln in lines[start:start + n]], np.float64).reshape(-1, 3)


# ---------------------------------------------------------------------------------------
# sequence loading
# ---------------------------------------------------------------------------------------
def undistort_map(K: np.ndarray, dist, rows: int, cols: int):
    """undistortImage's sampling map (`VO.m:75-76`, OutputView 'same'): output pixel (u, v)
    samples the distorted image at K * distort(K^-1 [u, v, 1]) with the Brown-Conrady model
    (radial k1, k2[, k3], tangential p1, p2; `cameraIntrinsics` RadialDistortion /
    TangentialDistortion).  -> (us, vs) float64 [rows, cols] (0-based pixel coordinates)."""
    K = np.asarray(K, np.float64)
    k = list(dist) + [0.0] * (5 - len(dist))
    k1, k2, p1, p2, k3 = k[0], k[1], k[2], k[3], k[4]
    v, u = np.mgrid[0:rows, 0:cols].astype(np.float64)
    fx, fy, s, cx, cy = K[0, 0], K[1, 1], K[0, 1], K[0, 2], K[1, 2]
    y = (v - cy) / fy
    x = (u - cx - s * y) / fx
    r2 = x * x + y * y
    rad = 1.0 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2
    xd = x * rad + 2.0 * p1 * x * y + p2 * (r2 + 2.0 * x * x)
    yd = y * rad + p1 * (r2 + 2.0 * y * y) + 2.0 * p2 * x * y
    return fx * xd + s * yd + cx, fy * yd + cy


def undistort(img: np.ndarray, K: np.ndarray, dist=(0.0, 0.0, 0.0, 0.0)) -> np.ndarray:
    """undistortImage(I, intrinsics) for a u8 image: bilinear interpolation at the
    undistort_map positions, 0 outside the image, rounded back to u8 (MATLAB keeps the
    input class)."""
    img = np.asarray(img)
    rows, cols = img.shape
    us, vs = undistort_map(K, dist, rows, cols)
    x0, y0 = np.floor(us), np.floor(vs)
    fx, fy = us - x0, vs - y0
    x0, y0 = x0.astype(np.int64), y0.astype(np.int64)
    f = img.astype(np.float64)

    def at(yy, xx):
        ok = (yy >= 0) & (yy < rows) & (xx >= 0) & (xx < cols)
        return np.where(ok, f[np.clip(yy, 0, rows - 1), np.clip(xx, 0, cols - 1)], 0.0)
    out = (at(y0, x0) * (1 - fx) * (1 - fy) + at(y0, x0 + 1) * fx * (1 - fy)
           + at(y0 + 1, x0) * (1 - fx) * fy + at(y0 + 1, x0 + 1) * fx * fy)
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def undistort_identity(K: np.ndarray, dist=(0.0, 0.0, 0.0, 0.0), rows: int = 376, cols: int = 1241) -> bool:
    """True when undistortImage cannot change any u8 image: every sample position of
    undistort_map is within 1e-6 px of its own pixel, so the bilinear weights of the
    neighbours are < 1e-6 and the rounded result is the input byte.  `VO.m:50-51` builds
    cameraIntrinsics with zero distortion, which makes `VO.m:75-76` the identity: libvo takes
    the frames unchanged, and KittiSequence checks this for its calibration."""
    us, vs = undistort_map(K, dist, rows, cols)
    v, u = np.mgrid[0:rows, 0:cols]
    return bool(np.abs(us - u).max() < 1e-6 and np.abs(vs - v).max() < 1e-6)


def _read_png(path: Path) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        if im.mode != "L":
            im = im.convert("L")
        return np.asarray(im, np.uint8).copy()


@dataclass
class KittiSequence:
    """A KITTI odometry sequence in the reference's layout:
    <root>/<seq>/{image_0,image_1}/%06d.png, <root>/<seq>/{calib.txt,times.txt},
    optional ground truth <root>/poses/<seq>.txt."""
    root: Path
    seq: str = "00"
    threads: int = 8

    def __post_init__(self):
        self.root = Path(self.root)
        d = self.root / self.seq
        self.left = sorted((d / "image_0").glob("*.png"))
        self.right = sorted((d / "image_1").glob("*.png"))
        if not self.left or len(self.left) != len(self.right):
            raise FileNotFoundError(f"{d}: image_0/image_1 PNG lists missing or of different length")
        cal = read_calib(d / "calib.txt")
        self.P1, self.P2 = cal["P0"], cal["P1"]          # VO.m's p1 / p2 (left, right)
        first = _read_png(self.left[0])
        self.rows, self.cols = first.shape
        # VO.m:50-51 (zero distortion) makes VO.m:75-76 undistortImage the identity
        if not undistort_identity(self.P1[:, :3], rows=self.rows, cols=self.cols):
            raise ValueError("undistortImage with these intrinsics is not the identity")
        self.times = read_times(d / "times.txt") if (d / "times.txt").exists() else None
        gt = self.root / "poses" / f"{self.seq}.txt"
        self.gt = read_poses(gt) if gt.exists() else None
        self._pool = cf.ThreadPoolExecutor(max_workers=self.threads)

    def __len__(self) -> int:
        return len(self.left)

    def _load(self, i: int) -> tuple[np.ndarray, np.ndarray]:
        l, r = _read_png(self.left[i]), _read_png(self.right[i])
        if l.shape != (self.rows, self.cols) or r.shape != (self.rows, self.cols):
            raise ValueError(f"frame {i}: image size differs from frame 0")
        return l, r

    def batches(self, batch: int, start: int = 0, stop: int | None = None):
        """Yield (first_frame, L [b, H, W] u8, R [b, H, W] u8); PNG decode of the next batch
        runs on the thread pool while the caller processes the current one."""
        stop = len(self) if stop is None else min(stop, len(self))

        def submit(b0):
            return [self._pool.submit(self._load, i) for i in range(b0, min(b0 + batch, stop))]

        pending = submit(start) if start < stop else None
        b0 = start
        while pending:
            nxt = b0 + batch
            ahead = submit(nxt) if nxt < stop else None
            pairs = [f.result() for f in pending]
            yield b0, np.stack([p[0] for p in pairs]), np.stack([p[1] for p in pairs])
            pending, b0 = ahead, nxt

    def close(self):
        self._pool.shutdown(wait=True)


def _pipelined(ctx, batches, dev, on_collect=None, depth: int | None = None) -> list:
    """Drive the loop body through vo_step_submit_dev / vo_step_collect: while batch n's
    kernels run, the host decodes and uploads batch n+1 (threaded PNG decode, pinned H2D),
    and batch n+1's SIFT overlaps batch n's geometry.  Up to `depth` batches are in flight
    (default vo.STEP_DEPTH = 3, so batch n+2's scale space is queued before batch n's geometry
    ends; 2 with `on_collect`, whose vo_fetch_tracks needs the collected batch's buffer set
    intact).  Input tensors stay referenced until their batch is collected."""
    import torch
    from . import vo
    if depth is None:
        depth = 2 if on_collect is not None else vo.STEP_DEPTH
    outs, inflight = [], []

    def collect():
        outs.append(ctx.step_collect())
        b0, L = inflight.pop(0)[2:]
        if on_collect is not None:
            on_collect(b0, L, outs)
    for b0, L, R in batches:
        if isinstance(L, torch.Tensor):                       # device-resident frames
            dl, dr = L.contiguous(), R.contiguous()
            # the frames' producer (and any .contiguous() copy) ran on torch's current stream,
            # which libvo's non-blocking streams do not wait for: wait for it only when it still
            # has work queued (a resident, already-synchronised sequence costs a query per batch)
            ts = torch.cuda.current_stream(dl.device)
            if not ts.query():
                ts.synchronize()
            L = L.cpu().numpy() if on_collect is not None else None
        else:
            dl = torch.from_numpy(L).pin_memory().to(dev, non_blocking=True)
            dr = torch.from_numpy(R).pin_memory().to(dev, non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()     # inputs ready before the submit
        ctx.step_submit_dev(dl.data_ptr(), dr.data_ptr(), dl.shape[0])
        inflight.append((dl, dr, b0, L if on_collect is not None else None))
        if ctx.steps_pending() == depth:
            collect()
    while ctx.steps_pending():
        collect()
    return outs


def run(seq: KittiSequence, batch: int = 16, stop: int | None = None, device: int | None = None, ctx=None,
        viz_dir: str | os.PathLike | None = None, viz_every: int = 100):
    """The VO.m loop over a KITTI sequence through libvo: frames in batches of `batch`
    (pipelined vo_step_submit_dev / vo_step_collect, tracking carried across batches), H2D
    from pinned host buffers.  With `viz_dir`, every `viz_every`-th frame writes the reference's
    figures (`viz.snapshot`: img/<i>/view.png, map.svg, error.svg, 3d_map.svg; the landmark map
    in them includes the whole batch of frame i).
    Returns (poses [n, 4, 4] with frame 0 = identity, per-frame vo_step_out records,
    landmarks [L, 3])."""
    import torch
    from . import vo
    device = _local_device() if device is None else device
    own = ctx is None
    if own:
        ctx = vo.Context(seq.rows, seq.cols, batch, device=device, calib=vo.calib_from(seq.P1, seq.P2))
    hook = None
    if viz_dir is not None:
        from . import viz

        def hook(b0, L, done):                               # VO.m:168-199 every viz_every-th frame
            poses = np.stack([o["pose"] for o in np.concatenate(done)])
            for f in range(L.shape[0]):
                i = b0 + f
                if i > 0 and i % viz_every == 0:
                    viz.snapshot(viz_dir, i, L[f], ctx.fetch_tracks(f), poses[: i + 1], seq.gt, seq.times,
                                 ctx.get_landmarks())
    outs = _pipelined(ctx, seq.batches(batch, 0, stop), torch.device("cuda", device), hook)
    outs = np.concatenate(outs) if outs else np.zeros(0, vo.STEP_DTYPE)
    poses = np.stack([o["pose"] for o in outs]) if len(outs) else np.zeros((0, 4, 4))
    lm = ctx.get_landmarks()
    if own:
        ctx.close()
    return poses, outs, lm


def device_batches(dL, dR, batch: int, start: int = 0, stop: int | None = None):
    """Batches of device-resident frames (torch uint8 tensors [n, H, W] on the GPU), in the
    (first_frame, L, R) form `_pipelined` takes; no copies."""
    stop = dL.shape[0] if stop is None else min(stop, dL.shape[0])
    for b0 in range(start, stop, batch):
        yield b0, dL[b0:min(b0 + batch, stop)], dR[b0:min(b0 + batch, stop)]


def _local_device() -> int:
    """This process's GPU: LOCAL_RANK under torchrun (one process per GPU), else 0."""
    return int(os.environ.get("LOCAL_RANK", "0"))


def run_shard(seq, rank: int, world: int, batch: int = 16, device: int | None = None,
              stop: int | None = None, ctx=None, rows_to_host: bool = True):
    """One rank's part of a frame-sharded run (`sharding.py`): the block
    [start, end) of frames plus a one-frame halo, MSAC keyed by the global frame index,
    landmark rows kept in the camera frame.  `seq` is a KittiSequence (PNG frames) or a
    (L, R) pair of device tensors [n, H, W] holding the whole sequence (or at least
    frames [halo, end)).  Returns (outs: the block's STEP_DTYPE records [end - start],
    X [L, 3] float32, keep [L] bool: the block's camera-frame landmark rows).  With
    rows_to_host=False (and a caller-owned `ctx`) the rows stay in the context's device store
    for `finish_shard` and X, keep are None."""
    import torch
    from . import sharding, vo
    if not rows_to_host and ctx is None:        # checked before any context or frame work
        raise ValueError("run_shard: rows_to_host=False needs a caller-owned ctx (the rows live in it)")
    device = _local_device() if device is None else device
    on_device = isinstance(seq, tuple)
    n_all = seq[0].shape[0] if on_device else len(seq)
    n = n_all if stop is None else min(stop, n_all)
    s, e = sharding.shard_range(n, world, rank)
    h = sharding.halo_start(s)
    own = ctx is None
    if own:
        rows, cols = (seq[0].shape[1], seq[0].shape[2]) if on_device else (seq.rows, seq.cols)
        ctx = vo.Context(rows, cols, batch, device=device, calib=vo.calib_from(seq_calib(seq)[0], seq_calib(seq)[1]))
    ctx.reset()
    ctx.set_landmark_frame(True)
    ctx.set_frame_index(h)
    src = device_batches(seq[0], seq[1], batch, h, e) if on_device else seq.batches(batch, h, e)
    outs = _pipelined(ctx, src, torch.device("cuda", device))
    X, keep = ctx.get_landmark_rows() if rows_to_host else (None, None)
    if own:
        ctx.close()
    outs = np.concatenate(outs) if outs else np.zeros(0, vo.STEP_DTYPE)
    return outs[s - h:], X, keep


def seq_calib(seq):
    """(P1, P2) of a KittiSequence, or of a device-frame tuple (L, R[, P1, P2])."""
    if isinstance(seq, tuple):
        if len(seq) >= 4:
            return seq[2], seq[3]
        from .synthetic import KITTI00_P0, KITTI00_P1
        return KITTI00_P0, KITTI00_P1
    return seq.P1, seq.P2


def assemble(steps: dict, X: np.ndarray, keep: np.ndarray, to_world=None):
    """World poses (VO.m:130 chain, failed frames hold the pose) and the world landmark map
    (CreateLandmarksFromFeatures.m:17 per frame, after the chain) from gathered frame records
    and camera-frame landmark rows.  Default: libvo's host functions (vo_chain_poses,
    vo_landmarks_to_world_frames: one C call each); with `to_world` (the oracle's, in the
    libvo-free tests) the Python chain of `sharding` and one call per frame."""
    from . import sharding
    if to_world is None:
        from . import vo
        poses = vo.chain_poses(steps["rel_pose"], steps["status"])
        return poses, vo.landmarks_to_world_frames(poses, steps["n_landmarks"], X, keep)
    poses = sharding.chain(steps["rel_pose"], status=steps["status"])
    lm = sharding.world_landmarks(poses, steps["n_landmarks"], X, keep, to_world)
    return poses, lm


def finish_shard(ctx, outs, n: int, rank: int, world: int, device: int, group=None, distributed: bool = True,
                 collective_device=None, timings: dict | None = None, map_out=None):
    """The tail of a frame-sharded run after `run_shard(..., rows_to_host=False)` (SURVEY §8(e)
    step 4-5, `sharding.py`):
      1. one all-gather of the per-frame records (relative pose, status, counts: 23 doubles per
         frame) -- skipped with distributed=False (one process);
      2. every rank chains the world poses itself (VO.m:130, libvo vo_chain_poses);
      3. every rank moves its OWN camera-frame rows to the world on the device with its frames'
         chained poses (CreateLandmarksFromFeatures.m:17, vo_landmarks_world_dev);
      4. the world rows go to rank 0 only (one dist.gather; RCCL from device buffers when
         collective_device is the rank's GPU, CPU tensors for gloo).
    Returns (world poses [n, 4, 4], gathered per-frame records, landmarks float32 [L, 3] on rank 0
    -- single-rounded values, equal to a single-process run's rows -- and None on other ranks).
    `timings` (a dict) receives the seconds of each step: records, chain, world (device
    transform), map (gather to rank 0 + its copy to the host).  `map_out`: rank 0's host buffer
    for the map (CPU float32 tensor [>= rows, 3], e.g. pinned, allocated ahead; the returned map
    is then a view of it)."""
    import time
    import torch
    from . import sharding, vo
    tm = timings if timings is not None else {}
    t0 = time.perf_counter()
    steps = sharding.gather_steps(outs, n, group=group, device=collective_device) if distributed \
        else sharding.steps_of(outs)
    t1 = time.perf_counter()
    poses = vo.chain_poses(steps["rel_pose"], steps["status"])
    t2 = time.perf_counter()
    counts = sharding.rank_row_counts(steps["n_landmarks"], n, world)
    s, e = sharding.shard_range(n, world, rank)
    h = sharding.halo_start(s)
    m = max(max(counts), 1)
    buf = torch.empty((m, 3), dtype=torch.float32, device=torch.device("cuda", device))
    rows = ctx.landmarks_world_dev(poses[h:e], buf.data_ptr(), m)
    bad = rows != counts[rank]
    if distributed and sharding.any_rank(bad, group=group, device=collective_device):
        # every rank learns of a mismatch before the gather, so none is left waiting in it
        raise RuntimeError(f"rank {rank}: {rows} landmark rows on the device, records say {counts[rank]}"
                           + ("" if bad else " on another rank"))
    if bad:
        raise RuntimeError(f"rank {rank}: {rows} landmark rows on the device, records say {counts[rank]}")
    t3 = time.perf_counter()
    if not distributed:
        lm = sharding.to_host(buf[:rows], map_out)
    else:
        lm = sharding.gather_rows_to_root(buf if collective_device is not None else buf[:rows].cpu(), counts,
                                          group=group, device=collective_device, out=map_out)
    tm.update(records=t1 - t0, chain=t2 - t1, world=t3 - t2, map=time.perf_counter() - t3)
    return poses, steps, lm


def run_distributed(seq, batch: int = 16, device: int | None = None, stop: int | None = None,
                    group=None):
    """Frame-sharded run over a torch.distributed group (one process per GPU; RCCL over
    xGMI with the nccl backend): every rank runs its block (`run_shard`, landmark rows kept on
    the device), then `finish_shard`: one all-gather of the per-frame records, the world-pose
    chain on every rank (host product of `VO.m:130`), each rank's own rows moved to the world on
    its device (`CreateLandmarksFromFeatures.m:17`) and gathered to rank 0.  Returns (world
    poses [n, 4, 4], gathered per-frame records, landmarks float32 [L, 3] on rank 0 / None on the
    other ranks), equal bit for bit to a single-process run."""
    import torch
    import torch.distributed as dist
    from . import sharding, vo
    device = _local_device() if device is None else device
    n_all = seq[0].shape[0] if isinstance(seq, tuple) else len(seq)
    n = n_all if stop is None else min(stop, n_all)
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if isinstance(seq, tuple):
        rows, cols = seq[0].shape[1], seq[0].shape[2]
    else:
        rows, cols = seq.rows, seq.cols
    P1, P2 = seq_calib(seq)
    ctx = vo.Context(rows, cols, batch, device=device, calib=vo.calib_from(P1, P2))
    try:
        outs, _, _ = run_shard(seq, rank, world, batch, device, n, ctx=ctx, rows_to_host=False)
        dev = torch.device("cuda", device) if dist.get_backend(group) == "nccl" else None
        return finish_shard(ctx, outs, n, rank, world, device, group=group, collective_device=dev)
    finally:
        ctx.close()
