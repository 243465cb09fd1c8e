#!/usr/bin/env python3
"""bench.py — stereo frames/s of the VO hot path on MI355X.

Workload (BASELINE.json configs[1]): SIFT detect+describe of both images +
stereo matchFeatures, on 1242x375 synthetic stereo pairs (~2k keypoints per
image), via libvo.so (hand-written HIP, gfx950).  One step = one batch of
`--batch` independent stereo frames already resident in HBM (default 256: +1.4 % at 128 over
64, +4.1-6.6 % at 256 over 128, 512 slower again -- profiles/r05_o_batch.txt).  With --gpus N
(one process per GPU, RCCL; under torchrun, or bench.py starts torchrun itself
when WORLD_SIZE is unset) each rank processes its own frames: weak scaling, no
data-path collective; value = all frames / max-over-ranks time.

Prints ONE JSON line (rank 0) with the driver's contract fields plus
`roofline` (dominant kernel, HIP-event durations measured in this process)
and `cpu_baseline` (the CPU oracle on a bounded sample, rank 0 at N=1).
`full_path` additionally times the full per-frame path (BASELINE configs[2]/[3]:
SIFT, stereo match, tracking, DLT, P3P+MSAC with 2048 hypotheses, landmarks) over
the KITTI-00 trajectory: 4541 frames rendered at 376x1241 along the reference's
ground truth (street.py), block-sharded over the ranks with a one-frame halo,
per-frame records all-gathered, poses chained on every rank, each rank's landmark
rows moved to the world on its device and gathered to rank 0; it reports the reference's lagged xz error
(PlotOnMap.m:8-20) and ATE against that trajectory (--seq-frames; 0 skips), and
`large` the 1920x1080 / ~8k keypoint configuration (configs[4]) per GPU with the
i8-MFMA rate of its dense stereo match block (--large-batch, default 128; 0 skips).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))   # cpu_baseline leg only

import numpy as np  # noqa: E402

ROWS, COLS = 375, 1242
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
F64_VECTOR_PEAK_TF = 78.6     # MI355X spec FP64 vector (the guide lists FP32 vector 157.3 TF; FP64 is half)
I8_MFMA_PEAK_TOPS = 5000.0     # MI355X_MICROARCH.md "Matrix cores": I8 = 2x the dense BF16 ~2.5 PF per clock
# per-launch HBM bytes of each kernel from rocprofv3 FETCH_SIZE/WRITE_SIZE passes on this
# workload (tools/pmc_passes.sh + tools/pmc_traffic.py; FETCH_SIZE doubled on gfx950)
# (the newest profiles/r<NN>_pmc_traffic.json)
def _traffic_key(p):
    # r<NN>_<tag>_pmc_traffic.json: the round, then the tag in a..z, aa..zz order
    parts = p.name.split("_")
    tag = parts[1] if len(parts) > 3 else ""
    return (int(parts[0][1:]) if parts[0][1:].isdigit() else 0, len(tag), tag)


TRAFFIC_FILE = max(ROOT.glob("profiles/r*_pmc_traffic.json"), key=_traffic_key,
                   default=ROOT / "profiles" / "r01_pmc_traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="timed steps per run (--batch frames each: 5120 frames per run at 256)")
    ap.add_argument("--runs", type=int, default=5, help="timed runs of --steps steps; value = the median run (SURVEY §8d)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="stereo frames per step (library maximum VO_MAX_BATCH = 512)")
    ap.add_argument("--cpu-frames", type=int, default=32, help="frames in the CPU-oracle baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16, help="host threads for the CPU baseline (the box's share)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=3)
    ap.add_argument("--concurrency", type=int, default=0, help="forked streams per batch (0: library default)")
    ap.add_argument("--seq-frames", type=int, default=4541,
                    help="KITTI-00 trajectory frames through the full per-frame path, sharded over the ranks (0: skip)")
    ap.add_argument("--seq-batch", type=int, default=256,
                    help="frames per vo_step_submit_dev call in the sequence leg (3 in flight; 64: 8644, 128: 8862, "
                         "256: 9128 stereo frames/s, profiles/r06_b_seq_*)")
    ap.add_argument("--dry-run", action="store_true",
                    help="rendezvous only (gloo, no GPU): rank 0 prints the world size it sees (launcher test)")
    ap.add_argument("--large-batch", type=int, default=128,
                    help="1920x1080 (~8k keypoints) stereo pairs per step for the configs[4] figure (0: skip)")
    return ap.parse_args()


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N ranks with torchrun (one process per
    GPU, rendezvous on 127.0.0.1) as a child process -- before this process touches the GPU --
    and return its exit code.  Rank 0 prints the JSON line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve())] + sys.argv[1:]
    # stdout carries exactly the JSON line: collective-library chatter (gloo prints its
    # connection log to stdout) goes to stderr
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    for line in p.stdout:
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    return p.wait()


def feature_traffic(fmodel, kt, kt_iso, profile_steps, B):
    """Per-kernel feature-stage bytes of one call: the algorithmic and line-floor model
    (roofline.feature_bytes) beside the PMC traffic of the same workload (TRAFFIC_FILE: FETCH_SIZE
    x 2 + WRITE_SIZE, per launch x launches per call) and the algorithmic GB/s in situ / isolated."""
    tr = json.loads(TRAFFIC_FILE.read_text())["kernels"] if TRAFFIC_FILE.exists() else {}
    calls = tr.get("k_blur_base", {}).get("launches", 0) or 1       # one octave-0 base launch per call
    out, tot_pmc, tot_alg = {}, 0.0, 0.0
    for name, m in fmodel.items():
        e = {"algorithmic_bytes": m["algorithmic"], "line_floor_bytes": m["line_floor"]}
        t = tr.get(name)
        if t:
            pmc = t["hbm_bytes_per_launch"] * t["launches"] / calls
            e.update(pmc_bytes=pmc, pmc_over_algorithmic=pmc / m["algorithmic"] if m["algorithmic"] else None,
                     pmc_over_line_floor=pmc / m["line_floor"] if m["line_floor"] else None)
            tot_pmc += pmc
        tot_alg += m["algorithmic"]
        if name in kt and kt[name][0] > 0:
            e["gbs_in_situ"] = round(m["algorithmic"] / (kt[name][0] / profile_steps * 1e-3) / 1e9, 1)
        if name in kt_iso and kt_iso[name][0] > 0:
            e["gbs_isolated"] = round(m["algorithmic"] / (kt_iso[name][0] / profile_steps * 1e-3) / 1e9, 1)
        out[name] = e
    return {"kernels": out, "pmc_gb_per_64_frames": tot_pmc / 1e9 * 64 / B, "algorithmic_gb_per_64_frames": tot_alg / 1e9 * 64 / B,
            "traffic_source": str(TRAFFIC_FILE.relative_to(ROOT)) if TRAFFIC_FILE.exists() else None,
            "note": "per call of --batch frames; PMC of the kernels the traffic file holds (FETCH_SIZE calibrated at 1/2 of "
                    "the 128-B line bytes for these access shapes, profiles/r06_c_fetch_calib.txt)"}


def sequence_leg(args, torch, rank, world, local, dist, barrier, max_over_ranks, gather_over_ranks):
    """KITTI-00 (BASELINE configs[2] at N=1, configs[3] at N=8): frames rendered along the
    reference's ground truth (street.py) into HBM -- each rank only its block + halo -- then
    timed: the sharded VO loop (vo_step_submit_dev / vo_step_collect, 2048 MSAC hypotheses),
    the all-gather of per-frame records, the pose chain (every rank), the world transform of
    each rank's own landmark rows on its device and the gather of the world rows to rank 0.  Accuracy vs the rendered trajectory: PlotOnMap.m:8-20's
    lagged xz error and ATE RMSE."""
    from r7020e_visual_odometry_amd import vo, street, kitti, sharding
    gt = street.kitti00_gt()
    n = min(args.seq_frames, len(gt))
    P0, P1 = street.kitti00_calib()
    s, e = sharding.shard_range(n, world, rank)
    h = sharding.halo_start(s)
    t0 = time.perf_counter()
    wld = street.kitti00_world(device=f"cuda:{local}", poses=gt)
    dL = torch.empty((n, street.KITTI_ROWS, street.KITTI_COLS), dtype=torch.uint8, device=f"cuda:{local}")
    dR = torch.empty_like(dL)
    street.render_frames(wld, gt, range(h, e), P0, P1, out=(dL[h:e], dR[h:e]))
    del wld
    torch.cuda.synchronize()
    render_s = time.perf_counter() - t0
    rp = vo.default_ransac_params()
    rp.max_num_trials = 2048                                   # BASELINE configs[2]
    # frames per submit: --seq-batch, but at least 8 submits per rank's block so the three-deep
    # pipeline's fill and drain stay a small part of it (8 ranks over KITTI-00: 568-frame blocks,
    # 71 per submit; one rank: 256)
    block = -(-n // world)
    SB = max(1, min(args.seq_batch, max(16, -(-block // 8))))
    ctx = vo.Context(street.KITTI_ROWS, street.KITTI_COLS, SB, device=local, calib=vo.calib_from(P0, P1), ransac=rp)
    seq = (dL, dR, P0, P1)
    ctx.reset()                                                # warm-up: the block's first two batches
    kitti._pipelined(ctx, kitti.device_batches(dL, dR, SB, h, min(e, h + 2 * SB)), torch.device("cuda", local))
    torch.cuda.synchronize()
    dev = torch.device("cuda", local) if dist is not None and dist.get_backend() == "nccl" else None
    # rank 0's host buffer for the gathered map, pinned ahead of the timed region (one DMA at the
    # end instead of a pageable copy: 0.75 vs 2.7 ms for KITTI-00's 42 MB, profiles/r05_c_*);
    # 1024 rows per frame is above any frame's count here (the map falls back to .cpu() if not)
    map_out = torch.empty((n * 1024, 3), dtype=torch.float32, pin_memory=True) if rank == 0 else None
    barrier()
    t0 = time.perf_counter()
    outs, _, _ = kitti.run_shard(seq, rank, world, SB, local, n, ctx=ctx, rows_to_host=False)
    t_loop = time.perf_counter() - t0
    # the tail: per-frame records all-gathered, chain on every rank, own rows to the world on the
    # device, world rows gathered to rank 0 only (kitti.finish_shard)
    tparts = {}
    poses, steps, lm = kitti.finish_shard(ctx, outs, n, rank, world, local, distributed=dist is not None,
                                          collective_device=dev, timings=tparts, map_out=map_out)
    el = time.perf_counter() - t0
    t_tail = el - t_loop
    barrier()
    mine = [t_loop, t_tail] + [tparts[k] for k in ("records", "chain", "world", "map")]
    per_rank = gather_over_ranks(mine)
    el = max_over_ranks(el)
    t_tail = max_over_ranks(t_tail)
    n_lm = int(np.asarray(steps["n_landmarks"]).sum())
    # load balance of the block partition: measured over this run's ranks, and projected for
    # 2 / 4 / 8 ranks from this run's per-frame keypoint counts (the SIFT + descriptor work, the
    # bulk of a frame's cost, scales with them; the scale space is the same for every frame)
    kp_cost = np.asarray(steps["n_left"], np.float64) + np.asarray(steps["n_right"], np.float64)
    loops = [v[0] for v in per_rank]
    proj = {str(w): round(sharding.block_imbalance(kp_cost, w), 4) for w in (2, 4, 8)}
    # projected 8-rank efficiency: each rank's loop = this run's per-frame loop time x its block
    # (1/8 of the frames + a halo frame) x the block's cost imbalance, plus a ~3 ms tail
    t1 = el * world / max(n, 1)                     # s per frame on one rank
    t8 = t1 * (n / 8 + 1) * proj["8"] + 3e-3
    balance = {"loop_max_over_mean": round(max(loops) / (sum(loops) / len(loops)), 4) if world > 1 else None,
               "projected_block_cost_max_over_mean": proj,
               "cost_proxy": "keypoints per frame (n_left + n_right), halo frame included",
               "projected_8_rank_efficiency": round((n * t1) / (8 * t8), 4) if world == 1 else None,
               "projected_8_rank_note": "N=1 per-frame time x (1/8 of the frames + halo) x block cost imbalance + 3 ms tail"}
    if lm is not None and len(lm) != n_lm:
        raise RuntimeError(f"landmark map has {len(lm)} rows, the records {n_lm}")
    # per-kernel HIP-event durations of the full path over the block's first PB batches (a
    # separate profiling pass: vo_step_collect synchronises every stream while profiling, so
    # these are the kernels' own durations without the pipeline's overlap), ms per SB frames
    PB = max(1, min(args.profile_steps * 3, (e - h) // SB))
    ctx.reset()
    ctx.set_landmark_frame(True)
    ctx.set_frame_index(h)
    ctx.set_profiling(True)
    pouts = np.concatenate(kitti._pipelined(ctx, kitti.device_batches(dL, dR, SB, h, h + PB * SB), torch.device("cuda", local)))
    fkt = ctx.kernel_times()
    ctx.set_profiling(False)
    ctx.close()
    del dL, dR
    fk_ms = {k: round(v[0] / PB, 4) for k, v in sorted(fkt.items(), key=lambda kv: -kv[1][0])}
    geom = ("k_compose", "k_gather_tri", "k_msac", "k_msac_gen", "k_stereo_pos", "k_lm_filter", "k_lm_tri", "k_lm_pack", "k_tri_list")
    # k_msac (lazy MSAC: slots generated and scored in chunks of 64 until the adaptive replay
    # stops -- one chunk at these inlier ratios): every scored slot reprojects every tracked
    # point -- R X + t (18), two divisions, K (6), residual and square (5), MSAC sum (1): 32 f64
    # FLOP per (slot, point).  Counted for the first chunk of every frame only, so `achieved`
    # is a lower bound; the kernel also runs the chunk's P3P solves and the replay.
    sc_ms = fkt.get("k_msac", (0.0, 1))[0]
    sc_flop = 32.0 * 64 * float(np.maximum(pouts["n_tracked"], 0).sum())
    msac = {"kernel": "k_msac", "bound": "f64 VALU", "unit": "TFLOP/s (f64)", "flop_per_slot_point": 32,
            "slots_counted": 64, "slots_configured": 2048, "frames": int(len(pouts)), "flop": sc_flop, "ms": sc_ms,
            "achieved": sc_flop / (sc_ms * 1e-3) / 1e12 if sc_ms > 0 else None, "peak": F64_VECTOR_PEAK_TF,
            "frac": sc_flop / (sc_ms * 1e-3) / 1e12 / F64_VECTOR_PEAK_TF if sc_ms > 0 else None,
            "peak_source": "MI355X spec FP64 vector 78.6 TFLOP/s (half the guide's 157.3 TF FP32 vector rate)"}
    err = kitti.lagged_xz_error(poses, gt[:n])
    ok = steps["status"][1:] == 0
    # the reference's own run (VO.m on MATLAB, the real KITTI-00 images): its lagged x-z error
    # curve digitised from reference 4500/error.png (tests/golden/digitize_ref_error.py)
    ref_curve = np.loadtxt(ROOT / "data" / "kitti" / "ref_error_digitized.csv", delimiter=",")
    return {"metric": "stereo frames/sec, full per-frame path over the KITTI-00 trajectory (BASELINE configs[2]; configs[3] at 8 GPUs)",
            "value": n / el, "unit": "stereo frames/s", "frames": n, "frames_per_rank": e - s, "batch": SB,
            "partition": f"block + one-frame halo over {world} rank(s); all-gather of per-frame records, "
                         f"landmark world rows gathered to rank 0",
            "rows": street.KITTI_ROWS, "cols": street.KITTI_COLS, "ransac_hypotheses": 2048,
            "frames_with_pose": int(ok.sum()), "mean_inliers": float(steps["n_inliers"][1:].mean()),
            "mean_keypoints_per_image": float((steps["n_left"] + steps["n_right"]).mean() / 2),
            "mean_stereo_matches": float(steps["n_stereo"].mean()), "mean_tracked": float(steps["n_tracked"][1:].mean()),
            "landmark_rows": n_lm,
            "tail_ms": round(t_tail * 1e3, 3),
            "load_balance": balance,
            "per_rank_ms": [{"rank": r, "loop": round(v[0] * 1e3, 2), "tail": round(v[1] * 1e3, 3),
                             "records": round(v[2] * 1e3, 3), "chain": round(v[3] * 1e3, 3),
                             "world": round(v[4] * 1e3, 3), "map": round(v[5] * 1e3, 3)}
                            for r, v in enumerate(per_rank)],
            "tail_note": "max over ranks: records all-gather + chain + own rows to the world on the device + "
                         "gather of world rows to rank 0 (+ its one D2H of the map)",
            "accuracy": {"lagged_xz_error_m": {"mean": float(err.mean()), "max": float(err.max()), "final": float(err[-1])},
                         "ate_rmse_m": kitti.ate_rmse(poses, gt[:n]),
                         "trajectory_length_m": float(np.linalg.norm(np.diff(gt[:n, :3, 3], axis=0), axis=1).sum()),
                         "reference": "PlotOnMap.m:8-20 (estimate of frame k vs ground truth of frame k-1); "
                                      "ATE: positions by frame index, both anchored at frame 0",
                         "reference_run_lagged_xz_error_m": {
                             "mean": float(ref_curve[:, 1].mean()), "max": float(ref_curve[:, 1].max()),
                             "final": float(ref_curve[-1, 1]),
                             "source": "VO.m on MATLAB over the real KITTI-00 images, digitised from reference "
                                       "4500/error.png (data/kitti/ref_error_digitized.csv); different input "
                                       "images than this run, so context rather than parity"}},
            "kernel_ms_per_step": fk_ms,
            "geometry_ms_per_step": round(sum(v for k, v in fk_ms.items() if k in geom), 4),
            "kernel_profile": f"HIP events, first {PB} batches of {SB} frames, collect synchronising every stream",
            "msac_score_roofline": msac,
            "render_s": render_s,
            "data": "synthetic street world rendered along reference kitti/poses/00.txt with kitti/00/calib.txt P0/P1 "
                    "(KITTI-00 images are not available)",
            "note": "timed: sharded loop body + record all-gather + pose chain + landmark world transform (device) + "
                    "gather of the world map to rank 0; inputs resident in HBM"}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    # stdout carries exactly the one JSON line: native libraries' chatter on fd 1 (RCCL prints its
    # version banner at communicator creation) goes to stderr; the line goes to a saved copy
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    import vo_amd  # noqa: F401
    from r7020e_visual_odometry_amd import vo, synthetic as syn, roofline

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (not used by the driver): several ranks on one GPU over gloo
    if os.environ.get("VO_BENCH_SAME_GPU"):
        local = 0
    backend = os.environ.get("VO_BENCH_BACKEND", "nccl")
    if args.dry_run:
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            dist.barrier()
            dist.destroy_process_group()
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world}), file=json_out, flush=True)
        return
    # VO_BENCH_FORCE_DIST=1: take the process-group branch (RCCL with the default backend) even
    # at one rank -- the only way this pool can run the collectives on hardware before an
    # 8-GPU node is available (env rendezvous on 127.0.0.1 when no launcher set it)
    force_dist = os.environ.get("VO_BENCH_FORCE_DIST") == "1"
    if force_dist and world == 1:
        import socket
        if "MASTER_PORT" not in os.environ:
            s_ = socket.socket()
            s_.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(s_.getsockname()[1])
            s_.close()
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    torch.cuda.set_device(local)
    dist = None
    if world > 1 or force_dist:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    def max_over_ranks(x: float) -> float:
        if dist is None:
            return x
        dev = f"cuda:{local}" if backend == "nccl" else "cpu"
        t = torch.tensor([x], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def gather_over_ranks(v) -> list:
        """Every rank's list of floats (same length), in rank order (reporting only)."""
        if dist is None:
            return [list(v)]
        dev = f"cuda:{local}" if backend == "nccl" else "cpu"
        t = torch.tensor(v, device=dev, dtype=torch.float64)
        parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, t)
        return [p.cpu().tolist() for p in parts]

    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}; reporting {world}", file=sys.stderr)
    B = args.batch
    # synthetic pairs: rank r renders frames [r*B, (r+1)*B) (seed 0x5EED0000 + frame); texture
    # cell of 15 px puts the oracle at ~2000 keypoints per image (2000 +- 200)
    L, R = syn.independent_pairs(B, ROWS, COLS, first=rank * B, px_per_cell=syn.BENCH_PX_PER_CELL,
                                 threads=args.cpu_threads)
    d_l = torch.from_numpy(L).to(f"cuda:{local}")
    d_r = torch.from_numpy(R).to(f"cuda:{local}")
    torch.cuda.synchronize()

    ctx = vo.Context(ROWS, COLS, B, device=local)
    if args.concurrency > 0:
        ctx.set_concurrency(args.concurrency)
    stats = ctx.sift_match_batch_dev(d_l.data_ptr(), d_r.data_ptr(), B, stats=True)
    for _ in range(args.warmup):
        ctx.sift_match_batch_dev(d_l.data_ptr(), d_r.data_ptr(), B, stats=False)
    torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # --runs timed runs of exactly --steps steps each, every run bracketed by a barrier +
    # synchronize and reduced max-over-ranks; value = the median run (median of 5)
    run_s = []
    for _ in range(max(1, args.runs)):
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ctx.sift_match_batch_dev(d_l.data_ptr(), d_r.data_ptr(), B, stats=False)
        torch.cuda.synchronize()
        el_ = time.perf_counter() - t0
        barrier()
        run_s.append(max_over_ranks(el_))
    elapsed = sorted(run_s)[len(run_s) // 2]
    frames = B * args.steps * world
    fps = frames / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    timed_runs = {"n": len(run_s), "steps_per_run": args.steps, "frames_per_run": frames,
                  "ms_per_step": [round(x / args.steps * 1e3, 4) for x in run_s],
                  "value_median": fps, "value_min": frames / max(run_s), "value_max": frames / min(run_s)}

    # H2D of one batch of u8 pairs (pinned host -> HBM), reported beside `value` (which starts
    # from resident inputs): the PCIe-inclusive rate if the frames came from the host each step
    hl = torch.from_numpy(L).pin_memory()
    hr = torch.from_numpy(R).pin_memory()
    h2d_ms = []
    for _ in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        d_l.copy_(hl, non_blocking=True)
        d_r.copy_(hr, non_blocking=True)
        e1.record()
        e1.synchronize()
        h2d_ms.append(e0.elapsed_time(e1))
    h2d = sorted(h2d_ms[1:])[len(h2d_ms[1:]) // 2]
    h2d_bytes = 2 * B * ROWS * COLS
    del hl, hr
    h2d_line = {"bytes_per_step": h2d_bytes, "ms_per_step": h2d, "gb_s": h2d_bytes / (h2d * 1e-3) / 1e9,
                "frames_per_s_serial_computed": B / ((ms_per_step + h2d) * 1e-3),
                "frames_per_s_overlapped_computed": B / (max(ms_per_step, h2d) * 1e-3),
                "note": f"measured: the pinned host -> HBM copy of the step's 2x{B} u8 images (torch, one stream), "
                        "median of 5.  COMPUTED, not measured: serial = 1 / (copy + compute), overlapped = "
                        "1 / max(copy, compute) (copy of step N+1 beside compute of step N)"}

    # ---- per-kernel HIP-event durations on libvo's streams (separate passes) ----
    # in situ: calls issued back to back exactly like the timed loop (the scale space of
    # call N+1 overlaps the feature stages of call N), so durations include that sharing
    # and agree with a rocprofv3 kernel trace of this command;
    # isolated: each call synchronised, kernels never overlap (the kernels' own speed).
    def kernel_pass(sync):
        ctx.set_profiling(True)
        for _ in range(args.profile_steps):
            ctx.sift_match_batch_dev(d_l.data_ptr(), d_r.data_ptr(), B, stats=sync)
        torch.cuda.synchronize()
        res = ctx.kernel_times()
        ctx.set_profiling(False)
        return res

    kt = kernel_pass(False)
    kt_iso = kernel_pass(True)
    model = roofline.kernel_bytes(ROWS, COLS, 2 * B)
    dom = max(kt.items(), key=lambda kv: kv[1][0])
    dom_name, (dom_ms, dom_calls) = dom
    avg_ms = dom_ms / dom_calls
    roof = {"kernel": dom_name, "bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": None,
            "avg_launch_us": avg_ms * 1e3}
    if TRAFFIC_FILE.exists():
        tr = json.loads(TRAFFIC_FILE.read_text())["kernels"].get(dom_name)
        if tr:
            roof["traffic"] = tr["hbm_bytes_per_launch"]
            roof["traffic_source"] = f"{TRAFFIC_FILE.relative_to(ROOT)} (PMC FETCH_SIZE x2 + WRITE_SIZE, per launch)"
    if dom_name in model:
        per_call_bytes, launches = model[dom_name]
        per_launch = per_call_bytes / launches
        achieved = per_launch / (avg_ms * 1e-3) / 1e9
        roof.update({"achieved": achieved, "frac": achieved / HBM_PEAK_GBS, "bytes_per_launch": per_launch})
        if dom_name in kt_iso:
            iso_ms = kt_iso[dom_name][0] / kt_iso[dom_name][1]
            roof["isolated"] = {"avg_launch_us": iso_ms * 1e3, "achieved": per_launch / (iso_ms * 1e-3) / 1e9,
                                "frac": per_launch / (iso_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    else:
        roof.update({"achieved": None, "frac": None, "bytes_per_launch": None})
    # every kernel the byte model prices: algorithmic GB/s in situ and isolated
    roof["per_kernel_gbs"] = {
        n: {"bytes_per_call": b, "in_situ": round(b / (kt[n][0] / args.profile_steps * 1e-3) / 1e9, 1),
            "isolated": round(b / (kt_iso[n][0] / args.profile_steps * 1e-3) / 1e9, 1) if n in kt_iso else None}
        for n, (b, _l) in model.items() if n in kt and kt[n][0] > 0}
    # whole-pyramid figure (SURVEY §8(d) per-frame model over the pyramid kernels' time)
    pyr_names = [n for n in kt if n.startswith(("k_blur", "k_down"))]
    pyr_ms = sum(kt[n][0] for n in pyr_names) / args.profile_steps
    pyr_bytes = 2 * B * roofline.pyramid_bytes_per_image(ROWS, COLS)
    roof["pyramid_model_gbs"] = pyr_bytes / (pyr_ms * 1e-3) / 1e9 if pyr_ms > 0 else None
    roof["kernel_ms_per_step"] = {n: round(v[0] / args.profile_steps, 4) for n, v in sorted(kt.items(), key=lambda kv: -kv[1][0])}
    roof["kernel_ms_per_step_isolated"] = {n: round(v[0] / args.profile_steps, 4)
                                           for n, v in sorted(kt_iso.items(), key=lambda kv: -kv[1][0])}

    # ---- feature stages: byte model from this call's counts against the PMC traffic ----
    # (the last call's results: the same frames as every call of the loop)
    nc = np.array([ctx.fetch_candidate_counts(i) for i in range(2 * B)])
    kps = [ctx.fetch_keypoints(i, descriptors=False)[0] for i in range(2 * B)]
    allk = np.concatenate(kps)
    fmodel = roofline.feature_bytes(ROWS, COLS, nc[:, 0], nc[:, 1], allk["size"], allk["octave"], allk["angle"],
                                    np.repeat(np.arange(2 * B), [len(k) for k in kps]), [s_[:3] for s_ in stats])
    roof["feature_traffic"] = feature_traffic(fmodel, kt, kt_iso, args.profile_steps, B)
    roof["feature_traffic"]["mean_candidates_per_image"] = float(nc[:, 0].mean())
    roof["feature_traffic"]["mean_accepted_per_image"] = float(nc[:, 1].mean())
    ctx.close()                                                # the legs below make their own contexts
    del d_l, d_r

    # ---- BASELINE configs[2]/[3]: the full per-frame path over the KITTI-00 trajectory ----
    full = None
    if args.seq_frames > 0:
        full = sequence_leg(args, torch, rank, world, local, dist, barrier, max_over_ranks, gather_over_ranks)

    # ---- BASELINE configs[4]: 1920x1080 synthetic stereo, ~8k keypoints per image, the dense
    # 8k x 8k descriptor block on the i8 matrix cores (k_match_partial) ----
    large = None
    if args.large_batch > 0:
        LB = args.large_batch
        GL, GR = syn.large_pairs(LB, first=rank * LB, threads=args.cpu_threads)
        d_gl = torch.from_numpy(GL).to(f"cuda:{local}")
        d_gr = torch.from_numpy(GR).to(f"cuda:{local}")
        lctx = vo.Context(syn.LARGE_ROWS, syn.LARGE_COLS, LB, device=local)
        lst = lctx.sift_match_batch_dev(d_gl.data_ptr(), d_gr.data_ptr(), LB, stats=True)
        for _ in range(2):
            lctx.sift_match_batch_dev(d_gl.data_ptr(), d_gr.data_ptr(), LB, stats=False)
        lsteps = max(3, args.steps // 2)
        lruns = []
        for _ in range(max(1, min(args.runs, 3))):           # median of 3 timed runs, like the headline's 5
            barrier()
            t0 = time.perf_counter()
            for _ in range(lsteps):
                lctx.sift_match_batch_dev(d_gl.data_ptr(), d_gr.data_ptr(), LB, stats=False)
            torch.cuda.synchronize()
            lel_ = time.perf_counter() - t0
            barrier()
            lruns.append(max_over_ranks(lel_))
        lel = sorted(lruns)[len(lruns) // 2]
        lctx.set_profiling(True)
        for _ in range(args.profile_steps):
            lctx.sift_match_batch_dev(d_gl.data_ptr(), d_gr.data_ptr(), LB, stats=True)
        torch.cuda.synchronize()
        lkt = lctx.kernel_times()
        lctx.set_profiling(False)
        # exact int8 MAC work of the stereo blocks: 2 ops x n1 x n2 x 128 per frame
        ops = sum(2.0 * s_[0] * s_[1] * 128 for s_ in lst)
        mp_ms = lkt.get("k_match_partial", (0.0, 1))[0] / args.profile_steps
        large = {"metric": "stereo frames/sec @1920x1080 (SIFT x2 + stereo matchFeatures, BASELINE configs[4] per GPU)",
                 "value": LB * lsteps * world / lel, "unit": "stereo frames/s", "batch": LB,
                 "timed_runs_ms_per_step": [round(x / lsteps * 1e3, 3) for x in lruns],
                 "mean_keypoints_per_image": float(np.mean([s_[0] + s_[1] for s_ in lst]) / 2),
                 "mean_stereo_matches": float(np.mean([s_[2] for s_ in lst])),
                 "match_block": {"kernel": "k_match_partial", "bound": "mfma", "unit": "TOP/s (i8)",
                                 "ops_per_step": ops, "ms_per_step": mp_ms,
                                 "achieved": ops / (mp_ms * 1e-3) / 1e12 if mp_ms > 0 else None,
                                 "peak": I8_MFMA_PEAK_TOPS,
                                 "frac": ops / (mp_ms * 1e-3) / 1e12 / I8_MFMA_PEAK_TOPS if mp_ms > 0 else None},
                 "kernel_ms_per_step": {n: round(v[0] / args.profile_steps, 4)
                                        for n, v in sorted(lkt.items(), key=lambda kv: -kv[1][0])}}
        lctx.close()
        del d_gl, d_gr

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # the CPU oracle (plain C restatement, test infrastructure) on the host cores: one
        # stereo pair per call (one C call, GIL released), `threads` calls in flight, over the
        # first --cpu-frames pairs of the GPU batch; plus a single-threaded sample
        import oracle
        from concurrent.futures import ThreadPoolExecutor
        oracle.build()
        n = args.cpu_frames
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1, n))
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda f: oracle.sift_match_pair(L[f % B], R[f % B]), range(n)))
        dt = time.perf_counter() - t0
        n1 = min(4, n)
        t0 = time.perf_counter()
        for f in range(n1):
            oracle.sift_match_pair(L[f % B], R[f % B])
        dt1 = time.perf_counter() - t0
        cpu = {"value": n / dt, "unit": "stereo frames/s", "cores": threads, "kind": "port",
               "sample": f"{n} synthetic 1242x375 stereo pairs (first {n} of the GPU batch), SIFT x2 + stereo match, "
                         f"oracle/liboracle.so, one pair per thread, {threads} threads, {dt:.1f} s wall",
               "single_thread": {"value": n1 / dt1, "cores": 1, "sample": f"{n1} pairs, {dt1:.1f} s"}}

    if rank == 0:
        kp = np.mean([s[0] + s[1] for s in stats]) / 2
        st = np.mean([s[2] for s in stats])
        line = {
            "metric": "stereo frames/sec @1242x375 (SIFT detect+describe x2 + stereo matchFeatures)",
            "value": fps, "unit": "stereo frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "ms_per_64_frames": ms_per_step * 64 / B, "timed_runs": timed_runs, "h2d": h2d_line,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32 (i8 MFMA for exact descriptor dot products)", "data": "synthetic",
            "config": {"workload": "BASELINE configs[1]: SIFT detect+describe + BF match on 1242x375 synthetic stereo, "
                                   "~2k keypoints/image", "frames_per_step_per_gpu": B, "rows": ROWS, "cols": COLS,
                       "mean_keypoints_per_image": float(kp), "mean_stereo_matches": float(st),
                       "parallelism": f"frames sharded over {world} GPU(s)",
                       "process_group": dist.get_backend() if dist is not None else None},
            "roofline": roof,
            "cpu_baseline": cpu,
            "full_path": full,
            "large": large,
        }
        print(json.dumps(line), file=json_out, flush=True)
    if dist is not None:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
