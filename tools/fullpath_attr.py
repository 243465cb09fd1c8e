#!/usr/bin/env python3
"""Attribute the gap between BASELINE configs[1] (SIFT x2 + stereo match) and configs[2] (the
full per-frame path) on the SAME frames: N KITTI-00 street frames are rendered into HBM once,
then
  (a) configs[1]-style: vo_sift_match_batch_dev over them in batches of B, back to back;
  (b) the full path: the pipelined vo_step_submit_dev / vo_step_collect loop (bench.py's
      sequence leg, 2048 MSAC hypotheses) over the same frames;
  (c) per-kernel HIP-event times of (a) and (b) (profiling pass; collect syncs every stream),
      in ms per B frames;
  (d) (a) on the bench's synthetic 1242x375 pairs, for the keypoint-density difference;
  (e) the "content" factor per kernel: isolated (synchronised) per-kernel times of (a) on the
      street frames and on the synthetic pairs, with the keypoints' octave / layer mix and their
      descriptor-window size (sum of squared octave-relative scales, which k_desc's and k_orient's
      sample counts are proportional to) for one batch of each.
usage: python tools/fullpath_attr.py [frames=1024] [batch=64]  -> one JSON line on stdout"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import vo_amd  # noqa: E402,F401
from r7020e_visual_odometry_amd import vo, street, kitti, synthetic as syn  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
dev = torch.device("cuda", 0)
gt = street.kitti00_gt()[:N]
P0, P1 = street.kitti00_calib()
wld = street.kitti00_world(device="cuda:0", poses=street.kitti00_gt())
dL = torch.empty((N, street.KITTI_ROWS, street.KITTI_COLS), dtype=torch.uint8, device=dev)
dR = torch.empty_like(dL)
street.render_frames(wld, street.kitti00_gt(), range(N), P0, P1, out=(dL, dR))
del wld
torch.cuda.synchronize()
fs = street.KITTI_ROWS * street.KITTI_COLS
rp = vo.default_ransac_params()
rp.max_num_trials = 2048
ctx = vo.Context(street.KITTI_ROWS, street.KITTI_COLS, B, calib=vo.calib_from(P0, P1), ransac=rp)
nb = N // B


def sift_only():
    for b in range(nb):
        ctx.sift_match_batch_dev(dL.data_ptr() + b * B * fs, dR.data_ptr() + b * B * fs, B, stats=False)
    torch.cuda.synchronize()


def full():
    ctx.reset()
    return kitti._pipelined(ctx, kitti.device_batches(dL, dR, B, 0, nb * B), dev)


def timed(fn, reps=2):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def profiled(fn):
    ctx.set_profiling(True)
    fn()
    torch.cuda.synchronize()
    kt = ctx.kernel_times()
    ctx.set_profiling(False)
    return {k: round(v[0] / nb, 4) for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0])}


def iso_times(c, dl, dr, nrep=3):
    """(e): per-kernel times of synchronised calls (no overlap), ms per B frames."""
    c.set_profiling(True)
    for _ in range(nrep):
        c.sift_match_batch_dev(dl, dr, B, stats=True)
    torch.cuda.synchronize()
    kt = c.kernel_times()
    c.set_profiling(False)
    return {k: round(v[0] / nrep, 4) for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0])}


def kp_mix(c, dl, dr):
    """Octave / layer histogram and window-size sum of one batch's keypoints (all 2B images)."""
    st = c.sift_match_batch_dev(dl, dr, B, stats=True)
    octs, lays, w = [], [], 0.0
    for i in range(2 * B):
        k, _ = c.fetch_keypoints(i)
        octs += k["octave"].tolist()
        lays += k["layer"].tolist()
        s = k["scale"].astype(np.float64) / np.exp2(k["octave"].astype(np.float64))   # octave-relative scale
        w += float((s * s).sum())
    octs, lays = np.array(octs), np.array(lays)
    return {"keypoints_per_image": len(octs) / (2 * B), "stereo_matches_per_frame": float(np.mean([x[2] for x in st])),
            "octave_hist": {int(o): int((octs == o).sum()) for o in np.unique(octs)},
            "layer_hist": {int(l_): int((lays == l_).sum()) for l_ in np.unique(lays)},
            "mean_octave_rel_scale": float(np.sqrt(w / max(len(octs), 1))),
            "window_scl2_per_image": w / (2 * B)}


t_sift = timed(sift_only)
t_full = timed(full)
outs = np.concatenate(full())
kt_sift = profiled(sift_only)
kt_full = profiled(full)
st = ctx.sift_match_batch_dev(dL.data_ptr(), dR.data_ptr(), B, stats=True)
ctx.close()
# (d) the bench's synthetic pairs
L, R = syn.independent_pairs(B, 375, 1242, first=0, px_per_cell=syn.BENCH_PX_PER_CELL)
sl, sr = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
c2 = vo.Context(375, 1242, B)
st2 = c2.sift_match_batch_dev(sl.data_ptr(), sr.data_ptr(), B, stats=True)


def syn_only():
    for _ in range(nb):
        c2.sift_match_batch_dev(sl.data_ptr(), sr.data_ptr(), B, stats=False)
    torch.cuda.synchronize()


t_syn = timed(syn_only)
iso_syn = iso_times(c2, sl.data_ptr(), sr.data_ptr())
mix_syn = kp_mix(c2, sl.data_ptr(), sr.data_ptr())
c2.close()
c3 = vo.Context(street.KITTI_ROWS, street.KITTI_COLS, B)
iso_street = iso_times(c3, dL.data_ptr(), dR.data_ptr())
mix_street = kp_mix(c3, dL.data_ptr(), dR.data_ptr())
c3.close()
geom = {k: v for k, v in kt_full.items() if k not in kt_sift}
shared = {k: round(kt_full[k] - kt_sift[k], 4) for k in kt_sift if k in kt_full}
print(json.dumps({
    "frames": nb * B, "batch": B,
    "ms_per_batch": {"sift_match_street": t_sift / nb * 1e3, "full_path_street": t_full / nb * 1e3,
                     "sift_match_synthetic": t_syn / nb * 1e3},
    "fps": {"sift_match_street": nb * B / t_sift, "full_path_street": nb * B / t_full,
            "sift_match_synthetic": nb * B / t_syn},
    "keypoints_per_image": {"street": float(np.mean([s[0] + s[1] for s in st]) / 2),
                            "synthetic": float(np.mean([s[0] + s[1] for s in st2]) / 2)},
    "mean_tracked": float(outs["n_tracked"][1:].mean()), "mean_inliers": float(outs["n_inliers"][1:].mean()),
    "kernel_ms_per_batch": {"sift_match": kt_sift, "full_path": kt_full},
    "content": {"isolated_ms_per_batch": {"street": iso_street, "synthetic": iso_syn,
                                          "street_minus_synthetic": {k: round(iso_street[k] - iso_syn.get(k, 0.0), 4)
                                                                     for k in iso_street}},
                "keypoints": {"street": mix_street, "synthetic": mix_syn},
                "note": "street = the first B KITTI-00 frames at 376x1241, synthetic = the bench pairs at 375x1242"},
    "full_minus_sift": {"kernels_only_in_full_path": geom, "geometry_sum_ms": round(sum(geom.values()), 4),
                        "shared_kernels_delta_ms": shared},
}))
