"""Divergence of the deterministic spec (oracle/liboracle.so, = libvo bit for bit) from the
OpenCV-literal float SIFT + MATLAB-literal float matcher (oracle/liboracle_cv.so): the
measurement behind tests/test_spec_divergence.py and DESIGN.md §3.8.  Test infrastructure."""
from __future__ import annotations

import numpy as np


def _ang_diff(a, b):
    d = np.abs(a - b) % 360.0
    return np.minimum(d, 360.0 - d)


def match_keypoints(ks, kc, ang_tol: float = 2.0):
    """spec keypoint i <-> cv keypoint j: same x, y, octave, layer (bitwise: the pyramid and
    the refinement are shared) and orientation within ang_tol degrees.  -> (idx_s, idx_c)."""
    from collections import defaultdict
    buckets = defaultdict(list)
    for j, k in enumerate(kc):
        buckets[(float(k["x"]), float(k["y"]), int(k["octave"]), int(k["layer"]))].append(j)
    used = np.zeros(len(kc), bool)
    si, ci = [], []
    for i, k in enumerate(ks):
        best, bd = -1, ang_tol
        for j in buckets.get((float(k["x"]), float(k["y"]), int(k["octave"]), int(k["layer"])), ()):
            if used[j]:
                continue
            d = _ang_diff(float(k["angle"]), float(kc[j]["angle"]))
            if d <= bd:
                best, bd = j, d
        if best >= 0:
            used[best] = True
            si.append(i)
            ci.append(best)
    return np.array(si, np.int64), np.array(ci, np.int64)


def image_divergence(oracle, img):
    ks, ds = oracle.sift(img)
    kc, dc = oracle.sift(img, cv=True)
    si, ci = match_keypoints(ks, kc)
    agree = len(si) / max(len(ks), len(kc), 1)
    # the spec keeps exact duplicates (same x, y, octave, layer, angle) that OpenCV's
    # removeDuplicatedSorted drops: agreement net of that one documented difference
    uniq = len({(float(k["x"]), float(k["y"]), int(k["octave"]), int(k["layer"]), float(k["angle"])) for k in ks})
    agree_dedup = len(si) / max(uniq, len(kc), 1)
    diff = np.abs(ds[si].astype(np.int32) - dc[ci].astype(np.int32)).max(axis=1) if len(si) else np.zeros(1)
    return {"n_spec": len(ks), "n_spec_unique": uniq, "n_cv": len(kc), "agreement": agree,
            "agreement_dedup": agree_dedup, "cv_unmatched": len(kc) - len(ci),
            "desc_linf_max": int(diff.max()), "desc_linf_p99": float(np.percentile(diff, 99)),
            "desc_linf_mean": float(diff.mean())}, (ks, ds, kc, dc, si, ci)


def pair_divergence(oracle, left, right):
    """keypoints, descriptors and stereo matches of one pair under both implementations."""
    a, (ksl, dsl, kcl, dcl, sil, cil) = image_divergence(oracle, left)
    b, (ksr, dsr, kcr, dcr, sir, cir) = image_divergence(oracle, right)
    ps = oracle.match(dsl, dsr)
    pc = oracle.match(dcl, dcr, cv=True)
    # cv pairs in spec indices (pairs whose keypoints have no spec counterpart stay distinct)
    mapl = {int(c): int(s) for s, c in zip(sil, cil)}
    mapr = {int(c): int(s) for s, c in zip(sir, cir)}
    S = {(int(i) - 1, int(j) - 1) for i, j in ps}
    Cset = {(mapl.get(int(i) - 1, -1 - int(i)), mapr.get(int(j) - 1, -1 - int(j))) for i, j in pc}
    jac = len(S & Cset) / max(len(S | Cset), 1)
    return {"left": a, "right": b, "n_match_spec": len(ps), "n_match_cv": len(pc), "match_jaccard": jac}


def sequence_divergence(oracle, L, R, P1, P2, gt=None):
    """World poses of the VO.m loop under both implementations: max translation / rotation gap
    (and, with the rendered ground truth gt [n, 4, 4], each one's max position error)."""
    os_, _ = oracle.run_sequence(L, R, P1, P2)
    oc, _ = oracle.run_sequence(L, R, P1, P2, cv=True)
    dt = np.linalg.norm(os_["pose"][:, :3, 3] - oc["pose"][:, :3, 3], axis=1)
    Rrel = np.einsum("nji,njk->nik", os_["pose"][:, :3, :3], oc["pose"][:, :3, :3])
    ang = np.degrees(np.arccos(np.clip((np.trace(Rrel, axis1=1, axis2=2) - 1) / 2, -1, 1)))
    step = np.linalg.norm(np.diff(os_["pose"][:, :3, 3], axis=0), axis=1)
    return {"frames": len(L), "max_translation_gap_m": float(dt.max()), "max_rotation_gap_deg": float(ang.max()),
            "path_length_m": float(step.sum()), "status_spec": os_["status"].tolist(), "status_cv": oc["status"].tolist(),
            **({} if gt is None else {
                "max_error_spec_m": float(np.linalg.norm(os_["pose"][:, :3, 3] - (np.linalg.inv(gt[0]) @ gt)[:, :3, 3], axis=1).max()),
                "max_error_cv_m": float(np.linalg.norm(oc["pose"][:, :3, 3] - (np.linalg.inv(gt[0]) @ gt)[:, :3, 3], axis=1).max())})}
