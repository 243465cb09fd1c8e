#!/usr/bin/env python3
"""In-situ resource model of the pipelined step (VERDICT r3 "next" 1).

rocprofv3 collects counters per dispatch with the dispatches serialised, so the counters of a
kernel are known only in isolation; its in-situ duration comes from a kernel trace of the same
asynchronous loop.  This tool spreads each launch's counter totals (tools/pmc_passes.sh: HBM
bytes, VALU / LDS / VMEM wave instructions) uniformly over the launch's in-situ interval and sums
the rates of all kernels running at each instant.  The time-weighted result says which resource
the two overlapping streams keep saturated.

    python3 tools/insitu_model.py <pmc dir> <kernel_trace.csv> [out.json]

Rates are priced against: HBM 5.3 TB/s (tools/mallprobe.hip beyond the MALL) and 8 TB/s (peak);
VALU 1024 SIMDs x 2.4 GHz, 2 cycles per wave64 instruction; LDS 256 CUs x 2.4 GHz, 2 cycles per
wave64 instruction (32 lanes/clk); vector memory (TA) 256 CUs x 2.4 GHz, 4 cycles per wave64
instruction (16 lanes/clk).  The uniform-rate assumption smooths bursts inside a launch, so the
shares are lower bounds on the peaks and fair figures for the averages."""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import libvo_name  # noqa: E402

CLK = 2.4e9
CAP = {"valu": 1024 * CLK / 2, "lds": 256 * CLK / 2, "vmem": 256 * CLK / 4}
SCALE = ("k_blur_base", "k_blur_fused", "k_blur_small", "k_base_src<true>")


def launch_key(r):
    """(kernel symbol, grid size): one symbol serves several octaves; the grid tells them apart"""
    if r.get("Grid_Size"):
        g = int(float(r["Grid_Size"]))                     # counter CSV: total work-items
    else:
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    return (r["Kernel_Name"], g)


def counters(pmc_dir):
    """per launch key: average counter value per dispatch"""
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    for f in glob.glob(f"{pmc_dir}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if libvo_name(r["Kernel_Name"]) is None:
                continue
            n = launch_key(r)
            tot[n][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[n][r["Counter_Name"]].add(r["Dispatch_Id"])
    avg = {}
    for n, c in tot.items():
        avg[n] = {k: v / max(len(disp[n][k]), 1) for k, v in c.items()}
    return avg


def main():
    pmc_dir, trace = sys.argv[1], sys.argv[2]
    c = counters(pmc_dir)
    per = {}
    for n, v in c.items():
        per[n] = {
            "hbm": v.get("FETCH_SIZE", 0) * 2048 + v.get("WRITE_SIZE", 0) * 1024,   # KiB; gfx950 FETCH x2
            "valu": v.get("SQ_INSTS_VALU", 0),
            "lds": v.get("SQ_INSTS_LDS", 0),
            "vmem": v.get("SQ_INSTS_VMEM_RD", 0) + v.get("SQ_INSTS_VMEM_WR", 0),
        }
    ev = []
    missing = set()
    for r in csv.DictReader(open(trace)):
        if libvo_name(r["Kernel_Name"]) is None:
            continue
        n = launch_key(r)
        if n not in per:
            missing.add(n)
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e > s:
            ev.append((s, e, n))
    if missing:
        print("no counters for", sorted(missing)[:5], file=sys.stderr)
    ev.sort()
    # skip the first quarter of the trace (pipeline fill) and the last launch's drain
    t0 = ev[0][0] + (ev[-1][1] - ev[0][0]) // 4
    t1 = max(e for _, e, _ in ev)
    pts = sorted({t for s, e, _ in ev for t in (s, e) if t0 <= t <= t1} | {t0, t1})
    keys = ("hbm", "valu", "lds", "vmem")
    acc = {k: 0.0 for k in keys}
    share = {"hbm_over_4.5TBs": 0.0, "hbm_over_5.3TBs": 0.0, "valu_over_50pct": 0.0,
             "both_streams": 0.0, "scale_only": 0.0, "feature_only": 0.0, "idle": 0.0}
    hist = defaultdict(float)
    low = defaultdict(float)                 # kernels live while the summed HBM demand is < 3 TB/s
    low_t = 0.0
    low_acc = {"valu": 0.0, "lds": 0.0, "vmem": 0.0, "hbm": 0.0}
    for a, b in zip(pts, pts[1:]):
        dt = (b - a) * 1e-9
        if dt <= 0:
            continue
        live = [(s, e, n) for s, e, n in ev if s <= a and e >= b]
        rate = {k: sum(per[n][k] / ((e - s) * 1e-9) for s, e, n in live) for k in keys}
        for k in keys:
            acc[k] += rate[k] * dt
        sc = any(libvo_name(n[0]) in SCALE for _, _, n in live)
        ft = any(libvo_name(n[0]) not in SCALE for _, _, n in live)
        share["both_streams" if sc and ft else "scale_only" if sc else "feature_only" if ft else "idle"] += dt
        share["hbm_over_4.5TBs"] += dt * (rate["hbm"] > 4.5e12)
        share["hbm_over_5.3TBs"] += dt * (rate["hbm"] > 5.3e12)
        share["valu_over_50pct"] += dt * (rate["valu"] / CAP["valu"] > 0.5)
        hist[min(int(rate["hbm"] / 1e12), 7)] += dt
        if rate["hbm"] < 3e12:
            low_t += dt
            for k in low_acc:
                low_acc[k] += rate[k] * dt
            for combo in {libvo_name(n[0]) for _, _, n in live}:
                low[combo] += dt
    T = (t1 - t0) * 1e-9
    out = {
        "window_ms": T * 1e3,
        "mean": {"hbm_TBs": acc["hbm"] / T / 1e12, "valu_util": acc["valu"] / T / CAP["valu"],
                 "lds_util": acc["lds"] / T / CAP["lds"], "vmem_ta_util": acc["vmem"] / T / CAP["vmem"]},
        "time_share": {k: v / T for k, v in share.items()},
        "hbm_demand_histogram_TBs": {f"{k}-{k + 1}": v / T for k, v in sorted(hist.items())},
        "below_3TBs": {"time_share": low_t / T,
                       "mean": {"hbm_TBs": low_acc["hbm"] / max(low_t, 1e-12) / 1e12,
                                "valu_util": low_acc["valu"] / max(low_t, 1e-12) / CAP["valu"],
                                "lds_util": low_acc["lds"] / max(low_t, 1e-12) / CAP["lds"],
                                "vmem_ta_util": low_acc["vmem"] / max(low_t, 1e-12) / CAP["vmem"]},
                       "kernel_live_share": {k: v / max(low_t, 1e-12) for k, v in sorted(low.items(), key=lambda kv: -kv[1])}},
        "per_launch": {f"{libvo_name(k[0])} grid {k[1]}": v for k, v in per.items()},
        "assumptions": __doc__.split("Rates are priced against: ")[1].strip(),
    }
    txt = json.dumps(out, indent=1, sort_keys=True)
    if len(sys.argv) > 3:
        Path(sys.argv[3]).write_text(txt)
    m = out["mean"]
    print(f"window {out['window_ms']:.2f} ms  HBM {m['hbm_TBs']:.2f} TB/s  VALU {m['valu_util']:.2f}  "
          f"LDS {m['lds_util']:.2f}  TA {m['vmem_ta_util']:.2f}")
    print("time share", {k: round(v, 3) for k, v in out["time_share"].items()})
    print("below 3 TB/s:", round(low_t / T, 3), "of the window;", {k: round(v, 2) for k, v in out["below_3TBs"]["mean"].items()},
          "live kernels:",
          {k: round(v, 2) for k, v in out["below_3TBs"]["kernel_live_share"].items()})
    print("HBM demand histogram", {k: round(v, 3) for k, v in out["hbm_demand_histogram_TBs"].items()})


if __name__ == "__main__":
    main()
