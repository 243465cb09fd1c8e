#!/usr/bin/env python3
"""Per-launch HBM traffic of libvo kernels from rocprofv3 counter passes.

Reads the FETCH_SIZE pass (p2) and WRITE_SIZE pass (p3) written by
tools/pmc_passes.sh and writes a JSON summary keyed by the libvo profiler
names bench.py reports.  Corrections per MI355X_MICROARCH.md (HBM/rocprofv3):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the
bytes of wide streaming reads, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane streaming stores.

usage: tools/pmc_traffic.py gpurun_out/pmc_<tag> profiles/<round>_pmc_traffic.json
"""
import csv
import json
import re
import sys
from collections import defaultdict

# rocprofv3 kernel symbol -> libvo profiler name (bench.py roofline keys)
RULES = [
    (r"k_blur_stream<\d+, [15](, \d+)?>", "k_blur_base"),
    (r"k_blur_stream<\d+, [02](, \d+)?>", "k_blur_fused"),
    (r"k_blur_pipe<", "k_blur_fused"),
    (r"k_small_pyr", "k_blur_small"),
    (r"k_base_src<true>", "k_base_src<true>"),
    (r"k_ext_stream<(\d)>", r"k_ext_stream<\1>"),
    (r"k_ext_inner<(\d)>", r"k_ext_inner<\1>"),
    (r"vo::(k_\w+)", r"\1"),
]


def libvo_name(sym):
    for pat, rep in RULES:
        m = re.search(pat, sym)
        if m:
            return m.expand(rep)
    return None


def load(path, counter):
    per = defaultdict(float)      # dispatch id -> value
    name = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        d = r["Dispatch_Id"]
        per[d] += float(r["Counter_Value"])
        name[d] = r["Kernel_Name"]
    return per, name


def main(src, dst):
    fetch, fname = load(f"{src}/p2/p_counter_collection.csv", "FETCH_SIZE")
    write, wname = load(f"{src}/p3/p_counter_collection.csv", "WRITE_SIZE")
    out = defaultdict(lambda: {"launches_fetch": 0, "launches_write": 0, "fetch_bytes": 0.0, "write_bytes": 0.0})
    for d, v in fetch.items():
        n = libvo_name(fname[d])
        if n:
            out[n]["launches_fetch"] += 1
            out[n]["fetch_bytes"] += 2.0 * v * 1024.0
    for d, v in write.items():
        n = libvo_name(wname[d])
        if n:
            out[n]["launches_write"] += 1
            out[n]["write_bytes"] += v * 1024.0
    res = {}
    for n, e in out.items():
        lf, lw = max(e["launches_fetch"], 1), max(e["launches_write"], 1)
        res[n] = {"fetch_bytes_per_launch": e["fetch_bytes"] / lf, "write_bytes_per_launch": e["write_bytes"] / lw,
                  "hbm_bytes_per_launch": e["fetch_bytes"] / lf + e["write_bytes"] / lw,
                  "launches": e["launches_fetch"]}
    json.dump({"source": src, "correction": "FETCH_SIZE x2 (gfx950), KiB -> bytes", "kernels": res},
              open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e6, 1) for k, v in sorted(res.items())}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
