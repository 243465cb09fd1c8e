#!/bin/bash
# Kernel trace of the sequence leg alone (KITTI-00 trajectory, 1024 frames, no other legs) and its
# per-kernel totals, to see what the full per-frame path adds over SIFT + stereo matching.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/seqtrace_$1; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o k -- python3 bench.py --no-cpu --steps 3 --warmup 1 --large-batch 0 --seq-frames 1024 > $O/bench.json 2> $O/err.log
python3 - $O <<'PY'
import csv, glob, json, sys
o = sys.argv[1]
f = glob.glob(f"{o}/**/*kernel_stats.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "vo::" in r["Name"]]
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"libvo kernels total {tot / 1e6:.2f} ms")
for r in rows[:40]:
    print(f"{r['Name'].split('(')[0][:60]:60s} calls {int(r['Calls']):6d} total {float(r['TotalDurationNs'])/1e6:8.2f} ms  {float(r['Percentage']):5.1f}%")
d = json.load(open(f"{o}/bench.json"))
print("seq", round(d["full_path"]["value"], 1), "fps over", d["full_path"]["frames"])
PY
find $O -name "*kernel_trace.csv" -delete
