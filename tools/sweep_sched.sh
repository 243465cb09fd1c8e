#!/bin/bash
# Scheduling sweep: bench line (SIFT x2 + stereo match only) under stream-priority / feature-grid knobs.
#   bash tools/sweep_sched.sh "<ENV settings>" ...   (each argument one variant, e.g. "VO_SS_PRIO=1 VO_DESC_GRID=2048")
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sched
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 200 python3 bench.py --no-cpu --full-frames 0 --large-batch 0 --steps 20 --warmup 3 > gpurun_out/sched/b$i.json 2> gpurun_out/sched/b$i.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sched/b$i.json')); print(sys.argv[1], '|', round(d['value'],1), round(d['ms_per_step'],3), {k: v for k, v in list(d['roofline']['kernel_ms_per_step_isolated'].items())[:6]})" "$v"
done
