#!/bin/bash
# Sweep the number of sub-batches per call (vo_set_concurrency) on the bench line.
#   bash tools/sweep_conc.sh 2 3 4 ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/conc
for n in "$@"; do
  timeout -k 10 200 python3 bench.py --no-cpu --full-frames 0 --large-batch 0 --concurrency $n > gpurun_out/conc/c$n.json 2> gpurun_out/conc/c$n.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/conc/c$n.json')); print('parts', $n, '|', round(d['value'],1), round(d['ms_per_step'],3))"
done
