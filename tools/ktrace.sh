#!/bin/bash
# Kernel-trace pass (no counters): per-launch durations for the bench workload.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ktrace${1:-}
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o k -- python3 tools/prof_run.py 64 2 > $OUT/log 2>&1
echo ktrace-done
