#!/bin/bash
# Measurement bundle for profiles/: bench line (with CPU baseline), kernel-trace stats
# of the bench command, and the PMC traffic passes.  Run on the GPU box:
#   bash tools/profile_round.sh <tag>      -> gpurun_out/prof_<tag>/...
set -e
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o k -- python3 bench.py --steps 10 --warmup 2 --no-cpu --seq-frames 0 --large-batch 0 > $OUT/ktrace.log 2>&1
bash tools/pmc_passes.sh _$TAG
python3 tools/pmc_traffic.py gpurun_out/pmc_$TAG $OUT/pmc_traffic.json
echo profile-done
