#!/bin/bash
# k_octave wait-time statistics (diagnostic build: bash tools/build_variant.sh ostats -DOF_STATS)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03d; mkdir -p $O
VO_LIBPATH=tools/variants/ostats/libvo.so timeout -k 10 120 python3 tools/prof_run.py 64 2 > $O/stats.out 2> $O/stats.txt
grep "k_octave" $O/stats.txt | tail -2
