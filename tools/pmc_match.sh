#!/bin/bash
# Counter passes over k_match_partial on the 1920x1080 configuration (bench's large leg).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_match
mkdir -p $OUT
B="python3 bench.py --no-cpu --full-frames 0 --batch 2 --steps 2 --warmup 1 --large-batch 8 --profile-steps 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o p --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES -- $B > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 -o p --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY -- $B > $OUT/p2.log 2>&1
echo pmc-match-done
