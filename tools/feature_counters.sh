#!/bin/bash
# Where the feature-stream kernels (k_desc, k_orient) and the scale space spend their cycles:
# two separate counter passes over tools/prof_run.py (3 batches of the bench workload).
#   bash tools/feature_counters.sh <tag>   -> gpurun_out/fc_<tag>/{a,b}, summary in fc_<tag>/sum.txt
set -e
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/fc_$TAG; mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/a -o p --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_INST_LEVEL_VMEM -- python3 tools/prof_run.py 64 2 > $OUT/a.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/b -o p --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM_RD -- python3 tools/prof_run.py 64 2 > $OUT/b.log 2>&1
python3 tools/pmc_sum.py $OUT/a > $OUT/sum.txt
python3 tools/pmc_sum.py $OUT/b >> $OUT/sum.txt
cat $OUT/sum.txt
