#!/bin/bash
# Counter passes (each its own rocprofv3 run, kernel-trace only; never combined with sys/runtime traces).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o p --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -- python3 tools/prof_run.py 16 2 > $OUT/p1.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 -o p --pmc FETCH_SIZE GRBM_GUI_ACTIVE -- python3 tools/prof_run.py 16 2 > $OUT/p2.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p3 -o p --pmc WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_UNALIGNED_STALL -- python3 tools/prof_run.py 16 2 > $OUT/p3.log 2>&1
echo pmc-done
