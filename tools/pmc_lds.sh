#!/bin/bash
# LDS/VALU counter passes for the descriptor/orientation kernels (kernel-trace only, no sys/runtime traces).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_lds
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o p --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -- python3 tools/prof_run.py 32 2 > $OUT/p1.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 -o p --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -- python3 tools/prof_run.py 32 2 > $OUT/p2.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p3 -o p --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES -- python3 tools/prof_run.py 32 2 > $OUT/p3.log 2>&1
echo pmc-done
