#!/bin/bash
# Counter passes comparing blur variants (kernel-trace only; never with sys/runtime traces).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_blur${1:-}
mkdir -p $OUT
run() { timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/$1 -o p --pmc ${@:2} -- python3 tools/prof_run.py 32 2 > $OUT/$1.log 2>&1; }
run p1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES
run p2 FETCH_SIZE WRITE_SIZE
run p3 SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_BUSY_CYCLES
run p4 TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE
echo pmc-done
