#!/bin/bash
# Counter passes (each its own rocprofv3 run, kernel-trace only; never combined with sys/runtime traces).
# FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950.  Batch = bench.py's default (PMC_BATCH, 256).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc${1:-}
mkdir -p $OUT
run() { timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/$1 -o p --pmc ${@:2} -- python3 tools/prof_run.py ${PMC_BATCH:-256} 2 > $OUT/$1.log 2>&1; }
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS
run p2 FETCH_SIZE
run p3 WRITE_SIZE
run p4 SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
echo pmc-done
