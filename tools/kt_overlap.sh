#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/kt1; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o k -- python3 tools/prof_run.py 64 6 > $O/trace.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/p1 -o p --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD -- python3 tools/prof_run.py 64 2 > $O/p1.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/p2 -o p --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES -- python3 tools/prof_run.py 64 2 > $O/p2.log 2>&1
echo done
