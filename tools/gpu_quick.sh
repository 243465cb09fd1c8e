#!/bin/bash
# Kernel iteration on the GPU: selected -m gpu tests, a configs[1]-only bench line (no sequence,
# large or CPU legs), then optionally one LDS/VALU counter pass over the same workload.
#   bash tools/gpu_quick.sh <tag> [pmc] -- <pytest targets...>
set -e
TAG=$1; shift
PMC=0; if [ "$1" = "pmc" ]; then PMC=1; shift; fi
[ "$1" = "--" ] && shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
  tail -1 gpurun_out/tests_$TAG.log
fi
timeout -k 10 300 python bench.py --no-cpu --seq-frames 0 --large-batch 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
python3 - "$TAG" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/bench_{sys.argv[1]}.json"))
r = d["roofline"]
print("value", round(d["value"], 1), "ms/step", round(d["ms_per_step"], 3), "kp", round(d["config"]["mean_keypoints_per_image"], 1))
print("insitu", r["kernel_ms_per_step"])
print("iso", r["kernel_ms_per_step_isolated"])
PY
if [ $PMC = 1 ]; then
  OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o p --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -- python3 tools/prof_run.py 64 2 > $OUT/p1.log 2>&1
  python3 tools/pmc_sum.py $OUT/p1
fi
