#!/bin/bash
# A/B of a libvo variant (tools/variants/<name>): its SIFT/match GPU parity tests, bench lines
# default/variant/default, and one LDS counter pass each.   bash tools/gpu_ab.sh <name> [pytest targets]
set -e
V=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${*:-tests/test_gpu_sift_match.py}
VO_LIBPATH=$GRAFT_REPO_ROOT/tools/variants/$V/libvo.so timeout -k 10 300 python -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$V.log 2>&1 || { tail -30 gpurun_out/tests_$V.log; exit 1; }
tail -1 gpurun_out/tests_$V.log
bash tools/variant_bench.sh $V
for v in default $V; do
  if [ $v = default ]; then unset VO_LIBPATH; else export VO_LIBPATH=$GRAFT_REPO_ROOT/tools/variants/$v/libvo.so; fi
  OUT=gpurun_out/pmc_ab_$v; mkdir -p $OUT
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT -o p --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -- python3 tools/prof_run.py 64 2 > $OUT.log 2>&1
  echo "== $v"; python3 tools/pmc_sum.py $OUT | grep -E 'k_desc|k_orient'
done
