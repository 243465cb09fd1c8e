#!/bin/bash
# Parity tests of every named variant library (tools/variants/<name>) on the keypoint/descriptor
# path, then the configs[1] A/B bench lines: default, each variant, default (one box).
#   bash tools/gpu_variants_ab.sh <variant>...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  VO_LIBPATH=$GRAFT_REPO_ROOT/tools/variants/$v/libvo.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sift_match.py tests/test_gpu_edge.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$v.log 2>&1 || { tail -30 gpurun_out/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/tests_$v.log)"
done
bash tools/variant_bench.sh "$@"
