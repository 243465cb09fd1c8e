#!/bin/bash
# Parity tests of a variant library (tools/variants/<name>) on the descriptor path, then the
# configs[1] A/B bench lines: default, each variant, default.
#   bash tools/gpu_variant_ab.sh <test-variant> <variant>...
set -e
TV=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VO_LIBPATH=$GRAFT_REPO_ROOT/tools/variants/$TV/libvo.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sift_match.py tests/test_gpu_edge.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$TV.log 2>&1 || { tail -30 gpurun_out/tests_$TV.log; exit 1; }
tail -1 gpurun_out/tests_$TV.log
bash tools/variant_bench.sh "$@"
