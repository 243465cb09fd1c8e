#!/bin/bash
# k_desc change on one box: the descriptor parity tests with the in-tree library, then the
# configs[1] bench line for the default library and each named variant (tools/variants/<name>).
#   bash tools/gpu_desc_ab.sh <tag> <variant>...
set -e
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sift_match.py tests/test_gpu_edge.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tests_$TAG.log
bash tools/variant_bench.sh "$@"
