#!/bin/bash
# Match-kernel A/B: parity tests (match ties, SIFT+match) per variant, then bench lines with the
# 1920x1080 leg (configs[4], where the dense match block is largest).   bash tools/gpu_match_ab.sh v1 v2 ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in default "$@"; do
  if [ $v = default ]; then unset VO_LIBPATH; else export VO_LIBPATH=$GRAFT_REPO_ROOT/tools/variants/$v/libvo.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_sift_match.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/mtests_$v.log 2>&1 || { echo "$v tests failed"; tail -30 gpurun_out/mtests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/mtests_$v.log)"
done
for v in default "$@" default; do
  if [ $v = default ]; then unset VO_LIBPATH; else export VO_LIBPATH=$GRAFT_REPO_ROOT/tools/variants/$v/libvo.so; fi
  timeout -k 10 300 python bench.py --no-cpu --seq-frames 0 > gpurun_out/mvar_$v.json 2>/dev/null || { echo "$v bench failed"; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/mvar_$v.json')); r=d['roofline']; k=r['kernel_ms_per_step']; i=r['kernel_ms_per_step_isolated']; L=d['large']
print('$v', round(d['value'],1), round(d['ms_per_step'],3), 'match', k['k_match_partial'], i['k_match_partial'], 'large', round(L['value'],1), L['match_block']['ms_per_step'], round(L['match_block']['frac'],4))"
done
