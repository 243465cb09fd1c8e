#!/bin/bash
# configs[1] bench line for the default library and each named variant (tools/variants/<name>)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in default "$@" default; do
  if [ $v = default ]; then unset VO_LIBPATH; else export VO_LIBPATH=$GRAFT_REPO_ROOT/tools/variants/$v/libvo.so; fi
  timeout -k 10 200 python bench.py --no-cpu --seq-frames 0 --large-batch 0 > gpurun_out/var_$v.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/var_$v.json')); r=d['roofline']; k=r['kernel_ms_per_step']; i=r['kernel_ms_per_step_isolated']
print('$v', round(d['value'],1), round(d['ms_per_step'],3), 'base', k['k_blur_base'], i['k_blur_base'], 'blur', k['k_blur_fused'], i['k_blur_fused'], 'desc', k['k_desc'], i['k_desc'], 'ext', k.get('k_ext_inner<3>', k.get('k_ext_stream<3>')), i.get('k_ext_inner<3>', i.get('k_ext_stream<3>')), 'orient', k['k_orient'], i['k_orient'], 'match', k.get('k_match_partial'), i.get('k_match_partial'), 'refine', k.get('k_refine'), i.get('k_refine'), 'small', k.get('k_blur_small'), i.get('k_blur_small'), 'outer', k.get('k_ext_outer'), i.get('k_ext_outer'))"
done
