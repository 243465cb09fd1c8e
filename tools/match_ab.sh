#!/bin/bash
# configs[1] and the 1080p leg (configs[4]) for the default library and each named variant
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?outdir}; shift; mkdir -p $O
for v in default "$@" default; do
  if [ $v = default ]; then unset VO_LIBPATH; else export VO_LIBPATH=$GRAFT_REPO_ROOT/tools/variants/$v/libvo.so; fi
  timeout -k 10 400 python3 bench.py --no-cpu --seq-frames 0 --large-batch 64 --runs 3 > $O/m_$v.json 2> $O/m_$v.err || { tail -5 $O/m_$v.err; echo "$v failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/m_$v.json'));r=d['roofline'];k=r['kernel_ms_per_step'];i=r['kernel_ms_per_step_isolated'];l=d['large'];print('$v',round(d['value'],1),round(d['ms_per_step'],3),'match',k.get('k_match_partial'),i.get('k_match_partial'),'large',round(l['value'],1),'mb_frac',round(l['match_block']['frac'],4),'mb_ms',round(l['match_block']['ms_per_step'],3))"
done
