#!/bin/bash
# configs[1] bench line of HEAD and of other revisions' whole trees (varlib/<rev>, each built in
# place), on one box:  bash tools/rev_ab.sh <outdir> <rev> [<rev> ...]   -> head, revs..., head
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?outdir}; shift; mkdir -p $O
for v in head "$@" head; do
  if [ $v = head ]; then D=$GRAFT_REPO_ROOT; else D=$GRAFT_REPO_ROOT/varlib/$v; fi
  (cd $D && timeout -k 10 240 python3 bench.py --no-cpu --seq-frames 0 --large-batch 0 > $GRAFT_REPO_ROOT/$O/ab_$v.json 2> $GRAFT_REPO_ROOT/$O/ab_$v.err) \
    || { tail -20 $O/ab_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/ab_$v.json')); r=d['roofline']; k=r['kernel_ms_per_step']; i=r['kernel_ms_per_step_isolated']
print('$v', round(d['value'],1), round(d['ms_per_step'],3), d['timed_runs']['ms_per_step'], 'blur', k['k_blur_fused'], i['k_blur_fused'], 'desc', k['k_desc'], i['k_desc'], 'ext', k.get('k_ext_inner<3>'), i.get('k_ext_inner<3>'), 'orient', k.get('k_orient'), i.get('k_orient'), 'refine', k.get('k_refine'), i.get('k_refine'))" | tee -a $O/ab.txt
done
