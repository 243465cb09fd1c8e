#!/bin/bash
# full path (configs[2]) for the default library and each named variant (tools/variants/<name>),
# default first and last:   bash tools/seq_ab.sh <outdir> <seq-batch> <variant>...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?outdir}; SB=${2:?batch}; shift 2; mkdir -p $O
for v in default "$@" default; do
  if [ $v = default ]; then unset VO_LIBPATH; else export VO_LIBPATH=$GRAFT_REPO_ROOT/tools/variants/$v/libvo.so; fi
  timeout -k 10 300 python3 bench.py --no-cpu --large-batch 0 --runs 3 --seq-batch $SB > $O/ab_$v.json 2> $O/ab_$v.err || { tail -5 $O/ab_$v.err; echo "$v failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$v.json'));f=d['full_path'];print('$v','configs1',round(d['value']),'full',round(f['value']),round(f['value']/d['value'],3),f['landmark_rows'],round(f['accuracy']['ate_rmse_m'],4))"
done
