#!/bin/bash
# full path (configs[2]) at several --seq-batch values, one bench line each (run through gpurun)
#   bash tools/seqdepth.sh <outdir> [batch...]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?outdir}; shift; mkdir -p $O
for sb in ${@:-64 256}; do
  timeout -k 10 300 python3 bench.py --no-cpu --large-batch 0 --runs 3 --seq-batch $sb > $O/seq_$sb.json 2> $O/seq_$sb.err || { tail -20 $O/seq_$sb.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/seq_$sb.json'));f=d['full_path'];print('seq-batch',$sb,'configs1',round(d['value']),'full',round(f['value']),round(f['value']/d['value'],3),f['landmark_rows'],round(f['accuracy']['ate_rmse_m'],4),f['per_rank_ms'][0]['loop'])"
done
