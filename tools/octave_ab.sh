#!/bin/bash
# configs[1] on the product library, then on the test build with the fused octave (k_octave) selected
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?outdir}; mkdir -p $O
for v in default octave default; do
  if [ $v = default ]; then
    timeout -k 10 300 python3 bench.py --no-cpu --seq-frames 0 --large-batch 0 --runs 3 > $O/oct_$v.json 2> $O/oct_$v.err || { tail -5 $O/oct_$v.err; exit 1; }
  else
    timeout -k 10 300 python3 tools/exp_bench.py 1 0 --no-cpu --seq-frames 0 --large-batch 0 --runs 3 > $O/oct_$v.json 2> $O/oct_$v.err || { tail -5 $O/oct_$v.err; exit 1; }
  fi
  python3 -c "import json;d=json.load(open('$O/oct_$v.json'));r=d['roofline'];k=r['kernel_ms_per_step'];print('$v',round(d['value'],1),round(d['ms_per_step'],3),{n:v for n,v in list(k.items())[:6]})"
done
