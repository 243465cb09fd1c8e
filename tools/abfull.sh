#!/bin/bash
# configs[1] and the full path (--seq-frames, default 2304 = 9 submits of 256) for the default
# library and each named variant (tools/variants/<name>/libvo.so), default first and last
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?outdir}; shift; mkdir -p $O
for var in default "$@" default; do
  if [ $var = default ]; then unset VO_LIBPATH; else export VO_LIBPATH=$GRAFT_REPO_ROOT/tools/variants/$var/libvo.so; fi
  timeout -k 10 300 python3 bench.py --no-cpu --large-batch 0 --seq-frames ${SEQ:-2304} > $O/abf_$var.json 2> $O/abf_$var.err || { tail -5 $O/abf_$var.err; echo "$var failed"; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/abf_$var.json'));f=d['full_path'];k=f['kernel_ms_per_step'];r=d['roofline']['kernel_ms_per_step']
print('$var',round(d['value'],1),round(d['ms_per_step'],3),'full',round(f['value'],1),round(f['value']/d['value'],3),f['landmark_rows'],round(f['accuracy']['ate_rmse_m'],4),'blur',r.get('k_blur_fused'),k.get('k_blur_fused'),'refine',r.get('k_refine'),k.get('k_refine'))" | tee -a $O/abfull.txt
done
