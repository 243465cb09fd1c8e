#!/bin/bash
# kernel trace of 6 back-to-back batches (overlap analysis), a 1-vs-2-part concurrency check, and
# the 2-rank bench rehearsal on one GPU over gloo.  Each step under its own time limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/trace_$1; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o k -- python3 tools/prof_run.py 64 6 > $O/log 2>&1
python3 tools/overlap.py $(ls $O/*kernel_trace.csv $O/*/*kernel_trace.csv 2>/dev/null | head -1) "k_blur_stream<10, 0, 4>" "k_blur_stream<5, 5, 4>" "k_desc" > $O/overlap.txt
cat $O/overlap.txt
for c in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu --seq-frames 0 --large-batch 0 --concurrency $c > gpurun_out/conc_$c.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/conc_$c.json')); print('concurrency $c', round(d['value'],1), round(d['ms_per_step'],3))"
done
VO_BENCH_BACKEND=gloo VO_BENCH_SAME_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --seq-frames 600 --large-batch 0 --no-cpu > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err
python3 -c "
import json; d=json.load(open('gpurun_out/rehearse2.json')); f=d['full_path']
print('rehearsal n_gpus', d['n_gpus'], 'value', round(d['value'],1), 'seq', round(f['value'],1), f['frames'], f['frames_per_rank'], f['frames_with_pose'], f['landmark_rows'], f['accuracy']['ate_rmse_m'])"
