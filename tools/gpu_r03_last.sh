#!/bin/bash
# Short evidence pass on one box: GPU suite, smoke, rocprofv3 kernel stats of the configs[1]
# bench, the default bench line.   bash tools/gpu_r03_last.sh [outdir]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03last}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kprof -o k -- python3 bench.py --steps 10 --warmup 2 --no-cpu --seq-frames 0 --large-batch 0 > $O/kprof_bench.json 2> $O/kprof.err
find $O/kprof -name "*kernel_trace.csv" -delete
echo kprof-done
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel'],r['frac']);print('full',d['full_path']['value'],'large',d['large']['value'],'cpu',d['cpu_baseline']['value'])"
