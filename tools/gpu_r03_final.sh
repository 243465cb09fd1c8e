#!/bin/bash
# Round-3 evidence on one box: GPU suite, smoke, rocprofv3 kernel stats of the configs[1] bench,
# FETCH_SIZE / WRITE_SIZE counter passes (each its own run), the default bench line, then the
# rocprofv3 kernel stats of the full-path (sequence) bench.   bash tools/gpu_r03_final.sh [outdir]
# Every GPU step bounded; the script stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03final}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kprof -o k -- python3 bench.py --steps 10 --warmup 2 --no-cpu --seq-frames 0 --large-batch 0 > $O/kprof_bench.json 2> $O/kprof.err
find $O/kprof -name "*kernel_trace.csv" -delete
echo kprof-done
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/pmc/p2 -o p --pmc FETCH_SIZE -- python3 tools/prof_run.py 64 2 > $O/pmc_p2.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/pmc/p3 -o p --pmc WRITE_SIZE -- python3 tools/prof_run.py 64 2 > $O/pmc_p3.log 2>&1
python3 tools/pmc_traffic.py $O/pmc profiles/r03_pmc_traffic.json > $O/pmc_traffic.txt
cp profiles/r03_pmc_traffic.json $O/
find $O/pmc -name "*.csv" -size +4M -delete
echo pmc-done
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/seqprof -o s -- python3 bench.py --steps 5 --warmup 2 --no-cpu --large-batch 0 > $O/seqprof_bench.json 2> $O/seqprof.err
find $O/seqprof -name "*kernel_trace.csv" -delete
echo seqprof-done
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel'],r['frac'],r.get('traffic'));print('full',d['full_path']['value'],'large',d['large']['value'],'cpu',d['cpu_baseline']['value'])"
