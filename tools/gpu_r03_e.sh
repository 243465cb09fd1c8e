#!/bin/bash
# Round 3: per-level default path + packed landmark copy: parity (incl. the experimental k_octave
# path against the default), the whole GPU suite, full-path attribution, rocprofv3 kernel stats
# of the sequence bench, then the bench line.  Each step bounded; stop at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pyramid.py -x -v --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python3 tools/fullpath_attr.py 1024 64 > $O/attr.json 2> $O/attr.err
echo attr-done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/seqprof -o k -- python3 bench.py --steps 5 --warmup 2 --no-cpu --large-batch 0 > $O/seqprof_bench.json 2> $O/seqprof.err
find $O/seqprof -name "*kernel_trace.csv" -delete
echo seqprof-done
timeout -k 10 600 python3 bench.py --no-cpu > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];f=d['full_path'];print(d['value'],d['ms_per_step'],r['kernel'],r['frac']);print(r['kernel_ms_per_step_isolated']);print('full',f['value'],f.get('kernel_ms_per_step'));print('large',d['large']['value'])"
