#!/bin/bash
# Round 3: k_octave (fused octave scale space + extremum test) and the packed landmark copy:
# parity first, then the whole GPU suite, then the bench.  Each step bounded; stop at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_sift_match.py -x -v --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python3 bench.py --no-cpu > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];f=d['full_path'];print(d['value'],d['ms_per_step'],r['kernel'],r['frac']);print(r['kernel_ms_per_step']);print(r['kernel_ms_per_step_isolated']);print('full',f['value'],f['kernel_ms_per_step']);print('large',d['large']['value'])"
