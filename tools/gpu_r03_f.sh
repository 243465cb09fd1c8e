#!/bin/bash
# Round 3: next-octave base from the level-3 blur's store path (no k_down), 2-D k_small_pyr.
# Parity first, the GPU suite, the bench line, then the multi-rank rehearsal (2 gloo ranks on
# the one GPU) against the N=1 sequence leg.  Each step bounded; stop at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_sift_match.py -x -v --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python3 bench.py --no-cpu > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];f=d['full_path'];print(d['value'],d['ms_per_step'],r['kernel'],r['frac']);print(r['kernel_ms_per_step_isolated']);print('full',f['value']);print('large',d['large']['value'])"
timeout -k 10 300 python3 bench.py --seq-frames 4541 --large-batch 0 --no-cpu > $O/seq_n1.json 2> $O/seq_n1.err
echo n1-done
VO_BENCH_BACKEND=gloo VO_BENCH_SAME_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --seq-frames 4541 --large-batch 0 --no-cpu > $O/seq_n2_gloo_same_gpu.json 2> $O/seq_n2.err
python3 - <<PY
import json
a=json.load(open("$O/seq_n1.json"))["full_path"]; b=json.load(open("$O/seq_n2_gloo_same_gpu.json"))["full_path"]
print("n1", a["value"], a["landmark_rows"], a["accuracy"]); print("n2", b["value"], b["landmark_rows"], b["accuracy"])
print("equal", a["landmark_rows"] == b["landmark_rows"] and a["accuracy"] == b["accuracy"])
PY
