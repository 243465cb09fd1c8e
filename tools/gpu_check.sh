#!/bin/bash
# GPU iteration helper: full -m gpu suite, then a bench line (no CPU leg).  Each step has its
# own time limit; the script stops at the first failure.
#   bash tools/gpu_check.sh <tag> [bench args...]
set -e
TAG=${1:-cur}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 400 python bench.py --no-cpu "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
python3 - "$TAG" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/bench_{sys.argv[1]}.json"))
print("value", round(d["value"], 1), "ms/step", round(d["ms_per_step"], 3))
print("iso", d["roofline"]["kernel_ms_per_step_isolated"])
if d.get("large"): print("large", round(d["large"]["value"], 1), d["large"]["match_block"]["frac"], d["large"]["kernel_ms_per_step"])
if d.get("full_path"): print("full", round(d["full_path"]["value"], 1))
PY
