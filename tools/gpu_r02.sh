#!/bin/bash
# round-2 GPU iteration: selected -m gpu tests, then the default bench (as the driver runs it),
# each step under its own time limit; stops at the first failure.
#   bash tools/gpu_r02.sh <tag> <pytest target...>
set -e
TAG=${1:-cur}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest "$@" -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
( time timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err ) 2> gpurun_out/bench_$TAG.time
cat gpurun_out/bench_$TAG.time
python3 - "$TAG" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/bench_{sys.argv[1]}.json"))
print("value", round(d["value"], 1), "ms/step", round(d["ms_per_step"], 3), "kp", d["config"]["mean_keypoints_per_image"])
f = d.get("full_path")
if f: print("full", json.dumps({k: f[k] for k in ("value", "frames", "frames_with_pose", "mean_keypoints_per_image", "mean_inliers", "landmark_rows", "accuracy", "render_s")}))
print("cpu", d.get("cpu_baseline"))
PY
