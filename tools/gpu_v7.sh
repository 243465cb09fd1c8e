set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/tests_v7.log 2>&1 || { tail -40 gpurun_out/tests_v7.log; exit 1; }
tail -1 gpurun_out/tests_v7.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_v7.log 2>&1
tail -2 gpurun_out/smoke_v7.log
bash tools/profile_round.sh r02_v7
python3 -c "import json;d=json.load(open('gpurun_out/prof_r02_v7/bench.json'));print(d['value'],d['ms_per_step'],d['roofline'])"
timeout -k 10 120 ./tools/base_probe > gpurun_out/base_probe_v7.txt 2>&1
cat gpurun_out/base_probe_v7.txt
