set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/tests_final.log 2>&1 || { tail -40 gpurun_out/tests_final.log; exit 1; }
tail -1 gpurun_out/tests_final.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1
tail -1 gpurun_out/smoke_final.log
timeout -k 10 600 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
python3 -c "import json;d=json.load(open('gpurun_out/bench_final.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['full_path']['value'],d['large']['value'])"
