# configs[1] throughput vs frames per step (bench.py --batch), one box
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/bp
for b in ${@:-64 128 64}; do
  timeout -k 10 300 python3 bench.py --no-cpu --seq-frames 0 --large-batch 0 --runs 3 --batch $b > gpurun_out/bp/b$b.json 2> gpurun_out/bp/b$b.err
  python3 -c "import json;d=json.load(open('gpurun_out/bp/b$b.json'));print($b, round(d['value'],1), round(d['ms_per_step'],3), d['timed_runs'])"
done
