set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/lb
for b in ${@:-32 64}; do
  timeout -k 10 300 python3 bench.py --no-cpu --seq-frames 0 --runs 1 --steps 6 --large-batch $b > gpurun_out/lb/b$b.json 2> gpurun_out/lb/b$b.err
  python3 -c "import json;d=json.load(open('gpurun_out/lb/b$b.json'));l=d['large'];print($b, round(l['value'],1), l['kernel_ms_per_step'])"
done
