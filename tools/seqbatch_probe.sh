# full path (configs[2]) throughput vs frames per vo_step_submit_dev call (bench.py --seq-batch), one box
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sb
for b in ${@:-64 128 64}; do
  timeout -k 10 300 python3 bench.py --no-cpu --large-batch 0 --runs 1 --steps 5 --seq-batch $b > gpurun_out/sb/b$b.json 2> gpurun_out/sb/b$b.err
  python3 -c "import json;d=json.load(open('gpurun_out/sb/b$b.json'));f=d['full_path'];print($b, round(f['value'],1), f['tail_ms'], f['frames_with_pose'], f['accuracy']['ate_rmse_m'])"
done
