set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_match_ab.sh mpf1 mpf4b2 mpf8b2 any4b2
timeout -k 10 120 ./tools/base_probe > gpurun_out/base_probe_v9.txt 2>&1 || { cat gpurun_out/base_probe_v9.txt; exit 1; }
head -4 gpurun_out/base_probe_v9.txt
