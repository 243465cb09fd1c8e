set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/base_probe > gpurun_out/base_probe_v10.txt 2>&1 || { cat gpurun_out/base_probe_v10.txt; exit 1; }
cat gpurun_out/base_probe_v10.txt
