set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VO_LIBPATH=$GRAFT_REPO_ROOT/tools/variants/cu4x/libvo.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sift_match.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_cu4x.log 2>&1 || { tail -30 gpurun_out/tests_cu4x.log; exit 1; }
tail -1 gpurun_out/tests_cu4x.log
bash tools/variant_bench.sh cu4x cu3x cu5x cu4s
