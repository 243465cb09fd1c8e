cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/tests_th128.log 2>&1 || { tail -20 gpurun_out/tests_th128.log; exit 1; }
tail -1 gpurun_out/tests_th128.log
run() { tag=$1; shift; timeout -k 10 120 "$@" > gpurun_out/sw_$tag.json 2>/dev/null || exit 1; }
B="python bench.py --no-cpu --full-frames 0 --large-batch 0 --steps 30"
run base $B
VO_LIBPATH=tools/variants/ext60/libvo.so run ext60 $B
VO_LIBPATH=tools/variants/ext90/libvo.so run ext90 $B
run c3 $B --concurrency 3
run c4 $B --concurrency 4
run b48 $B --batch 48
run b64 $B --batch 64
run b64c4 $B --batch 64 --concurrency 4
echo done
