cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/sw_$tag.json 2>gpurun_out/sw_$tag.err || exit 1; }
B="python bench.py --no-cpu --full-frames 0 --steps 20"
VO_LIBPATH=build/variants/ch1024/libvo.so timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_large.py tests/test_gpu_sift_match.py -x -q --timeout 180 --timeout-method thread > gpurun_out/tests_ch.log 2>&1 || { tail -30 gpurun_out/tests_ch.log; exit 1; }
VO_LIBPATH=build/variants/ch2048/libvo.so timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_large.py -x -q --timeout 180 --timeout-method thread >> gpurun_out/tests_ch.log 2>&1 || { tail -30 gpurun_out/tests_ch.log; exit 1; }
tail -1 gpurun_out/tests_ch.log
VO_LIBPATH=build/variants/ch1024/libvo.so run ch1024 $B
VO_LIBPATH=build/variants/ch2048/libvo.so run ch2048 $B
echo done
