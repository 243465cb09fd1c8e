cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/sw_$tag.json 2>gpurun_out/sw_$tag.err || exit 1; }
B="python bench.py --no-cpu --full-frames 0 --large-batch 0 --steps 20"
VO_BLUR_DMA=1 VO_LIBPATH=build/variants/d6/libvo.so run d6 $B
VO_BLUR_DMA=1 VO_LIBPATH=build/variants/d20/libvo.so run d20 $B
echo done
