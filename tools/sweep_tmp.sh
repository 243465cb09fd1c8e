cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/sw_$tag.json 2>gpurun_out/sw_$tag.err || exit 1; }
B="python bench.py --no-cpu --full-frames 0 --large-batch 0 --steps 20"
run c0 $B
VO_OCT0_CHUNK=4 run c4 $B
VO_OCT0_CHUNK=8 run c8 $B
VO_OCT0_CHUNK=16 run c16 $B
VO_OCT0_CHUNK=8 VO_BLUR_TH=64 run c8t64 $B
VO_OCT0_CHUNK=8 VO_BLUR_WAVES=512 run c8w512 $B
echo done
