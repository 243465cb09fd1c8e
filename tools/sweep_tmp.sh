cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 200 "$@" > gpurun_out/sw_$tag.json 2>gpurun_out/sw_$tag.err || exit 1; }
B="python bench.py --no-cpu --full-frames 0 --large-batch 0 --steps 30"
run cc1 $B --concurrency 1
run cc2 $B --concurrency 2
run cc2b32 $B --concurrency 2 --batch 32
run cc1b32 $B --concurrency 1 --batch 32
echo done
