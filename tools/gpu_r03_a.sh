#!/bin/bash
# Round 3, first box: HBM probe with loads in flight, full-path attribution on identical frames,
# rocprofv3 kernel stats of the sequence bench, and the default bench line.  Each step bounded.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 180 ./tools/mallprobe > $O/mallprobe.txt 2>&1
echo mallprobe-done
timeout -k 10 400 python3 tools/fullpath_attr.py 1024 64 > $O/attr.json 2> $O/attr.err
echo attr-done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/seqprof -o k -- python3 bench.py --steps 5 --warmup 2 --no-cpu --large-batch 0 > $O/seqprof_bench.json 2> $O/seqprof.err
find $O/seqprof -name "*kernel_trace.csv" -delete
echo seqprof-done
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
echo bench-done
