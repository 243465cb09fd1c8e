#!/bin/bash
# Round 3, box 2: blocked-sweep HBM probe; kernel-trace timeline of the pipelined full path.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 240 ./tools/mallprobe > $O/mallprobe.txt 2>&1
echo mallprobe-done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o k -- python3 tools/seq_timeline.py 640 64 > $O/timeline.json 2> $O/timeline.err
python3 tools/timeline.py $(find $O/tl -name "*kernel_trace.csv" | head -1) > $O/timeline.txt
find $O/tl -name "*kernel_trace.csv" -delete
echo timeline-done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
