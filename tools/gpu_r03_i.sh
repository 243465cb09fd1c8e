#!/bin/bash
# Round 3: lazy chunked MSAC (k_msac).  Geometry parity (incl. lazy vs eager vs oracle), the
# sequence tests, then the bench line with the full path.  Each step bounded.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_geometry.py tests/test_gpu_kitti.py tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread > $O/geom.log 2>&1 || { tail -40 $O/geom.log; exit 1; }
tail -1 $O/geom.log
timeout -k 10 600 python3 bench.py --no-cpu --large-batch 0 > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));f=d['full_path'];print(d['value'],d['ms_per_step']);print('full',f['value'],f['geometry_ms_per_step'],f['msac_score_roofline']['ms'],f['msac_score_roofline']['frac'], f['landmark_rows'], f['accuracy']['lagged_xz_error_m'])"
