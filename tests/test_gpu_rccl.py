"""RCCL on the hardware: a real `nccl` (= RCCL) process group on the GPU,
world size 1, env rendezvous on 127.0.0.1 -- the branch bench.py's ranks take -- runs the
sharded sequence path with its collectives on device tensors (kitti.finish_shard: the records
all-gather, the gather of device-transformed world rows to rank 0) and the max-over-ranks
all-reduce; the gathered
trajectory (VO.m:130-134) and landmark map (CreateLandmarksFromFeatures.m:17) equal a plain
single-process libvo run bit for bit.  The rank runs in a child process (tests/rccl_rank.py)
so that the process group is created before any other GPU work, as in bench.py."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_world1_sharded_path_equals_single_process():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, "-u", str(ROOT / "tests" / "rccl_rank.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert line, p.stdout[-2000:] + p.stderr[-2000:]
    r = json.loads(line[-1])
    assert r["backend"] == "nccl" and r["world"] == 1
    for k in ("poses_equal", "rel_equal", "status_equal", "n_landmarks_equal", "landmarks_equal"):
        assert r[k], (k, r)
    assert r["frames_with_pose"] == r["frames"] - 1 and r["landmark_rows"] > 0
    assert r["max_over_ranks"] == 0.25
