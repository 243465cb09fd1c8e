"""bench.py's multi-GPU launcher (CPU): `bench.py --gpus N` without torchrun starts N
ranks itself (one process per GPU, rendezvous on 127.0.0.1) and rank 0 reports the world
size it ran with.  --dry-run stops after the rendezvous (gloo), so no GPU is needed."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.parametrize("n", [1, 2])
def test_bench_gpus_flag_starts_n_ranks(n):
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--dry-run"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert json.loads(lines[0])["n_gpus"] == n
