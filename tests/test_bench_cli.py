"""bench.py's command line on the CPU (no GPU call is reached)."""
from __future__ import annotations

import os


def test_bench_rejects_gpus_not_world_size():
    """--gpus N under a launcher whose WORLD_SIZE differs is an error (exit 2), before any GPU work."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], cwd=root, env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 2, out.stderr[-2000:]
