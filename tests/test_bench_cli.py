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


def test_pmc_traffic_only_from_this_trees_sources(tmp_path):
    """roofline.traffic comes from profiles/pmc_summary.json only when that summary was measured on the
    HIP sources this tree builds (its recorded sources digest): a summary of other code is reported as
    stale with traffic None, not passed off as this binary's bytes."""
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    from visual_inertial_bundle_adjustment_amd.build import sources_digest
    good = tmp_path / "good.json"
    good.write_text(json.dumps({"fanin_kernel": {"hbm_bytes_per_launch": 123.0},
                                "_meta": {"sources_sha256": sources_digest(), "commit": "abc"}}))
    t, prov = bench.pmc_traffic("fanin_kernel", str(good))
    assert t == 123.0 and prov["measured_at_commit"] == "abc" and prov["status"].startswith("measured")
    stale = tmp_path / "stale.json"
    stale.write_text(json.dumps({"fanin_kernel": {"hbm_bytes_per_launch": 123.0},
                                 "_meta": {"sources_sha256": "0" * 64, "commit": "old"}}))
    t, prov = bench.pmc_traffic("fanin_kernel", str(stale))
    assert t is None and prov["status"].startswith("stale")
