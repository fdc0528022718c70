#!/bin/bash
# round-5 first check: symbolic statistics, the new and changed tests, the supernode factorization,
# default and supernode bench lines, then the multi-process tests
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v -s --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_session_gpu.py \
  "tests/test_parity_gpu.py::test_one_lm_step_matches_oracle" -m gpu > gpurun_out/pytest_r05a_new.log 2>&1 || { tail -40 gpurun_out/pytest_r05a_new.log; exit 1; }
grep -h "gradient entry errors\|supernode schedule" gpurun_out/pytest_r05a_new.log || true
timeout -k 10 600 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_r05a.json 2> gpurun_out/bench_r05a.log || exit $?
VIBA_SUPERNODE=1 timeout -k 10 600 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_r05a_sn.json 2> gpurun_out/bench_r05a_sn.log || exit $?
python - <<'PY'
import json
for t in ("", "_sn"):
    d = json.loads(open(f"gpurun_out/bench_r05a{t}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(t or "col", round(d["value"], 2), "ms", round(d["ms_per_step"], 2), "frac", round(r["frac"], 3), "launches/fact", r.get("fanin_launches_per_factorization"), d["phases_ms"])
PY
timeout -k 10 1500 $T tests/test_distributed_gpu.py -m gpu > gpurun_out/pytest_r05a_dist.log 2>&1 || { tail -40 gpurun_out/pytest_r05a_dist.log; exit 1; }
tail -3 gpurun_out/pytest_r05a_dist.log
