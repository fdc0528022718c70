#!/bin/bash
# streams + busy-time roofline: bench at 1 / 2 / 3 streams, rocprof trace of the default line (busy-union cross-check)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r05m
for n in 2 1 3; do
  VIBA_SN_STREAMS=$n timeout -k 10 300 python bench.py --no-cpu-baseline --no-banded-count > gpurun_out/bench_${T}_s$n.json 2> gpurun_out/bench_${T}_s$n.log || { tail -20 gpurun_out/bench_${T}_s$n.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_${T}_s$n.json').read().strip().splitlines()[-1]); r=d['roofline']; print('streams $n', round(d['value'],2), d['phases_ms']['factor_ms'], d['phases_ms']['total_ms'], 'busy/launch', round(r['busy_ms_per_launch'],4), 'avg', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],3), 'frac(per-launch avg)', round(r['frac_per_launch_duration'],3), 'launches/factor', r['fanin_launches_per_factorization'], 'busy/factor', round(r['busy_ms_per_factorization'],3))"
done
timeout -k 10 300 python scripts/kernel_probe.py C 5 fp64 12,13,14,20,21,22 > gpurun_out/probe_$T.json 2> gpurun_out/probe_$T.log || exit 1
cat gpurun_out/probe_$T.json
cd /tmp
(timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$T -o run -- python3 $R/bench.py --no-cpu-baseline --no-banded-count > $R/gpurun_out/bench_${T}_prof.json 2> $R/gpurun_out/bench_${T}_prof.log) || exit $?
cd $R
python scripts/busy_union.py gpurun_out/prof_$T/run_kernel_trace.csv fanin_kernel snpotrf sntrsm
python -c "import json; d=json.loads(open('gpurun_out/bench_${T}_prof.json').read().strip().splitlines()[-1]); r=d['roofline']; print('under rocprof', round(d['value'],2), 'busy/launch', round(r['busy_ms_per_launch'],4), 'avg', round(r['avg_launch_ms'],4))"
