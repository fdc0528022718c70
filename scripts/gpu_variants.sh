#!/bin/bash
# bench config C against several prebuilt library variants (build/<name>), one line each
mkdir -p gpurun_out
for d in "$@"; do
  VIBA_LIB_DIR=build/$d timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/var_$d.json 2> gpurun_out/var_$d.log || exit $?
  echo "$d: $(grep timed gpurun_out/var_$d.log | sed 's/.*last it: //') | $(python -c "import json;r=json.load(open('gpurun_out/var_$d.json'))['roofline'];print(r['achieved'],r['unit'])")"
done
