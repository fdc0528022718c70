#!/bin/bash
# AddressSanitizer + UndefinedBehaviorSanitizer build of the CPU-side native code -- the oracle
# (oracle/refcpu.cpp), the synthetic generator (csrc/synth.cpp) and the session adapter's host code
# (csrc/session.cpp) -- and the CPU test suite run over it (host code only: the HIP library is the
# in-tree build, and no test in this suite calls into the GPU).
#
#     bash scripts/sanitize.sh [out_dir=/tmp/viba_san] [pytest args ...]
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-/tmp/viba_san}
shift || true
mkdir -p "$OUT/lib"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1"
CS=$R/visual_inertial_bundle_adjustment_amd/csrc
g++ $SAN -std=c++17 -fPIC -shared -o "$OUT/lib/libviba_synth.so" "$CS/synth.cpp" &
g++ $SAN -std=c++17 -fPIC -shared -o "$OUT/lib/libviba_host.so" "$CS/session.cpp" &
g++ $SAN -std=c++17 -march=x86-64-v3 -fopenmp -fPIC -shared -o "$OUT/librefcpu.so" "$R/oracle/refcpu.cpp" &
wait
for f in libviba_hip.so libviba_hip_mixed.so; do ln -sf "$R/visual_inertial_bundle_adjustment_amd/lib/$f" "$OUT/lib/$f"; done
# the ASan runtime must come first in the process (python itself is not instrumented), libstdc++ right
# after it (else ASan cannot resolve the real __cxa_throw for the oracle's exceptions); python's own
# allocations are not leak-checked
cd "$R"
VIBA_LIB_DIR="$OUT/lib" VIBA_ORACLE_LIB="$OUT/librefcpu.so" \
  LD_PRELOAD="$(g++ -print-file-name=libasan.so) $(g++ -print-file-name=libstdc++.so.6)" \
  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:detect_odr_violation=0 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider "$@"
