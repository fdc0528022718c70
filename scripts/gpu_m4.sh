set -o pipefail
mkdir -p gpurun_out
VIBA_LIB_DIR=$GRAFT_REPO_ROOT/visual_inertial_bundle_adjustment_amd/lib_m4 timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -k "one_step or ordering or fused" > gpurun_out/m4_pytest.log 2>&1; tail -3 gpurun_out/m4_pytest.log
bash scripts/gpu_ab.sh m4 lib_m4 lib lib_m4 lib
