set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD; OUT=$ROOT/gpurun_out/kdfill; mkdir -p $OUT
timeout -k 10 280 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_reference_mode.py tests/test_gpu_hash.py tests/test_gpu_build_sizes.py tests/test_gpu_00_configs.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/ref_time.py c2 c5 > $OUT/ref.log 2>&1 || exit 2
echo ok
