set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD; OUT=$ROOT/gpurun_out/msd5; mkdir -p $OUT
timeout -k 10 280 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_build_sizes.py tests/test_gpu_refit.py tests/test_gpu_parity.py tests/test_gpu_00_configs.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 100 python tools/msd_pathology.py > $OUT/path_msd.log 2>&1 || exit 2
BM_MSD_MAX_N=0 timeout -k 10 100 python tools/msd_pathology.py > $OUT/path_lsd.log 2>&1 || exit 3
timeout -k 10 120 python tools/build_bench.py > $OUT/bench.log 2>&1 || exit 4
echo ok
