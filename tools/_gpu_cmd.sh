set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD; OUT=$ROOT/gpurun_out/msdl; mkdir -p $OUT
timeout -k 10 280 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_build_sizes.py tests/test_gpu_refit.py > $OUT/tests.log 2>&1 || exit 1
BM_BS_CAP=0 timeout -k 10 250 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_build_sizes.py > $OUT/tests_g.log 2>&1 || exit 1
for i in 1 2; do
BM_MSD_LARGE=0 timeout -k 10 120 python tools/build_bench.py tyra_proxy,merged_proxy >> $OUT/lsd.log 2>&1 || exit 3
timeout -k 10 120 python tools/build_bench.py tyra_proxy,merged_proxy >> $OUT/msd.log 2>&1 || exit 4
done
echo ok
