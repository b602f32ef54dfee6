set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD; OUT=$ROOT/gpurun_out/gtpt; mkdir -p $OUT
timeout -k 10 280 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_build_sizes.py tests/test_gpu_refit.py > $OUT/tests.log 2>&1 || exit 1
BM_GATHER_TPT2_N=0 timeout -k 10 250 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_build_sizes.py > $OUT/tests_t2.log 2>&1 || exit 1
for i in 1 2; do
BM_GATHER_TPT2_N=4000000000 timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy >> $OUT/t1.log 2>&1 || exit 3
BM_GATHER_TPT2_N=0 timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy >> $OUT/t2.log 2>&1 || exit 4
done
echo ok
