set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD; OUT=$ROOT/gpurun_out/lm2; mkdir -p $OUT
timeout -k 10 280 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_build_sizes.py tests/test_gpu_00_configs.py tests/test_gpu_refit.py > $OUT/tests.log 2>&1 || exit 1
for i in 1 2 3; do
timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy >> $OUT/new.log 2>&1 || exit 3
BEAM_HIP_LIB=$ROOT/raytracercuda_amd/libbeam_hip_prev.so timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy >> $OUT/old.log 2>&1 || exit 4
done
echo ok
