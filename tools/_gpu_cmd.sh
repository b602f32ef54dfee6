set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD; OUT=$ROOT/gpurun_out/kds7; mkdir -p $OUT
timeout -k 10 280 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_reference_mode.py tests/test_gpu_00_configs.py tests/test_gpu_hash.py > $OUT/tests.log 2>&1 || exit 1
BDIAG_KD=1 BEAM_HIP_LIB=$ROOT/raytracercuda_amd/libbeam_hip_bdiag.so timeout -k 10 120 python tools/build_diag.py bunny > $OUT/diag_new.log 2>&1 || exit 3
timeout -k 10 120 python tools/kd_build_bench.py >> $OUT/new.log 2>&1 || exit 5
BM_KD_START=0 timeout -k 10 120 python tools/kd_build_bench.py >> $OUT/old.log 2>&1 || exit 4
echo ok
