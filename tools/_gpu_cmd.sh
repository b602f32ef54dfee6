set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD; OUT=$ROOT/gpurun_out/kdpf; mkdir -p $OUT
timeout -k 10 280 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_reference_mode.py tests/test_gpu_00_configs.py > $OUT/tests.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 200 python tools/ref_time.py c2 filled c5 >> $OUT/pf1.log 2>&1 || exit 2
BEAM_HIP_LIB=$ROOT/raytracercuda_amd/libbeam_hip_pf0.so timeout -k 10 200 python tools/ref_time.py c2 filled c5 >> $OUT/pf0.log 2>&1 || exit 3
done
echo ok
