set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/llds
BEAM_HIP_LIB=$PWD/raytracercuda_amd/libbeam_hip_leaflds.so timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_00_configs.py > gpurun_out/llds/tests.log 2>&1 && \
bash tools/ab_libs.sh llds $PWD/raytracercuda_amd/libbeam_hip.so $PWD/raytracercuda_amd/libbeam_hip_leaflds.so
