set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/f2
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_build_sizes.py tests/test_gpu_parity.py tests/test_gpu_refit.py tests/test_gpu_reference_mode.py tests/test_gpu_bvh8.py > gpurun_out/f2/tests.log 2>&1 && \
timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy > gpurun_out/f2/bb.log 2>&1 && \
BEAM_HIP_LIB=$PWD/raytracercuda_amd/libbeam_hip_nofuse.so timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy > gpurun_out/f2/bb_nofuse.log 2>&1 && \
bash tools/gpu_build_diag.sh f2diag bunny,merged_proxy
