set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/p4
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_build_sizes.py tests/test_gpu_parity.py tests/test_gpu_refit.py > gpurun_out/p4/tests.log 2>&1 && \
timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy > gpurun_out/p4/bb.log 2>&1 && \
bash tools/gpu_build_diag.sh p4diag bunny,merged_proxy
