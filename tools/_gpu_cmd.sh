set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v6; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_build_sizes.py tests/test_gpu_parity.py tests/test_gpu_refit.py tests/test_gpu_00_configs.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
 for v in libbeam_hip.so libbeam_hip_bu.so libbeam_hip_nonrm.so; do
  echo "-- $v $r"; BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy 2>&1 | grep -v amdgpu.ids || exit 4
 done
done
echo "== diag"; BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/libbeam_hip_bdiag.so timeout -k 10 120 python tools/build_diag.py bunny,armadillo_proxy,merged_proxy 2>&1 | grep -v amdgpu.ids || exit 5
