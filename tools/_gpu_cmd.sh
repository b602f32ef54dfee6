set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v70; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_build_sizes.py tests/test_gpu_refit.py tests/test_gpu_parity.py tests/test_gpu_00_configs.py tests/test_gpu_variants.py tests/test_gpu_reference_mode.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
 for v in libbeam_hip_prev.so libbeam_hip.so; do
  echo "-- $v"; BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy > $OUT/t.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/t.log | cut -c1-80; [ $rc -eq 0 ] || exit 4
 done
done
bash tools/gpu_inflight_ab.sh "c3 c2" "libbeam_hip_prev.so" > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; exit $rc
