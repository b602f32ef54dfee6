set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v31; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_variants.py tests/test_gpu_00_configs.py tests/test_gpu_shadow.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
 for v in libbeam_hip_x0.so libbeam_hip.so libbeam_hip_x64.so; do
  echo "-- $v"; BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 300 python tools/host_rate.py c3 c2 c5 > $OUT/t.log 2>&1; rc=$?; grep -v "amdgpu.ids" $OUT/t.log | grep "every -\|every 4"; [ $rc -eq 0 ] || exit 4
 done
done
