set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v61; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_reference_mode.py tests/test_gpu_00_configs.py -k "reference or kd or golden" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
 for v in libbeam_hip_os0.so libbeam_hip.so; do
  echo "-- $v"; BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 120 python tools/ref_time.py c2 filled c5 > $OUT/t.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/t.log | grep -v "2 frames"; [ $rc -eq 0 ] || exit 4
 done
done
