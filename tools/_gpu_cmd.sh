set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v20; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_reference_mode.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/libbeam_hip_wd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_reference_mode.py > $OUT/tests_wd.log 2>&1
rc=$?; tail -2 $OUT/tests_wd.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
 for v in libbeam_hip.so libbeam_hip_wd.so; do
   echo "-- $v"; BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 120 python tools/ref_time.py c2 filled c5 2>&1 | grep -v "amdgpu.ids\|frames in flight" || exit 4
 done
done
