set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v67; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hash.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
 for v in libbeam_hip_hp0.so libbeam_hip.so; do
  echo "-- $v"; BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 200 python tools/hash_time.py c2 > $OUT/t.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/t.log; [ $rc -eq 0 ] || exit 4
 done
done
