set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v19; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for v in libbeam_hip_old.so libbeam_hip.so; do
  echo "-- $v"; BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 120 python tools/kd_build_bench.py bunny,armadillo_proxy,merged_proxy 2>&1 | grep -v amdgpu.ids || exit 4
done
timeout -k 10 120 python tools/ref_time.py c2 filled c5 2>&1 | grep -v "amdgpu.ids" || exit 4
