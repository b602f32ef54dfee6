set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v39; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_00_configs.py tests/test_gpu_variants.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/rays_timeline.py c3 > $OUT/tl.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/tl.log; [ $rc -eq 0 ] || exit 5
bash tools/gpu_inflight_ab.sh "c3 c2 c5" "libbeam_hip_lpt0.so" > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; exit $rc
