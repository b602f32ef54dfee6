set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v37; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_00_configs.py tests/test_gpu_variants.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_inflight_ab.sh "c3 c2 c5" "libbeam_hip_xq0.so libbeam_hip_xq2.so" > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; exit $rc
