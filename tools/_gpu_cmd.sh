set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v25; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_reference_mode.py tests/test_gpu_00_configs.py -k "reference or golden" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
 for kv in 3 4; do
   echo "-- variant $kv"; BM_KD_VARIANT=$kv timeout -k 10 120 python tools/ref_time.py c2 filled c5 2>&1 | grep -v "amdgpu.ids\|frames in flight" || exit 4
 done
done
timeout -k 10 120 python tools/kd_build_bench.py bunny,armadillo_proxy 2>&1 | grep -v amdgpu.ids || exit 5
echo "== timeline c2"; timeout -k 10 120 python tools/kd_timeline.py c2 2>&1 | grep -v amdgpu.ids || exit 6
