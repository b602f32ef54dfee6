set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v81; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_00_configs.py tests/test_gpu_variants.py tests/test_gpu_parity.py tests/test_gpu_shadow.py tests/test_gpu_multidevice.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_inflight_ab.sh "c3 c2 c4 c5" "libbeam_hip_npf.so" > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3 4; do
 for v in "" libbeam_hip_npf.so; do
  lib=""; [ -n "$v" ] && lib=$(pwd)/raytracercuda_amd/$v
  line=$(BEAM_HIP_LIB=$lib timeout -k 10 180 python bench.py --config c3 --only inflight --no-extra --no-cpu-baseline --steps 20 --warmup 5 2>/dev/null | grep '^{') || exit 3
  python -c "import json,sys; r=json.loads(sys.argv[1]); print('${v:-prefetch}', round(r['value']), round(r['ms_per_step']*1e3,1))" "$line"
 done
done
