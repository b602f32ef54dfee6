set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v24; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_variants.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
 for v in libbeam_hip_head.so libbeam_hip.so; do
  for sc in 2 3; do
   [ $v = libbeam_hip_head.so ] && [ $sc = 3 ] && continue
   echo "-- $v sched $sc"
   BM_TRACE_SCHED=$sc BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 120 python tools/ab_trace.py bunny,armadillo_proxy,merged_proxy 30 2>&1 | grep -v amdgpu.ids || exit 4
   AB_SHADOW=1 BM_TRACE_SCHED=$sc BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 120 python tools/ab_trace.py merged_proxy 30 2>&1 | grep -v amdgpu.ids || exit 4
  done
 done
done
timeout -k 10 400 python3 bench.py --config c5 --only single --steps 20 --warmup 5 --no-cpu-baseline --param trace_sched=3 > $OUT/bench_c5_s3.log 2>&1 || exit 6
cp gpurun_out/bench_full.json $OUT/bench_c5_s3_full.json
timeout -k 10 400 python3 bench.py --config c5 --only single --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c5_s2.log 2>&1 || exit 7
cp gpurun_out/bench_full.json $OUT/bench_c5_s2_full.json
tail -c 300 $OUT/bench_c5_s3.log
