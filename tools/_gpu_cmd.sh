set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v47; mkdir -p $OUT
for v in 0 1 2 3; do
  echo "-- kd_sched $v"; BM_KD_SCHED=$v timeout -k 10 120 python tools/ref_time.py c2 c5 > $OUT/t.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/t.log | grep -v "2 frames"; [ $rc -eq 0 ] || exit 4
done
