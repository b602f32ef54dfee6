set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v53; mkdir -p $OUT
bash tools/gpu_inflight_ab.sh "c3 c2 c4" "libbeam_hip_u8.so libbeam_hip_u2.so" > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; exit $rc
