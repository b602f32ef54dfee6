set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v30; mkdir -p $OUT
for v in libbeam_hip_head.so libbeam_hip_hl.so libbeam_hip.so; do
  echo "-- $v"; BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 300 python tools/hash_time.py c2 c3 > $OUT/t.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/t.log; [ $rc -eq 0 ] || exit 4
done
