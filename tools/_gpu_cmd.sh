set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v80; mkdir -p $OUT
for r in 1 2; do
 for v in libbeam_hip_st3.so libbeam_hip.so libbeam_hip_st6.so; do
  echo "-- $v"; BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 120 python tools/ref_time.py c2 filled c5 > $OUT/t.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/t.log | grep -v "2 frames" | grep -v "3 frames"; [ $rc -eq 0 ] || exit 4
 done
done
