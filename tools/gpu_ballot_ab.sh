#!/usr/bin/env bash
# Round-6 A/B of the bool ballot (BM_BOOL_BALLOT 1, in-tree) against HIP's int __ballot (libbeam_hip_gb0.so) on
# every kernel family that ballots: builds (radix ranking), the kd march, the cull + survivor quads, packets.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in 1 2; do
  for v in "" libbeam_hip_gb0.so; do
    lib=""; [ -n "$v" ] && lib=$(pwd)/raytracercuda_amd/$v
    echo "-- build ${v:-bool} $r"; BEAM_HIP_LIB=$lib timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy 2>&1 | grep -v amdgpu.ids || exit 3
    echo "-- refmode ${v:-bool} $r"; BEAM_HIP_LIB=$lib timeout -k 10 120 python tools/ref_time.py c2 filled 2>&1 | grep -v amdgpu.ids || exit 4
  done
done
bash tools/gpu_packet_ab.sh $TAG "c3 c2" 2 "single inflight" "gb0=libbeam_hip_gb0.so: bool=-:" || exit 5
bash tools/gpu_packet_ab.sh $TAG "filled c4" 2 "single inflight" "old=libbeam_hip_pk_old.so:trace_variant=14 gb0=libbeam_hip_gb0.so:trace_variant=14 bool=-:trace_variant=14 sn=libbeam_hip_pk_sn.so:trace_variant=14" || exit 6
