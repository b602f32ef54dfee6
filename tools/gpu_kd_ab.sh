#!/usr/bin/env bash
# Reference-mode A/B: kd build times (tools/kd_build_bench.py) and C2 kd march (tools/ref_time.py),
# interleaved between the in-tree library and OTHER.so.   bash tools/gpu_kd_ab.sh OTHER.so [scenes]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
OTHER=$1; SC=${2:-bunny,armadillo_proxy,merged_proxy}
for r in 1 2; do
  for lib in raytracercuda_amd/libbeam_hip.so $OTHER; do
    echo "-- $lib $r"
    BEAM_HIP_LIB=$(pwd)/$lib timeout -k 10 120 python tools/kd_build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 3
    BEAM_HIP_LIB=$(pwd)/$lib timeout -k 10 120 python tools/ref_time.py c2 2>&1 | grep -v amdgpu.ids || exit 4
  done
done
