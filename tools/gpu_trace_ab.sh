#!/usr/bin/env bash
# Trace A/B of library builds: bench view (C2/C3/merged) and the filled view, interleaved twice.
#   bash tools/gpu_trace_ab.sh base.so [other.so ...]   (libbeam_hip.so is always included, last)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  for lib in "$@" libbeam_hip.so; do
    BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$lib timeout -k 10 120 python tools/ab_trace.py bunny,armadillo_proxy,merged_proxy 40 2>&1 | grep -v amdgpu.ids || exit $?
    AB_FILLED=1 BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$lib timeout -k 10 120 python tools/ab_trace.py armadillo_proxy 30 2>&1 | grep -v amdgpu.ids | sed 's/^/filled /' || exit $?
    AB_SHADOW=1 BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$lib timeout -k 10 120 python tools/ab_trace.py merged_proxy 30 2>&1 | grep -v amdgpu.ids | sed 's/^/shadow /' || exit $?
  done
done
