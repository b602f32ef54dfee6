#!/usr/bin/env bash
# A/B of two builds of libbeam_hip.so on the bench camera (ab_trace.py), interleaved twice, plus the
# GPU test suite on the new build. Usage: bash tools/gpu_lib_ab.sh <base.so> [scenes]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
BASE=$1; SC=${2:-bunny,armadillo_proxy,merged_proxy}
mkdir -p gpurun_out/libab
for r in 1 2; do
  for lib in raytracercuda_amd/$BASE raytracercuda_amd/libbeam_hip.so; do
    BEAM_HIP_LIB=$(pwd)/$lib timeout -k 10 120 python tools/ab_trace.py $SC 50 2>&1 | grep -v amdgpu.ids || exit $?
    AB_SHADOW=1 BEAM_HIP_LIB=$(pwd)/$lib timeout -k 10 120 python tools/ab_trace.py merged_proxy 30 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/libab/tests.log 2>&1; rc=$?
tail -3 gpurun_out/libab/tests.log; exit $rc
