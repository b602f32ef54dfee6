#!/usr/bin/env bash
# Build iteration on one box: build A/B (tools/gpu_build_ab2.sh: GPU build tests, then interleaved
# build_bench against OTHER), then the per-kernel diag spans (tools/build_diag.py) of the diag builds
# libbeam_hip_bdiag.so and, if present, libbeam_hip_bdiag_<suffix>.so.
#   bash tools/gpu_build_round.sh TAG OTHER.so [suffix] [scenes]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; OTHER=$2; SUF=${3:-}; SC=${4:-bunny,armadillo_proxy,merged_proxy}
OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/gpu_build_ab2.sh $TAG $OTHER $SC || exit $?
for lib in libbeam_hip_bdiag.so ${SUF:+libbeam_hip_bdiag_$SUF.so}; do
  [ -f raytracercuda_amd/$lib ] || continue
  echo "== diag $lib"
  BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$lib timeout -k 10 120 python tools/build_diag.py $SC 2>&1 | grep -v amdgpu.ids || exit 5
done
