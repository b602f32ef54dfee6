#!/usr/bin/env bash
# A/B of the bucket sort's dispatch order (BM_BS_LPT builds, tools/build_ab.py): build times interleaved,
# then the build-size and refit parity tests on the last variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
LIBS=${LIBS:-"libbeam_hip.so libbeam_hip_lpt.so libbeam_hip_lpt2.so"}
for r in 1 2 3; do
  for lib in $LIBS; do
    echo "== $lib round $r"
    BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$lib timeout -k 10 120 python tools/build_bench.py ${SCENES:-bunny,armadillo_proxy,merged_proxy} 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
for lib in $LIBS; do
  BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_build_sizes.py tests/test_gpu_refit.py -q -x --timeout 300 --timeout-method thread 2>&1 | tail -1 || exit $?
done
