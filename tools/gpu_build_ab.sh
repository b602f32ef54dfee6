#!/usr/bin/env bash
# Build-time A/B of libbeam_hip builds (tools/build_bench.py under BEAM_HIP_LIB) + the BVH parity
# tests on each. Usage: bash tools/gpu_build_ab.sh lib1.so lib2.so ...   (names in raytracercuda_amd/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for lib in "$@"; do
  echo "== $lib"
  BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$lib timeout -k 10 120 python tools/build_bench.py 2>&1 | grep -v amdgpu.ids || exit $?
  BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$lib timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x \
    -k "bit_identical or armadillo_proxy_1080" --timeout 250 2>&1 | tail -1 || exit $?
done
