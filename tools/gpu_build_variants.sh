#!/usr/bin/env bash
# Build A/B over several variants on one box: GPU build tests on the in-tree library, then
# tools/build_bench.py per variant, interleaved over 3 rounds. A variant is a library under
# raytracercuda_amd/ or ENV=VALUE for tools/ab_env.py (a parameter of the in-tree library).
#   bash tools/gpu_build_variants.sh TAG SCENES VARIANT...   e.g. ... r04 bunny,armadillo_proxy BM_FRONT_MAX_N=0 libbeam_hip_pt0.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; SC=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_build_sizes.py \
  tests/test_gpu_parity.py tests/test_gpu_refit.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  echo "-- in-tree $r"; timeout -k 10 120 python tools/build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 3
  for v in "$@"; do
    echo "-- $v $r"
    case "$v" in
      *.so) BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 120 python tools/build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 4 ;;
      *) env "$v" timeout -k 10 120 python tools/build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 5 ;;
    esac
  done
done
