#!/usr/bin/env bash
# Build A/B on one box: GPU build tests on the in-tree library, then tools/build_bench.py interleaved
# between it and an A/B build (BEAM_HIP_LIB). Usage: bash tools/gpu_build_ab2.sh TAG other.so [scenes] [tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; OTHER=$2; SC=${3:-bunny,armadillo_proxy,merged_proxy}
TESTS=${4:-tests/test_gpu_build_sizes.py tests/test_gpu_parity.py tests/test_gpu_refit.py}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  echo "-- new $r"; timeout -k 10 120 python tools/build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 3
  echo "-- $OTHER $r"; BEAM_HIP_LIB=$(pwd)/$OTHER timeout -k 10 120 python tools/build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 4
done
