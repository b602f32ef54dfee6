#!/usr/bin/env bash
# k_front A/B on one box: GPU build tests, then tools/build_bench.py with the fused front launch
# (default) and without it (BM_FRONT_MAX_N=0 -> front_max_n 0), interleaved, then the build diag.
#   bash tools/gpu_front_ab.sh TAG [scenes]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; SC=${2:-bunny,armadillo_proxy,merged_proxy}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_build_sizes.py \
  tests/test_gpu_parity.py tests/test_gpu_refit.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  echo "-- front $r"; timeout -k 10 120 python tools/build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 3
  echo "-- separate $r"; BM_FRONT_MAX_N=0 timeout -k 10 120 python tools/build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 4
done
