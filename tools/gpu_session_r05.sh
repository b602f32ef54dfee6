#!/usr/bin/env bash
# Round-5 iteration session: GPU tests of the touched paths, then interleaved build A/B rounds
# (tools/build_bench.py per library), then a bench run (live PMC passes: per-kernel build traffic).
# Every GPU step under its own limit; a failing step ends the session.
#   bash tools/gpu_session_r05.sh TAG "tests" "scenes" "variant libs" "bench args"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; TESTS=${2:-}; SC=${3:-bunny,armadillo_proxy,merged_proxy}; VARS=${4:-}; BARGS=${5:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$VARS" ]; then
  for r in 1 2 3; do
    echo "-- in-tree $r"; timeout -k 10 120 python tools/build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 3
    for v in $VARS; do
      echo "-- $v $r"
      BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 120 python tools/build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 4
    done
  done
fi
if [ -n "$BARGS" ]; then
  timeout -k 10 400 python3 bench.py $BARGS > $OUT/bench.log 2>&1
  rc=$?; tail -2 $OUT/bench.log | cut -c1-300; cp gpurun_out/bench_full.json $OUT/ 2>/dev/null; [ $rc -eq 0 ] || exit 6
fi
echo "== session done"
