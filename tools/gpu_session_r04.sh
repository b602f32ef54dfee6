#!/usr/bin/env bash
# Round-4 iteration session: GPU tests for the touched paths, build diag spans of the diag libraries,
# then a profile session of the given configs (tools/gpu_profile.sh). Every step under its own limit;
# a failing step ends the session.
#   bash tools/gpu_session_r04.sh TAG "tests" "diag libs" "profile configs"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; TESTS=${2:-}; DIAG=${3:-}; PCFG=${4:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for lib in $DIAG; do
  echo "== diag $lib"
  BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$lib timeout -k 10 120 python tools/build_diag.py bunny,armadillo_proxy 2>&1 | grep -v amdgpu.ids || exit 5
done
if [ -n "$PCFG" ]; then
  timeout -k 10 900 bash tools/gpu_profile.sh $TAG/prof "$PCFG" > $OUT/profile.log 2>&1 || exit 6
  tail -2 $OUT/profile.log
fi
echo "== session done"
