#!/usr/bin/env bash
# Round-6 session on the GPU box: GPU tests (a list, or "all"), then the driver's default bench command,
# then (optionally) the profile passes of tools/gpu_profile.sh for some configs. Every GPU step under its
# own limit; a failing step ends the session.
#   bash tools/gpu_session_r06.sh TAG "tests|all|" "bench args|" "profile configs|"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; TESTS=${2:-}; BARGS=${3:-}; PROF=${4:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$TESTS" = "all" ]; then TESTS="tests"; SEL="-m gpu"; else SEL=""; fi
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q $SEL --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BARGS" ]; then
  [ "$BARGS" = "default" ] && BARGS=""
  timeout -k 10 500 python3 bench.py $BARGS > $OUT/bench.log 2>&1
  rc=$?; grep '^{' $OUT/bench.log | cut -c1-400; cp gpurun_out/bench_full.json $OUT/ 2>/dev/null; [ $rc -eq 0 ] || exit 6
  grep '^{' $OUT/bench.log > $OUT/bench_line.json
fi
if [ -n "$PROF" ]; then
  bash tools/gpu_profile.sh $TAG/prof "$PROF" > $OUT/prof.log 2>&1; rc=$?; tail -2 $OUT/prof.log; [ $rc -eq 0 ] || exit 7
fi
echo "== session done"
