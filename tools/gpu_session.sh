#!/usr/bin/env bash
# One GPU-box session: smoke -> gpu tests -> bench (-> optional rocprof). Every GPU step has its
# own time limit; a fault, abort, segfault or time limit (exit >= 124 or > 128) ends the session
# without starting further GPU work. Plain test failures (pytest exit 1) do not stop the bench.
# Usage: tools/gpu_session.sh [tag] [extra bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${1:-run}"; shift || true
OUT="gpurun_out/$TAG"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0

fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }

step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 5 "$OUT/$name.log" | tee -a "$OUT/session.log"
  if fatal $rc; then echo "FATAL in $name: stopping" | tee -a "$OUT/session.log"; exit $rc; fi
  return $rc
}

rocm-smi --showproductname > "$OUT/gpu.txt" 2>&1 || true
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -q -m gpu -p no:cacheprovider --timeout 600 -rf
step bench 600 python bench.py "$@"
echo "== done" | tee -a "$OUT/session.log"
