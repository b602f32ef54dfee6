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
if [ -n "${AB:-}" ]; then step variant_ab 240 python tools/variant_ab.py $AB; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -q -m gpu -p no:cacheprovider --timeout 600 -rf
step bench 600 python bench.py "$@"
if [ "${DIAG:-0}" = "1" ]; then
  step timeline 120 python tools/wave_timeline.py bunny
  step trace_cost 180 python tools/trace_cost.py
fi
if [ "${PROFILE:-0}" = "1" ]; then
  ROOT=$(pwd)
  # kernel trace + per-kernel stats of the same bench command (no PMC in this pass)
  (cd /tmp && export TMPDIR=/tmp && step_dir="$ROOT/$OUT/prof" && mkdir -p "$step_dir" && \
   timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$step_dir" -o bench -- \
     python3 "$ROOT/bench.py" --no-cpu-baseline --no-extra "$@" > "$ROOT/$OUT/prof.log" 2>&1)
  rc=$?; echo "== prof rc=$rc" | tee -a "$OUT/session.log"; tail -n 3 "$OUT/prof.log" | tee -a "$OUT/session.log"
  if fatal $rc; then exit $rc; fi
  if [ -n "${PMC:-}" ]; then
    for ctr in $PMC; do
      (cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/$OUT/pmc_$ctr" && \
       timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$ROOT/$OUT/pmc_$ctr" -o pmc -- \
         python3 "$ROOT/bench.py" --no-cpu-baseline --no-extra "$@" > "$ROOT/$OUT/pmc_$ctr.log" 2>&1)
      rc=$?; echo "== pmc $ctr rc=$rc" | tee -a "$OUT/session.log"
      if fatal $rc; then exit $rc; fi
    done
  fi
fi
echo "== done" | tee -a "$OUT/session.log"
