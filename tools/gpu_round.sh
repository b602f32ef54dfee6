#!/usr/bin/env bash
# One GPU-box session for a source revision: smoke -> config + full GPU tests -> bench (default) ->
# 2-rank shared-device rehearsal of the N>1 bench path -> profile session (tools/gpu_profile.sh).
# Every GPU step has its own time limit; a fault, abort, segfault or time limit ends the session.
#   tools/gpu_round.sh TAG [profile configs, default "c2 c3"]
# TESTS=0 / BENCH=0 skip those steps (a round split over several gpurun calls); REFPROF=1 adds a
# kernel trace of reference mode (tools/prof_refmode.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-round}; PCFG=${2:-c2 c3}
OUT="gpurun_out/$TAG"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 3 "$OUT/$name.log" | cut -c1-400 | tee -a "$OUT/session.log"
  if fatal $rc; then echo "FATAL in $name: stopping" | tee -a "$OUT/session.log"; exit $rc; fi
  return $rc
}
if [ "${TESTS:-1}" = "1" ]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step pytest_gpu 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -rf
fi
if [ "${L2CAL:-0}" = "1" ]; then  # L1 -> L2 request size (tools/pmc.py L2_REQ_BYTES)
  step l2_calib 120 python tools/l2_calib.py "$OUT/l2_calib"
fi
if [ "${BENCH:-1}" = "1" ]; then  # the driver's own command line
  step bench 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
  cp gpurun_out/bench_full.json "$OUT/bench_full.json" 2>/dev/null
fi
if [ "${REHEARSE:-1}" = "1" ] && [ "${BENCH:-1}" = "1" ]; then  # the self-launched N-rank path, on one GPU
  step rehearse2 300 env BM_BENCH_SHARED_DEVICE=1 python3 bench.py --gpus 2 --steps 20 --warmup 5
fi
if [ -n "$PCFG" ]; then
  step profile 900 bash tools/gpu_profile.sh "$TAG/prof" "$PCFG"
fi
if [ "${REFPROF:-0}" = "1" ]; then  # reference mode: kernel trace of 8 kd builds + 10 frames (C2)
  step refprof 300 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv \
    -d $PWD/$OUT/refprof -o ref -- python3 $PWD/tools/prof_refmode.py c2 8 10"
fi
echo "== done" | tee -a "$OUT/session.log"
