#!/usr/bin/env bash
# Final round-6 session: every GPU test, the driver's default bench command, the trace profiles of
# c3 / filled / c4 (tools/gpu_profile.sh) and a kernel trace of reference mode (builds + frames, c2).
#   bash tools/gpu_final_r06.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=$1
bash tools/gpu_session_r06.sh "$TAG" all default "c3 filled c4" || exit $?
OUT="$ROOT/gpurun_out/$TAG"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$OUT/refprof" -o ref -- python3 "$ROOT/tools/prof_refmode.py" c2 8 10 > "$OUT/refprof.log" 2>&1) || exit 8
echo "== final session done"
