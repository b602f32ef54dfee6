#!/usr/bin/env bash
# One PMC pass over the reference-mode build (tools/prof_refmode.py c2): instruction mix and wave time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT="$ROOT/gpurun_out/${1:-kdpmc}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU \
  --output-format csv -d "$OUT/pmc" -o p -- python3 "$ROOT/tools/prof_refmode.py" c2 2 1 > "$OUT/pmc.log" 2>&1
echo "pmc rc=$?"
