#!/usr/bin/env bash
# PMC passes over the trace kernel (one counter group per rocprofv3 run, no tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-pmc}; SCENE=${2:-bunny}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 ${PMC_TIMEOUT:-90} rocprofv3 --pmc $grp --kernel-trace --output-format csv \
     -d "$OUT/g$i" -o pmc -- python3 "$ROOT/tools/trace_once.py" "$SCENE" 5 > "$OUT/g$i.log" 2>&1)
  rc=$?; echo "group $i ($grp) rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done < "${PMC_GROUPS:-tools/pmc_groups.txt}"
