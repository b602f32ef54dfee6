#!/usr/bin/env bash
# PMC groups over the trace kernel for several trace variants (one rocprofv3 --pmc run per group and
# variant, kernel trace only, no tracing domains), then a per-kernel summary (tools/pmc_summary.py).
#   tools/pmc_compare.sh <tag> <variants e.g. 6,10> [scene]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-pmcc}; VARS=${2:-6,10}; SCENE=${3:-bunny}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
for v in ${VARS//,/ }; do
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp BM_TRACE_VARIANT=$v && timeout -k 10 ${PMC_TIMEOUT:-90} rocprofv3 --pmc $grp \
       --kernel-trace --output-format csv -d "$OUT/v${v}_g$i" -o pmc -- python3 "$ROOT/tools/trace_once.py" "$SCENE" 5 \
       > "$OUT/v${v}_g$i.log" 2>&1)
    rc=$?; echo "variant $v group $i ($grp) rc=$rc"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  done < "${PMC_GROUPS:-tools/pmc_groups_core.txt}"
done
python3 tools/pmc_summary.py "$OUT" | tee "$OUT/summary.txt"
