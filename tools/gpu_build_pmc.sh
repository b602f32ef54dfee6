#!/usr/bin/env bash
# PMC passes (one counter group per run) over tools/build_bench.py SCENE: bash tools/gpu_build_pmc.sh TAG SCENE "grp1" "grp2" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=$1; SC=$2; shift 2
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
i=0
for grp in "$@"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
     -d "$OUT/pmc_$i" -o pmc -- python3 "$ROOT/tools/build_bench.py" $SC > "$OUT/pmc_$i.log" 2>&1) || exit $?
  echo "== pmc $i ($grp) ok"
done
