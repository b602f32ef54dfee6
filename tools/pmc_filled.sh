#!/usr/bin/env bash
# Instruction-mix PMC passes of one bench config (single frame): where the quad kernel's issue goes.
#   tools/pmc_filled.sh TAG [config]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT="$ROOT/gpurun_out/$1"; CFG=${2:-filled}; mkdir -p "$OUT"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
     -d "$OUT/pmc_$i" -o pmc -- python3 "$ROOT/bench.py" --config $CFG --only single --no-extra --no-cpu-baseline \
     --steps 10 --warmup 3 > "$OUT/pmc_$i.log" 2>&1)
  rc=$?; echo "== pmc $i ($grp) rc=$rc"; tail -n 2 "$OUT/pmc_$i.log" | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
done
echo "== done"
