#!/usr/bin/env bash
# PMC passes (one counter group per rocprofv3 run) over any python command; prints mean per dispatch
# of the kernels whose name contains $FILTER.
#   FILTER=k_kd_march tools/pmc_quick.sh TAG python3 tools/ref_time.py c3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=$1; shift
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
     -d "$OUT/g$i" -o pmc -- "${@/#bench.py/$ROOT/bench.py}" > "$OUT/g$i.log" 2>&1)
  rc=$?; echo "group $i rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
python3 - "$OUT" "${FILTER:-k_}" <<'PY'
import collections, csv, glob, os, sys
src, flt = sys.argv[1], sys.argv[2]
per = collections.defaultdict(float)
for f in glob.glob(os.path.join(src, "g*", "pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if flt in r["Kernel_Name"]:
            per[(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
agg = collections.defaultdict(list)
for (c, d), v in per.items():
    agg[c].append(v)
for c in sorted(agg):
    print(f"  {c:34s} {sum(agg[c]) / len(agg[c]):16.1f}")
PY
