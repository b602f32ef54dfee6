#!/usr/bin/env bash
# Profile session for one or more bench configs, on the GPU box, from one source revision:
#   tools/gpu_profile.sh TAG "c2 c3"
# Per config: rocprofv3 --kernel-trace --stats of `bench.py --only single` and `--only inflight`
# (every averaged launch of one kind), then separate --pmc passes (one counter group per run, no
# tracing domains) of the single-frame and the in-flight commands (a sparse view in flight runs the
# cull + compacted quads kernels, bm_rt_trace_kind): FETCH_SIZE, WRITE_SIZE, L2 hit/miss, TA busy, SQ
# wave-state counters. The box's source stamp goes into $OUT/stamp.txt; on the CPU side
# tools/summarize_profile.py turns $OUT/<cfg> into profiles/<name>_<cfg>.md + _traffic.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-prof}; CONFIGS=${2:-c2}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import sys; sys.path.insert(0, '.'); from raytracercuda_amd import build; print(build.source_stamp())" > "$OUT/stamp.txt"
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
BENCH_ARGS="--no-extra --no-cpu-baseline --steps 30 --warmup 5"
for cfg in $CONFIGS; do
  D="$OUT/$cfg"; mkdir -p "$D"
  for mode in single inflight; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
       -d "$D/prof_$mode" -o bench -- python3 "$ROOT/bench.py" --config $cfg --only $mode $BENCH_ARGS \
       > "$D/prof_$mode.log" 2>&1)
    rc=$?; echo "== $cfg prof $mode rc=$rc"; tail -n 1 "$D/prof_$mode.log" | cut -c1-300
    if fatal $rc; then exit $rc; fi
  done
  i=0
  for pm in single inflight; do
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" \
             "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum TD_TC_STALL_sum"; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
       -d "$D/pmc_$i" -o pmc -- python3 "$ROOT/bench.py" --config $cfg --only $pm $BENCH_ARGS --steps 10 \
       > "$D/pmc_$i.log" 2>&1)
    rc=$?; echo "== $cfg pmc $pm $i ($grp) rc=$rc"
    if fatal $rc; then exit $rc; fi
  done
  done
done
echo "== done"
