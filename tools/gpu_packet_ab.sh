#!/usr/bin/env bash
# Wave packets (TRACE_PACKET = 14) against the default kernels, one frame at a time on the context stream
# and frames in flight, interleaved per config: bench.py --only single|inflight --param trace_variant=V.
#   bash tools/gpu_packet_ab.sh TAG "c2 c3 filled c4" ROUNDS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; CONFIGS=${2:-"c2 c3 filled c4"}; ROUNDS=${3:-2}; MODES=${4:-"single"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
 for cfg in $CONFIGS; do
  for mode in $MODES; do
   for v in default 14; do
    P=""; [ "$v" != default ] && P="--param trace_variant=$v"
    line=$(timeout -k 10 180 python bench.py --config $cfg --only $mode --no-extra --no-cpu-baseline --pmc off \
           --steps 40 --warmup 5 $P 2>>$OUT/stderr.log | grep '^{') || exit 3
    python -c "import json,sys; r=json.loads(sys.argv[1]); print('$r', '$cfg', '$mode', '$v', r['trace_kind'], round(r['value']), 'Mrays/s', round(r['trace_kernel_ms']*1e3,1), 'us/launch', round(r['ms_per_step']*1e3,1), 'us/step')" "$line"
   done
  done
 done
done
