#!/usr/bin/env bash
# A/B of trace kernels, interleaved per config and round: each case LABEL=LIB:PARAMS runs
# bench.py --config C --only MODE with that library (BEAM_HIP_LIB; "-" = in-tree) and --param list.
#   bash tools/gpu_packet_ab.sh TAG "c2 c3 filled c4" ROUNDS "single inflight" "quad=-: pk=-:trace_variant=14 pk6=libbeam_hip_pw6.so:trace_variant=14"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; CONFIGS=${2:-"c2 c3 filled c4"}; ROUNDS=${3:-2}; MODES=${4:-"single"}
CASES=${5:-"quad=-: pk=-:trace_variant=14"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
 for cfg in $CONFIGS; do
  for mode in $MODES; do
   for case in $CASES; do
    label=${case%%=*}; rest=${case#*=}; lib=${rest%%:*}; params=${rest#*:}
    P=""; for kv in ${params//,/ }; do P="$P --param $kv"; done
    L=""; [ "$lib" != "-" ] && L=$(pwd)/raytracercuda_amd/$lib
    line=$(BEAM_HIP_LIB=$L timeout -k 10 180 python bench.py --config $cfg --only $mode --no-extra --no-cpu-baseline \
           --pmc off --steps 40 --warmup 5 $P 2>>$OUT/stderr.log | grep '^{') || exit 3
    python -c "import json,sys; r=json.loads(sys.argv[1]); print('$r', '$cfg', '$mode', '$label', r['trace_kind'], round(r['value']), 'Mrays/s', round(r['trace_kernel_ms']*1e3,1), 'us/launch', round(r['ms_per_step']*1e3,1), 'us/step')" "$line"
   done
  done
 done
done
