#!/usr/bin/env bash
# C5 (fused shadow rays) A/B of library builds: one WRITE_SIZE pass and one FETCH_SIZE pass of
# `bench.py --config c5 --only single` per library (rocprofv3 --pmc, no tracing domains), then the
# single-frame bench line of each, interleaved twice.   tools/gpu_c5_ab.sh OUTDIR lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$1; shift; mkdir -p "gpurun_out/$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
CFG=${AB_CFG:-c5}
ARGS="--config $CFG --only single --no-extra --no-cpu-baseline --warmup 5"
for l in "$@"; do
  for ctr in WRITE_SIZE FETCH_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && BEAM_HIP_LIB="$ROOT/raytracercuda_amd/$l" timeout -s KILL 120 rocprofv3 --pmc $ctr \
       --kernel-trace --output-format csv -d "$ROOT/gpurun_out/$OUT/pmc_${l%.so}_$ctr" -o pmc -- \
       python3 "$ROOT/bench.py" $ARGS --steps 10 > "$ROOT/gpurun_out/$OUT/pmc_${l%.so}_$ctr.log" 2>&1)
    rc=$?; echo "pmc $l $ctr rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
for r in 1 2; do
  for l in "$@"; do
    BEAM_HIP_LIB="$ROOT/raytracercuda_amd/$l" timeout -k 10 120 python bench.py $ARGS --steps 30 \
      > "gpurun_out/$OUT/bench_${l%.so}_$r.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench $l rc=$rc"; exit $rc; }
    python - "gpurun_out/$OUT/bench_${l%.so}_$r.log" "$l" <<'P'
import json, sys
rec = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
sf = rec.get("single_frame", {})
print(f"{sys.argv[2]:32s} value {rec['value']:.0f} Mrays/s  trace_kernel_ms {rec.get('trace_kernel_ms')}  frame_check {rec.get('frame_check')}")
P
  done
done
