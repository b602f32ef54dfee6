#!/usr/bin/env bash
# GPU-box check of trace variants: variant parity tests, an A/B of trace times (frames and counters
# compared bit for bit) and the per-kernel rocprofv3 stats of one variant.
# Usage (from gpurun): bash tools/gpu_variant_check.sh [variants=10,12] [stats_variant=12]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=gpurun_out/vcheck; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
V=${1:-10,12}; SV=${2:-12}
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > $OUT/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids $OUT/$name.log | tail -15; [ $rc -lt 124 ] || exit $rc; }
run tests python -u -m pytest tests/test_gpu_variants.py -x -q --timeout 300
run ab python tools/variant_ab.py $V bunny,armadillo_proxy,merged_proxy 50
(cd /tmp && export TMPDIR=/tmp && BM_TRACE_VARIANT=$SV timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/stats -o k -- python3 $ROOT/tools/trace_once.py bunny 20 > $ROOT/$OUT/stats.log 2>&1) || exit $?
grep -h "k_trace\|k_cull" $ROOT/$OUT/stats/k_kernel_stats.csv | cut -c1-160
