#!/usr/bin/env bash
# Per-kernel build times: rocprofv3 --kernel-trace of tools/build_bench.py per scene (plus the
# build_bench medians), summarised by tools/build_kernels.py. Usage: tools/gpu_build_kernels.sh TAG [lib.so]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
[ -n "${2:-}" ] && export BEAM_HIP_LIB="$ROOT/raytracercuda_amd/$2"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy > "$OUT/bb.log" 2>&1 || exit $?
for sc in bunny armadillo_proxy merged_proxy; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv \
     -d "$OUT/k_$sc" -o b -- python3 "$ROOT/tools/build_bench.py" $sc > "$OUT/k_$sc.log" 2>&1) || exit $?
done
python tools/build_kernels.py "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/bb.log" "$OUT/summary.txt"
