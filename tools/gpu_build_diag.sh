#!/usr/bin/env bash
# Build-kernel spans (per-wave s_memrealtime / s_memtime) on the GPU box, idle and warm (a busy
# kernel on the stream right before each build). Library built on the CPU side:
#   python tools/build_ab.py raytracercuda_amd/libbeam_hip_bdiag.so BM_BUILD_DIAG=1
#   bash tools/gpu_build_diag.sh TAG [scenes]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-bdiag}; SC=${2:-bunny,armadillo_proxy,merged_proxy}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 BEAM_HIP_LIB=$ROOT/raytracercuda_amd/libbeam_hip_bdiag.so
timeout -k 10 120 python tools/build_diag.py "$SC" > "$OUT/diag.log" 2>&1 || exit $?

echo done
