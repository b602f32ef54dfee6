#!/usr/bin/env bash
# Reference-mode build times (tools/kd_build_bench.py), interleaved over libraries (BEAM_HIP_LIB; "-" = in-tree).
#   bash tools/gpu_kd_lib_ab.sh "LABEL=LIB ..." [scenes]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
CASES=$1; SC=${2:-bunny,armadillo_proxy,merged_proxy}
for r in 1 2; do
  for case in $CASES; do
    label=${case%%=*}; lib=${case#*=}
    L=""; [ "$lib" != "-" ] && L=$(pwd)/raytracercuda_amd/$lib
    echo "-- $label round $r"
    BEAM_HIP_LIB=$L timeout -k 10 120 python tools/kd_build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 3
  done
done
