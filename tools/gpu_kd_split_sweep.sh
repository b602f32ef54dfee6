#!/usr/bin/env bash
# Reference-mode build over hand-off depths (BM_KD_SPLIT -> kd_split param): tools/kd_build_bench.py per
# depth, twice.   bash tools/gpu_kd_split_sweep.sh "12 15 18 21 23" [scenes]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
SC=${2:-bunny,armadillo_proxy,merged_proxy}
for r in 1 2; do
  echo "-- default $r"; timeout -k 10 120 python tools/kd_build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 3
  for d in $1; do
    echo "-- split $d $r"; BM_KD_SPLIT=$d timeout -k 10 120 python tools/kd_build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 4
  done
done
