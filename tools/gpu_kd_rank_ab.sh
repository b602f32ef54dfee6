#!/usr/bin/env bash
# Reference-mode pair sort: ranked top digit (default) against four plain passes (BM_KD_TOP_RANK=0),
# kd build times interleaved; then the same builds under a kernel trace (tools/kd_build_timeline.py).
#   bash tools/gpu_kd_rank_ab.sh TAG [scenes]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; SC=${2:-bunny,armadillo_proxy,merged_proxy}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in 1 2; do
  for rank in 1 0; do
    echo "-- rank=$rank round $r"
    BM_KD_TOP_RANK=$rank timeout -k 10 120 python tools/kd_build_bench.py $SC 2>&1 | grep -v amdgpu.ids || exit 3
  done
done
for rank in 1 0; do
  (cd /tmp && export TMPDIR=/tmp && BM_KD_TOP_RANK=$rank timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv \
     -d "$OLDPWD/$OUT/kd$rank" -o kd -- python3 "$OLDPWD/tools/kd_build_bench.py" bunny > "$OLDPWD/$OUT/kd$rank.log" 2>&1) || exit 4
done
