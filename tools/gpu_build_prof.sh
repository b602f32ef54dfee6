#!/usr/bin/env bash
# Build timing + kernel trace of the BVH build per scene (tools/build_bench.py), on the GPU box.
#   tools/gpu_build_prof.sh TAG "bunny merged_proxy"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-bprof}; SCENES=${2:-bunny merged_proxy}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
timeout -k 10 200 python tools/build_bench.py f16,bunny,armadillo_proxy,merged_proxy > "$OUT/build_bench.log" 2>&1 || exit $?
cat "$OUT/build_bench.log"
for sc in $SCENES; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$OUT/$sc" -o b -- python3 "$ROOT/tools/build_bench.py" $sc > "$OUT/$sc.log" 2>&1) || exit $?
done
echo "== done"
