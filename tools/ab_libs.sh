#!/usr/bin/env bash
# A/B of library builds on the GPU box: trace times (tools/ab_trace.py) of each .so on the bench
# view, the filled view and with shadow rays, interleaved per library, every step time-limited.
#   tools/ab_libs.sh OUTDIR lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"
for view in bench filled shadow; do
  for lib in "$@"; do
    env_args=""
    [ "$view" = filled ] && env_args="AB_FILLED=1"
    [ "$view" = shadow ] && env_args="AB_SHADOW=1"
    echo "== $view $lib" >> "$OUT/ab.log"
    env $env_args BEAM_HIP_LIB="$lib" timeout -k 10 120 python tools/ab_trace.py bunny,armadillo_proxy,merged_proxy 40 >> "$OUT/ab.log" 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc" >> "$OUT/ab.log"; exit $rc; fi
  done
done
