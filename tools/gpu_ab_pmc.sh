#!/usr/bin/env bash
# A/B of library builds: trace times (tools/ab_libs.sh) and one WRITE_SIZE / FETCH_SIZE pass of a
# bunny single-frame trace per library (tools/trace_once.py), then the config parity tests on the
# in-tree library.   tools/gpu_ab_pmc.sh OUTDIR lib1.so lib2.so ...   (paths under raytracercuda_amd/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$1; shift; mkdir -p "gpurun_out/$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
libs=""; for l in "$@"; do libs="$libs $ROOT/raytracercuda_amd/$l"; done
bash tools/ab_libs.sh "$OUT" $libs || exit $?
for l in "$@"; do
  for ctr in WRITE_SIZE FETCH_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && BEAM_HIP_LIB="$ROOT/raytracercuda_amd/$l" timeout -s KILL 90 rocprofv3 --pmc $ctr \
       --kernel-trace --output-format csv -d "$ROOT/gpurun_out/$OUT/pmc_${l%.so}_$ctr" -o pmc -- \
       python3 "$ROOT/tools/trace_once.py" ${AB_SCENE:-bunny} 8 > "$ROOT/gpurun_out/$OUT/pmc_${l%.so}_$ctr.log" 2>&1)
    rc=$?; echo "pmc $l $ctr rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
if [ -n "${AB_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $AB_TESTS > "gpurun_out/$OUT/tests.log" 2>&1
  rc=$?; tail -3 "gpurun_out/$OUT/tests.log"; exit $rc
fi
