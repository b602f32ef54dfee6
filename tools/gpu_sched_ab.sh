#!/usr/bin/env bash
# A/B of the quad kernel's tile schedules (BM_TRACE_SCHED 1 = block-dynamic screen order, 2 = longest
# first by the last trace's tile times) + the variant parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do for sc in 1 2; do
  echo "sched=$sc"; BM_TRACE_SCHED=$sc timeout -k 10 120 python tools/ab_trace.py bunny,armadillo_proxy,merged_proxy 50 2>&1 | grep -v amdgpu.ids || exit $?
  BM_TRACE_SCHED=$sc AB_SHADOW=1 timeout -k 10 120 python tools/ab_trace.py merged_proxy 30 2>&1 | grep -v amdgpu.ids || exit $?
done; done
timeout -k 10 400 python -m pytest tests/test_gpu_variants.py -q -x --timeout 300 2>&1 | tail -2
