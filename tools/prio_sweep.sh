#!/usr/bin/env bash
# Sweep the priority-boost threshold/level for the persistent trace kernels (A/B, identical outputs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lvl in 2 3; do for after in 8 16 24 32 48; do
  echo "== level $lvl after $after"
  BM_TRACE_PRIO_LEVEL=$lvl BM_TRACE_PRIO_AFTER=$after timeout -k 10 120 python tools/trace_variants.py 6:0,7:0 || exit $?
done; done
