#!/usr/bin/env bash
# Reference-mode build, split descent: parity tests, then build/trace times over BM_KD_SPLIT values,
# then a kernel trace of the default. tools/gpu_kd_split.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="gpurun_out/${1:-kdsplit}"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_reference_mode.py tests/test_gpu_00_configs.py -q -m gpu -x \
  -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for sp in ${SPLITS:-0 default nogrid 24 27 28}; do
  unset BM_KD_SPLIT BM_KD_GRID BM_KD_PAIR
  case $sp in default) ;; nogrid) export BM_KD_GRID=0 ;; nopair) export BM_KD_PAIR=0 ;; *) export BM_KD_SPLIT=$sp ;; esac
  echo "== split $sp"
  timeout -k 10 120 python tools/ref_time.py c2 c3 c5 filled > "$OUT/time_$sp.log" 2>&1 || { tail "$OUT/time_$sp.log"; exit 1; }
  cat "$OUT/time_$sp.log" | grep -v amdgpu.ids
done
unset BM_KD_SPLIT BM_KD_GRID BM_KD_PAIR
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o k -- python3 "$ROOT/tools/prof_refmode.py" c2 8 10 > "$ROOT/$OUT/prof.log" 2>&1
echo "prof rc=$?"
