#!/usr/bin/env bash
# Per-kernel build times (rocprofv3 --kernel-trace --stats of tools/build_bench.py SCENE) for A/B
# library builds: bash tools/gpu_lib_prof.sh TAG SCENE lib1.so lib2.so ...  (names in raytracercuda_amd/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=$1; SC=$2; shift 2
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
for lib in "$@"; do
  export BEAM_HIP_LIB=$ROOT/raytracercuda_amd/$lib
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$OUT/$lib" -o b -- python3 "$ROOT/tools/build_bench.py" $SC > "$OUT/$lib.log" 2>&1) || exit $?
  echo "== $lib"; grep tris "$OUT/$lib.log"
  python3 - "$OUT/$lib/b_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'].replace('bm::(anonymous namespace)::','').split('(')[0][:40]:40s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.1f} us")
PY
done
