#!/usr/bin/env bash
# A/B of library builds through the bench itself (frames in flight and one frame at a time):
#   tools/ab_bench.sh OUTDIR "c2 c3 filled" lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; CFGS=$2; shift 2; mkdir -p "$OUT"
for round in 1 2; do
for cfg in $CFGS; do
  for lib in "$@"; do
    BEAM_HIP_LIB="$lib" timeout -k 10 120 python bench.py --config $cfg --no-extra --no-cpu-baseline --steps 40 --warmup 10 \
      > "$OUT/tmp.json" 2>> "$OUT/err.log"
    rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc $cfg $lib" >> "$OUT/ab.log"; exit $rc; fi
    python - "$OUT/tmp.json" "$cfg" "$lib" >> "$OUT/ab.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sf = d.get("single_frame", {})
print(f"{sys.argv[2]:7s} {sys.argv[3]:28s} inflight {d['value']:9.0f} Mrays/s ({d['trace_kind']}, {d['ms_per_step']*1e3:6.1f} us/frame)"
      f"  single {sf.get('mrays_s', 0):9.0f} Mrays/s (kernel {sf.get('trace_kernel_ms', 0)*1e3:6.1f} us)  check {d['frame_check']}")
PY
  done
done
done
