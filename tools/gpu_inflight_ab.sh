#!/usr/bin/env bash
# In-flight trace A/B by tuning parameter: bench.py --only inflight per config, default vs each
# --param NAME=VALUE (or a library under raytracercuda_amd/), interleaved twice.
#   bash tools/gpu_inflight_ab.sh "c3 c4" "trace_auto_compact=0 libbeam_hip_x.so ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  for cfg in $1; do
    for p in default $2; do
      extra=""; lib=""
      case "$p" in default) ;; *.so) lib="$(pwd)/raytracercuda_amd/$p" ;; *) extra="--param $p" ;; esac
      line=$(BEAM_HIP_LIB=$lib timeout -k 10 180 python bench.py --config $cfg --only inflight --no-extra --no-cpu-baseline --steps 50 --warmup 10 $extra 2>/dev/null | grep '^{') || exit 3
      python -c "import json,sys; r=json.loads(sys.argv[1]); print(f\"$cfg {'$p':28s} {r['value']:.0f} Mrays/s  {r['ms_per_step']*1e3:.1f} us/frame  kind {r.get('trace_kind')}\")" "$line"
    done
  done
done
