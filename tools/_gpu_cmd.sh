set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v55; mkdir -p $OUT
for r in 1 2 3 4 5 6; do
 for v in "" libbeam_hip_rows.so; do
  lib=""; [ -n "$v" ] && lib=$(pwd)/raytracercuda_amd/$v
  line=$(BEAM_HIP_LIB=$lib timeout -k 10 180 python bench.py --config c3 --only inflight --no-extra --no-cpu-baseline --steps 20 --warmup 5 2>/dev/null | grep '^{') || exit 3
  python -c "import json,sys; r=json.loads(sys.argv[1]); print('${v:-stripes}', round(r['value']), round(r['ms_per_step']*1e3,1))" "$line"
 done
done
