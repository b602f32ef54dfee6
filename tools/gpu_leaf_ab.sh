set -u
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in filled c4; do for leaf in 4 8 16; do for v in "" "--param trace_auto_packet=0"; do
  line=$(timeout -k 10 180 python bench.py --config $cfg --only single --no-extra --no-cpu-baseline --pmc off --steps 40 --warmup 5 --leaf-size $leaf $v 2>/dev/null | grep '^{') || exit 3
  python -c "import json,sys; r=json.loads(sys.argv[1]); print('$cfg leaf $leaf', r['trace_kind'], round(r['value']), round(r['trace_kernel_ms']*1e3,1), r['build_ms'])" "$line"
done; done; done
