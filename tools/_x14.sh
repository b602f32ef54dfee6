set -u
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 10 12; do for lf in 2 4 8; do
echo "v=$v leaf=$lf"; BM_TRACE_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --leaf-size $lf --steps 50 2>&1 | grep -o '"trace_kernel_ms": [0-9.]*\|"build_ms": [0-9.]*\|"node_records": [0-9.]*\|"tri_tests": [0-9.]*' | tr '\n' ' ' ; echo
done; done
